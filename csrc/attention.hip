// Fused scaled-dot-product attention for gfx950: O = softmax(Q K^T + bias) V with the scores never leaving the
// chip (flash-attention style online softmax), and the matching fused backward.
//
// Reference: S/nn/Attention.scala:90-103 (MM(transB) -> CAddTable(bias) -> SoftMax -> Dropout -> MM), the core of
// S/nn/Transformer.scala's self / encoder-decoder attention (SURVEY K-row "attention").
//
// Layout: Q [BH][Lq][D], K / V [BH][Lk][D] bf16 (q pre-scaled by D^-1/2 as in SplitHeads(mul=true)), D = 32, 64,
// 96 or 128; bias fp32 broadcast through element strides (sb, sh, sq, sk) over (batch, head, query, key), or causal.
// Outputs O fp32 [BH][Lq][D] and the row log-sum-exp (fp32 [BH][Lq]) kept for the backward.
//
// Forward: workgroup = 64 query rows (4 waves x 16) of one (batch, head); K / V stream through LDS in 64-key
// tiles. Per tile a wave computes S = Q K^T on v_mfma_f32_16x16x32_bf16 (Q fragments stay in VGPRs), runs the
// online softmax on the accumulators (row max / sum over the 16 lanes of a row group by xor shuffles), parks P
// (bf16) in its own LDS slice to turn the accumulator layout into the A-operand layout, and accumulates P V
// against V^T (transposed when the tile is staged) — all in fp32 accumulators.
// Backward (one workgroup per 64-key block, looping over query blocks): P is recomputed from the saved
// log-sum-exp; dV += P^T dO, dP = dO V^T, dS = P (dP - rowsum(dO o O)), dK += dS^T Q accumulate in VGPRs; dQ +=
// dS K is accumulated across key blocks with fp32 atomics.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int AT_BQ = 64;      // query rows per workgroup (forward)
constexpr int AT_BK = 64;      // keys per tile
constexpr float NEG_BIG = -1e30f;

__device__ __forceinline__ v8s lds8(const bf16_t* p) { return *reinterpret_cast<const v8s*>(p); }
__device__ __forceinline__ v4f mfma(v8s a, v8s b, v4f c) { return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0); }

struct AttnArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v;
  const float* bias; long sb, sh, sq, sk;
  float* o; float* lse;
  const float* dout;                  // backward: dO fp32 [BH][Lq][D]
  const float* delta;                 // backward: rowsum(dO o O) [BH][Lq]
  float* dq; float* dk; float* dv;    // backward outputs fp32
  int H, Lq, Lk, causal;
  // attention dropout (reference Attention.scala:59 attentionDropout on the softmax output): keep iff
  // hash(seed, row, key) >= drop_thr, kept probabilities scaled by drop_scale = 1 / (1 - p); drop_thr == 0: none
  unsigned drop_thr; float drop_scale; unsigned seed_lo, seed_hi;
};

// Counter-based dropout mask, identical in the forward and the backward whatever the tiling: a lowbias32-style
// integer hash (2 multiply-xorshift rounds) of the row hash and the key index. The row part is hashed once per
// query row; a mask element costs one hash (a handful of VALU ops) instead of a Philox block per element.
__device__ __forceinline__ unsigned mix32(unsigned x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ unsigned drop_row(const AttnArgs& a, int bh, int qi) {
  return mix32((unsigned)(bh * a.Lq + qi) ^ a.seed_lo);
}
__device__ __forceinline__ float drop_mul(const AttnArgs& a, unsigned row, int kj) {
  return mix32(row + (unsigned)kj * 0x9E3779B9u + a.seed_hi) >= a.drop_thr ? a.drop_scale : 0.f;
}

__device__ __forceinline__ float bias_at(const AttnArgs& a, int bh, int qi, int kj) {
  if (!a.bias) return 0.f;
  const int b = bh / a.H, h = bh % a.H;
  return a.bias[b * a.sb + h * a.sh + (long)qi * a.sq + (long)kj * a.sk];
}

// Stage a [64][D] bf16 tile (rows r0.., zero past `rows`) into LDS row-major, and optionally transposed [D][64].
template <int D>
__device__ __forceinline__ void stage(const bf16_t* __restrict__ src, int r0, int rows, bf16_t* rowmajor,
                                      bf16_t* transposed) {
  constexpr int GR = D / 8;                       // 16-byte granules per row
  for (int gi = threadIdx.x; gi < AT_BK * GR; gi += 256) {
    const int r = gi / GR, g = gi % GR;
    v4u val = {0u, 0u, 0u, 0u};
    if (r0 + r < rows) val = *reinterpret_cast<const v4u*>(src + (long)(r0 + r) * D + g * 8);
    if (rowmajor) *reinterpret_cast<v4u*>(rowmajor + r * D + g * 8) = val;
    if (transposed) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        transposed[(g * 8 + 2 * e) * AT_BK + r] = (bf16_t)(val[e] & 0xffff);
        transposed[(g * 8 + 2 * e + 1) * AT_BK + r] = (bf16_t)(val[e] >> 16);
      }
    }
  }
}

template <int D>
__global__ void __launch_bounds__(256) attn_fwd_kernel(AttnArgs a) {
  constexpr int KS = D / 32;                      // k-steps over the head dimension
  constexpr int NC = D / 16;                      // 16-column blocks of O
  __shared__ __attribute__((aligned(16))) bf16_t sK[AT_BK * D];
  __shared__ __attribute__((aligned(16))) bf16_t sVt[D * AT_BK];
  __shared__ __attribute__((aligned(16))) bf16_t sP[4][16 * AT_BK];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bh = blockIdx.y;
  const int q0 = blockIdx.x * AT_BQ + wave * 16;   // this wave's first query row
  const bf16_t* Q = a.q + (long)bh * a.Lq * D;
  const bf16_t* K = a.k + (long)bh * a.Lk * D;
  const bf16_t* V = a.v + (long)bh * a.Lk * D;
  // Q fragments (A operand): row q0 + (lane & 15), k = 32 s + 8 (lane >> 4)
  v8s qf[KS];
  {
    const int qr = q0 + (lane & 15);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      v8s z = {0, 0, 0, 0, 0, 0, 0, 0};
      qf[s] = qr < a.Lq ? *reinterpret_cast<const v8s*>(Q + (long)qr * D + 32 * s + 8 * (lane >> 4)) : z;
    }
  }
  v4f oacc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) oacc[c] = v4f{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { m[i] = NEG_BIG; l[i] = 0.f; }
  const int grp = lane >> 4, col = lane & 15;
  int kend = a.Lk;
  if (a.causal) {
    const int qlast = blockIdx.x * AT_BQ + AT_BQ - 1;
    kend = qlast + 1 < a.Lk ? qlast + 1 : a.Lk;
  }
  for (int k0 = 0; k0 < kend; k0 += AT_BK) {
    __syncthreads();                              // previous tile's sK / sVt / sP reads are done
    stage<D>(K, k0, a.Lk, sK, nullptr);
    stage<D>(V, k0, a.Lk, nullptr, sVt);
    __syncthreads();
    // S = Q K^T for 4 key sub-blocks of 16
    v4f s4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s)
        acc = mfma(qf[s], lds8(sK + (16 * j + col) * D + 32 * s + 8 * grp), acc);
      s4[j] = acc;                                // s4[j][i] = S[q0 + 4 grp + i][k0 + 16 j + col]
    }
    float mx[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int qi = q0 + 4 * grp + i;
      float v = NEG_BIG;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kj = k0 + 16 * j + col;
        float x = s4[j][i];
        if (kj >= a.Lk || (a.causal && kj > qi)) x = NEG_BIG;
        else if (qi < a.Lq) x += bias_at(a, bh, qi, kj);
        s4[j][i] = x;
        v = fmaxf(v, x);
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
      mx[i] = v;
    }
    float scale[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float mn = fmaxf(m[i], mx[i]);
      scale[i] = __expf(m[i] - mn);
      float rs = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float p = s4[j][i] <= NEG_BIG ? 0.f : __expf(s4[j][i] - mn);
        s4[j][i] = p;
        rs += p;
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) rs += __shfl_xor(rs, o, 64);
      l[i] = l[i] * scale[i] + rs;
      m[i] = mn;
    }
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) oacc[c][i] *= scale[i];
    // P (bf16) -> this wave's LDS slice [16 q][64 keys], read back as A fragments; attention dropout acts on the
    // normalised probabilities, so it scales what enters P V while the normaliser l keeps the un-dropped sums
    bf16_t* P = sP[wave];
    if (a.drop_thr) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const unsigned row = drop_row(a, bh, q0 + 4 * grp + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) s4[j][i] *= drop_mul(a, row, k0 + 16 * j + col);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) P[(4 * grp + i) * AT_BK + 16 * j + col] = f2bf(s4[j][i]);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < AT_BK / 32; ++t) {
      const v8s pf = lds8(P + col * AT_BK + 32 * t + 8 * grp);
#pragma unroll
      for (int c = 0; c < NC; ++c) oacc[c] = mfma(pf, lds8(sVt + (16 * c + col) * AT_BK + 32 * t + 8 * grp), oacc[c]);
    }
  }
  // O = acc / l, lse = m + log l
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int qi = q0 + 4 * grp + i;
    if (qi >= a.Lq) continue;
    const float inv = l[i] > 0.f ? 1.f / l[i] : 0.f;
    float* orow = a.o + ((long)bh * a.Lq + qi) * D;
#pragma unroll
    for (int c = 0; c < NC; ++c) orow[16 * c + col] = oacc[c][i] * inv;
    if (col == 0) a.lse[(long)bh * a.Lq + qi] = l[i] > 0.f ? m[i] + __logf(l[i]) : NEG_BIG;
  }
}

// ----------------------------------------------------------------------------------------------- backward
// Workgroup = one 64-key block of one (batch, head); wave w owns keys k0 + 16 w .. +15 for dK / dV. For every
// 64-row query block: S^T = K Q^T (per wave 16 keys x 64 q), P^T = exp(S^T + bias - lse), dP^T = V dO^T,
// dS^T = P^T (dP^T - delta); dV += P^T dO, dK += dS^T Q (A operands through the wave's LDS slice, B operands from
// transposed dO / Q tiles), dQ += dS K via fp32 atomics (dS gathered in LDS [q][key], K^T tile as B operand).
template <int D>
__global__ void __launch_bounds__(256) attn_bwd_kernel(AttnArgs a) {
  constexpr int KS = D / 32, NC = D / 16;
  __shared__ __attribute__((aligned(16))) bf16_t sQ[AT_BK * D];      // Q block, row-major [q][d]
  __shared__ __attribute__((aligned(16))) bf16_t sQt[D * AT_BK];     // Q^T [d][q]
  __shared__ __attribute__((aligned(16))) bf16_t sdO[AT_BK * D];     // dO block row-major
  __shared__ __attribute__((aligned(16))) bf16_t sdOt[D * AT_BK];    // dO^T
  __shared__ __attribute__((aligned(16))) bf16_t sKt[D * AT_BK];     // K^T of this key block [d][key]
  __shared__ __attribute__((aligned(16))) bf16_t sT[4][16 * AT_BK];  // per-wave scratch (P^T / dS^T as A operand)
  __shared__ __attribute__((aligned(16))) bf16_t sdS[AT_BK * AT_BK]; // dS [q][key] for the dQ GEMM
  __shared__ float sL[AT_BK], sDel[AT_BK];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int grp = lane >> 4, col = lane & 15;
  const int bh = blockIdx.y, k0 = blockIdx.x * AT_BK, kw = k0 + wave * 16;
  const bf16_t* Q = a.q + (long)bh * a.Lq * D;
  const bf16_t* K = a.k + (long)bh * a.Lk * D;
  const bf16_t* V = a.v + (long)bh * a.Lk * D;
  const float* dO = a.dout + (long)bh * a.Lq * D;
  // this wave's K / V rows as A fragments: row kw + col, k = 32 s + 8 grp
  v8s kf[KS], vf[KS];
  {
    const int kr = kw + col;
    v8s z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      kf[s] = kr < a.Lk ? *reinterpret_cast<const v8s*>(K + (long)kr * D + 32 * s + 8 * grp) : z;
      vf[s] = kr < a.Lk ? *reinterpret_cast<const v8s*>(V + (long)kr * D + 32 * s + 8 * grp) : z;
    }
  }
  stage<D>(K, k0, a.Lk, nullptr, sKt);
  v4f dk[NC], dv[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) { dk[c] = v4f{0.f, 0.f, 0.f, 0.f}; dv[c] = v4f{0.f, 0.f, 0.f, 0.f}; }
  const int qstart = a.causal ? (k0 / AT_BK) * AT_BK : 0;
  for (int q0 = qstart; q0 < a.Lq; q0 += AT_BK) {
    __syncthreads();
    stage<D>(Q, q0, a.Lq, sQ, sQt);
    // dO block (fp32 in HBM) -> bf16 row-major and transposed
    for (int gi = threadIdx.x; gi < AT_BK * (D / 8); gi += 256) {
      const int r = gi / (D / 8), g = gi % (D / 8);
      float f[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (q0 + r < a.Lq) {
        const v4f lo = *reinterpret_cast<const v4f*>(dO + (long)(q0 + r) * D + g * 8);
        const v4f hi = *reinterpret_cast<const v4f*>(dO + (long)(q0 + r) * D + g * 8 + 4);
        f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3]; f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
      }
      v4u pk;
#pragma unroll
      for (int e = 0; e < 4; ++e) pk[e] = pack2bf(f[2 * e], f[2 * e + 1]);
      *reinterpret_cast<v4u*>(sdO + r * D + g * 8) = pk;
#pragma unroll
      for (int e = 0; e < 8; ++e) sdOt[(g * 8 + e) * AT_BK + r] = f2bf(f[e]);
    }
    if (threadIdx.x < AT_BK) {
      const int qi = q0 + threadIdx.x;
      sL[threadIdx.x] = qi < a.Lq ? a.lse[(long)bh * a.Lq + qi] : 0.f;
      sDel[threadIdx.x] = qi < a.Lq ? a.delta[(long)bh * a.Lq + qi] : 0.f;
    }
    __syncthreads();
    // S^T and dP^T for this wave's 16 keys x 64 queries (4 sub-blocks of 16 queries)
    v4f st[4], dpt[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v4f s_acc = {0.f, 0.f, 0.f, 0.f}, p_acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        s_acc = mfma(kf[s], lds8(sQ + (16 * j + col) * D + 32 * s + 8 * grp), s_acc);
        p_acc = mfma(vf[s], lds8(sdO + (16 * j + col) * D + 32 * s + 8 * grp), p_acc);
      }
      st[j] = s_acc;                // st[j][i] = S[q0 + 16 j + col][kw + 4 grp + i]
      dpt[j] = p_acc;               // dP[q][key] likewise
    }
    bf16_t* T = sT[wave];
    // P^T (recomputed) -> scratch as [key][q], the A operand of dV += P_dropped^T dO; dm keeps the dropout factor
    // (0 or 1 / (1 - p)) of every element for dP = dm * (dO V^T)
    float dm[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int qi = q0 + 16 * j + col;
      const unsigned row = a.drop_thr ? drop_row(a, bh, qi) : 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kj = kw + 4 * grp + i;
        float p = 0.f;
        if (qi < a.Lq && kj < a.Lk && !(a.causal && kj > qi))
          p = __expf(st[j][i] + bias_at(a, bh, qi, kj) - sL[16 * j + col]);
        st[j][i] = p;
        dm[j][i] = a.drop_thr ? drop_mul(a, row, kj) : 1.f;
        T[(4 * grp + i) * AT_BK + 16 * j + col] = f2bf(p * dm[j][i]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < AT_BK / 32; ++t) {
      const v8s pf = lds8(T + col * AT_BK + 32 * t + 8 * grp);
#pragma unroll
      for (int c = 0; c < NC; ++c) dv[c] = mfma(pf, lds8(sdOt + (16 * c + col) * AT_BK + 32 * t + 8 * grp), dv[c]);
    }
    __syncthreads();
    // dS^T = P^T (dP^T - delta) -> scratch [key][q] (dK A operand) and sdS [q][key] (dQ A operand)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float ds = st[j][i] * (dpt[j][i] * dm[j][i] - sDel[16 * j + col]);
        const bf16_t d16 = f2bf(ds);
        T[(4 * grp + i) * AT_BK + 16 * j + col] = d16;
        sdS[(16 * j + col) * AT_BK + wave * 16 + 4 * grp + i] = d16;
      }
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < AT_BK / 32; ++t) {
      const v8s df = lds8(T + col * AT_BK + 32 * t + 8 * grp);
#pragma unroll
      for (int c = 0; c < NC; ++c) dk[c] = mfma(df, lds8(sQt + (16 * c + col) * AT_BK + 32 * t + 8 * grp), dk[c]);
    }
    // dQ[q0 + 16 w + ..][:] += dS[q rows of this wave][64 keys] . K[64 keys][:]
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < AT_BK / 32; ++t)
        acc = mfma(lds8(sdS + (wave * 16 + col) * AT_BK + 32 * t + 8 * grp),
                   lds8(sKt + (16 * c + col) * AT_BK + 32 * t + 8 * grp), acc);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qi = q0 + wave * 16 + 4 * grp + i;
        if (qi < a.Lq) atomicAdd(a.dq + ((long)bh * a.Lq + qi) * D + 16 * c + col, acc[i]);
      }
    }
  }
  // dK, dV rows kw + 4 grp + i
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kj = kw + 4 * grp + i;
    if (kj >= a.Lk) continue;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      a.dk[((long)bh * a.Lk + kj) * D + 16 * c + col] = dk[c][i];
      a.dv[((long)bh * a.Lk + kj) * D + 16 * c + col] = dv[c][i];
    }
  }
}

__global__ void attn_delta_kernel(const float* __restrict__ dout, const float* __restrict__ o, float* __restrict__ delta,
                                  long rows, int D) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  float s = 0.f;
  for (int c = lane; c < D; c += 64) s += dout[r * D + c] * o[r * D + c];
  s = wave_sum(s);
  if (lane == 0) delta[r] = s;
}

}  // namespace

static AttnArgs to_args(const AttnCall* c) {
  AttnArgs a;
  a.q = c->q; a.k = c->k; a.v = c->v; a.bias = c->bias; a.sb = c->sb; a.sh = c->sh; a.sq = c->sq; a.sk = c->sk;
  a.o = c->o; a.lse = c->lse; a.dout = c->dout; a.delta = c->delta; a.dq = c->dq; a.dk = c->dk; a.dv = c->dv;
  a.H = c->H; a.Lq = c->Lq; a.Lk = c->Lk; a.causal = c->causal;
  const double p = c->drop_p;
  a.drop_thr = p > 0.0 ? (unsigned)fmin(4294967295.0, p * 4294967296.0) : 0u;
  if (p > 0.0 && a.drop_thr == 0u) a.drop_thr = 1u;
  a.drop_scale = p > 0.0 && p < 1.0 ? (float)(1.0 / (1.0 - p)) : (p >= 1.0 ? 0.f : 1.f);
  a.seed_lo = (unsigned)c->seed; a.seed_hi = (unsigned)(c->seed >> 32);
  return a;
}

static bool attn_dim_ok(int D) { return D == 32 || D == 64 || D == 96 || D == 128; }

int bigdl_attn_fwd(const AttnCall* c, hipStream_t st) {
  if (!attn_dim_ok(c->D) || c->BH <= 0 || c->Lq <= 0 || c->Lk <= 0) return -1;
  const AttnArgs a = to_args(c);
  dim3 grid((c->Lq + AT_BQ - 1) / AT_BQ, c->BH);
  switch (c->D) {
    case 32: attn_fwd_kernel<32><<<grid, 256, 0, st>>>(a); break;
    case 64: attn_fwd_kernel<64><<<grid, 256, 0, st>>>(a); break;
    case 96: attn_fwd_kernel<96><<<grid, 256, 0, st>>>(a); break;
    default: attn_fwd_kernel<128><<<grid, 256, 0, st>>>(a); break;
  }
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_attn_bwd(const AttnCall* c, float* delta_ws, hipStream_t st) {
  if (!attn_dim_ok(c->D) || c->BH <= 0 || c->Lq <= 0 || c->Lk <= 0) return -1;
  const long rows = (long)c->BH * c->Lq;
  attn_delta_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(c->dout, c->o, delta_ws, rows, c->D);
  AttnArgs a = to_args(c);
  a.delta = delta_ws;
  dim3 grid((c->Lk + AT_BK - 1) / AT_BK, c->BH);
  switch (c->D) {
    case 32: attn_bwd_kernel<32><<<grid, 256, 0, st>>>(a); break;
    case 64: attn_bwd_kernel<64><<<grid, 256, 0, st>>>(a); break;
    case 96: attn_bwd_kernel<96><<<grid, 256, 0, st>>>(a); break;
    default: attn_bwd_kernel<128><<<grid, 256, 0, st>>>(a); break;
  }
  HIP_LAUNCH_CHECK();
  return 0;
}
