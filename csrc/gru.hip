// Fused GRU time-step kernels for gfx950: each launch is one recurrent GEMM on the bf16 MFMA with the gate math
// of that GEMM's consumers in its epilogue (no gate pre-activation ever touches HBM).
//
// Reference: S/nn/GRU.scala (preTopology order r, z, n; n = tanh(x_n + U_n (r * h)); h' = (1 - z) n + z h),
// fused whole-sequence MKL-DNN RNN (S/nn/mkldnn/RNN.scala:215-218 VanillaGru), SURVEY K10.
//
// A GRU step has two dependent GEMMs (the candidate needs r * h over ALL units), so a step is two launches;
// the backward sweep likewise (d(r*h) = dn_pre . U_n needs every dn_pre; dh_{t-1} needs d(r, z)_pre . U_rz):
//   forward  k1  D = h16_{t-1} . U_rz^T (N = 2H)  -> r, z; writes r*h (bf16, the next GEMM's operand)
//            k2  D = (r*h)16 . U_n^T   (N = H)   -> n, h_t (fp32 out + bf16 state)
//   backward S2  D = drz16_{t+1} . U_rz (N = H)  -> dh_t, then dn_pre_t / dz_pre_t (dx, bf16 GEMM operands)
//            S1  D = dn16_t . U_n       (N = H)  -> d(r*h): dr_pre_t, and the r-path of dh_{t-1}
// Tile = 16 batch rows x 16 output columns per workgroup, K split over up to 16 waves (each wave one or two
// groups of 8 MFMA k-steps, see csrc/lstm.hip for why), partials reduced in LDS, then 256 threads run the
// epilogue coalesced along the output columns.
#include "common.h"
#include "kernels.h"

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  const float e = __expf(-2.f * fabsf(x));
  const float t = (1.f - e) / (1.f + e);
  return x < 0.f ? -t : t;
}
__device__ __forceinline__ v8s ld8(const bf16_t* p) { return *(const v8s*)p; }

__device__ __forceinline__ v4f mfma_rows(const bf16_t* __restrict__ pa, const bf16_t* __restrict__ pb, int K, v4f acc) {
  constexpr int CH = 8;
  const int steps = K / 32, full = steps / CH * CH;
  for (int s = 0; s < full; s += CH) {
    v8s a[CH], b[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) { a[i] = ld8(pa + (s + i) * 32); b[i] = ld8(pb + (s + i) * 32); }
#pragma unroll
    for (int i = 0; i < CH; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[i], acc, 0, 0, 0);
  }
  for (int s = full; s < steps; ++s)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld8(pa + s * 32), ld8(pb + s * 32), acc, 0, 0, 0);
  return acc;
}

enum GruMode { FWD_RZ = 0, FWD_N = 1, BWD_H = 2, BWD_R = 3, BWD_H0 = 4 };

// D[b][n] = sum_k A[b][k] * W[n][k] for the workgroup's 16 x 16 tile, summed over the KS K-chunks in LDS.
// Returns with red[][] filled; every lane of the workgroup must call it (barrier inside).
__device__ __forceinline__ void tile_gemm(const bf16_t* __restrict__ A, long lda, const bf16_t* __restrict__ W,
                                          int K, int B, int b0, int n0, int KS, float (*red)[16][17]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kh = lane >> 4;
  if (wave < KS) {
    v4f acc = {0.f, 0.f, 0.f, 0.f};
    if (A != nullptr) {
      const int kl = K / KS;
      const int ba = b0 + r;
      // batch rows past B read row 0: an A row only feeds its own output row, which is never stored
      acc = mfma_rows(A + (long)(ba < B ? ba : 0) * lda + (long)wave * kl + kh * 8,
                      W + (long)(n0 + r) * K + (long)wave * kl + kh * 8, kl, acc);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) red[wave][kh * 4 + i][r] = acc[i];   // D[row = batch][col = output]
  }
  __syncthreads();
}

struct GruArgs {
  const bf16_t* A; long lda;          // GEMM activation operand [B][K] (nullptr: D = 0)
  const bf16_t* W;                     // [N][K] bf16
  int B, H, K, N, KS, mode;
  const float* xg; long ldx;           // preTopology output of this step (fwd): [B] rows, cols r|z|n
  const float* hprev; long ldhp;       // h_{t-1} fp32 [B][H] (nullptr: zeros)
  float* r; float* z; float* n;        // saved gates [B][H] of this step
  bf16_t* rh16;                        // fwd: r*h_{t-1} (bf16) [B][H]
  float* hout; long ldho;              // fwd: h_t fp32
  bf16_t* h16out;                      // fwd: h_t bf16 [B][H]
  const float* dout; long ldd;         // bwd: dL/dout_t (nullptr: none)
  float* dhp;                          // bwd: running partial of dh (z-path + r-path), [B][H]
  float* dx; long lddx;                // bwd: dL/d preTopology output of this step (cols r|z|n)
  bf16_t* dn16;                        // bwd: dn_pre (bf16) [B][H]
  bf16_t* drz16;                       // bwd: (dr_pre | dz_pre) (bf16) [B][2H]
  float* dh0;                          // BWD_H0 output [B][H]
};

__global__ void __launch_bounds__(1024) gru_step_kernel(GruArgs a) {
  __shared__ float red[16][16][17];
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  tile_gemm(a.A, a.lda, a.W, a.K, a.B, b0, n0, a.KS, red);
  if (threadIdx.x >= 256) return;
  const int m = threadIdx.x >> 4, c = threadIdx.x & 15;
  const int b = b0 + m, j = n0 + c;
  if (b >= a.B || j >= a.N) return;
  float v = 0.f;
  for (int k = 0; k < a.KS; ++k) v += red[k][m][c];
  const int H = a.H;
  switch (a.mode) {
    case FWD_RZ: {
      const float s = sigm(v + a.xg[(long)b * a.ldx + j]);
      if (j < H) {
        const float hp = a.hprev ? a.hprev[(long)b * a.ldhp + j] : 0.f;
        a.r[(long)b * H + j] = s;
        a.rh16[(long)b * H + j] = f2bf(s * hp);
      } else {
        a.z[(long)b * H + (j - H)] = s;
      }
      break;
    }
    case FWD_N: {
      const float nv = tanh_f(v + a.xg[(long)b * a.ldx + 2 * H + j]);
      const float zv = a.z[(long)b * H + j];
      const float hp = a.hprev ? a.hprev[(long)b * a.ldhp + j] : 0.f;
      const float h = (1.f - zv) * nv + zv * hp;
      a.n[(long)b * H + j] = nv;
      a.hout[(long)b * a.ldho + j] = h;
      a.h16out[(long)b * H + j] = f2bf(h);
      break;
    }
    case BWD_H: {
      float dh = v + a.dhp[(long)b * H + j];
      if (a.dout) dh += a.dout[(long)b * a.ldd + j];
      const float zv = a.z[(long)b * H + j], nv = a.n[(long)b * H + j];
      const float hp = a.hprev ? a.hprev[(long)b * a.ldhp + j] : 0.f;
      const float dn = dh * (1.f - zv) * (1.f - nv * nv);
      const float dz = dh * (hp - nv) * zv * (1.f - zv);
      float* dx = a.dx + (long)b * a.lddx;
      dx[H + j] = dz;
      dx[2 * H + j] = dn;
      a.dn16[(long)b * H + j] = f2bf(dn);
      a.drz16[(long)b * 2 * H + H + j] = f2bf(dz);
      a.dhp[(long)b * H + j] = dh * zv;           // z-path of dh_{t-1}; S1 adds the r-path
      break;
    }
    case BWD_R: {
      const float rv = a.r[(long)b * H + j];
      const float hp = a.hprev ? a.hprev[(long)b * a.ldhp + j] : 0.f;
      const float dr = v * hp * rv * (1.f - rv);
      a.dx[(long)b * a.lddx + j] = dr;
      a.drz16[(long)b * 2 * H + j] = f2bf(dr);
      a.dhp[(long)b * H + j] += v * rv;
      break;
    }
    default: {   // BWD_H0: dh_{-1} = r/z-paths accumulated in dhp + d(r,z)_pre_0 . U_rz
      a.dh0[(long)b * H + j] = v + a.dhp[(long)b * H + j];
      break;
    }
  }
}

int ksplit(int K, int cap) {
  int ks = K / 256;
  if (ks < 1) ks = 1;
  if (ks > cap) ks = cap;
  while (ks > 1 && (K % (ks * 32)) != 0) --ks;
  return ks;
}

}  // namespace

int bigdl_gru_step(const GruStepArgs* s, hipStream_t st) {
  GruArgs a;
  a.A = s->A; a.lda = s->lda; a.W = s->W; a.B = s->B; a.H = s->H; a.K = s->K; a.N = s->N; a.mode = s->mode;
  a.xg = s->xg; a.ldx = s->ldx; a.hprev = s->hprev; a.ldhp = s->ldhp; a.r = s->r; a.z = s->z; a.n = s->n;
  a.rh16 = s->rh16; a.hout = s->hout; a.ldho = s->ldho; a.h16out = s->h16out; a.dout = s->dout; a.ldd = s->ldd;
  a.dhp = s->dhp; a.dx = s->dx; a.lddx = s->lddx; a.dn16 = s->dn16; a.drz16 = s->drz16; a.dh0 = s->dh0;
  if (a.H % 32 != 0 || a.K % 32 != 0 || a.N % 16 != 0 || a.B <= 0) return -1;
  a.KS = ksplit(a.K, 16);
  const int waves = a.KS < 4 ? 4 : a.KS;            // >= 4 waves so all 256 epilogue threads exist
  dim3 grid(a.N / 16, (a.B + 15) / 16);
  gru_step_kernel<<<grid, 64 * waves, 0, st>>>(a);
  HIP_LAUNCH_CHECK();
  return 0;
}
