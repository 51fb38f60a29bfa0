// Vectorized elementwise / layout / pooling / loss / optimizer kernels for gfx950.
//
// Reference counterparts: ReLU/Threshold (S/nn/ReLU.scala:42, S/nn/Threshold.scala:38), CAddTable
// (S/nn/CAddTable.scala:82), NNPrimitive.maxPoolingForwardFloat/BackwardFloat (S/nn/NNPrimitive.scala:654,
// :714, NHWC :841, :936), SpatialAveragePooling (S/nn/SpatialAveragePooling.scala:323), LogSoftMax +
// ClassNLLCriterion (S/nn/LogSoftMax.scala:49, S/nn/ClassNLLCriterion.scala:69 = CrossEntropyCriterion
// S/nn/CrossEntropyCriterion.scala:31), SGD / Adam (S/optim/SGD.scala:54-120, S/optim/Adam.scala:36),
// L2-norm clipping (S/parameters/ParameterOperations.scala:71-133), LSTM cell (S/nn/LSTM.scala:158-185).
// Every memory-bound kernel moves 16 bytes per lane (cdna_hip_programming.md Guideline 13).
#include "common.h"
#include "kernels.h"
#include <algorithm>

namespace {

inline int grid_cap(long work, int cap = 8192) {
  long g = (work + 255) / 256;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

#define GRID_STRIDE(i, n) for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)

__global__ void relu_fwd_kernel(const v4u* __restrict__ x, v4u* __restrict__ y, long n8) {
  GRID_STRIDE(i, n8) {
    v4u v = x[i], o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2bf(fmaxf(lo_bf(v[e]), 0.f), fmaxf(hi_bf(v[e]), 0.f));
    y[i] = o;
  }
}
__global__ void relu_bwd_kernel(const v4u* __restrict__ dy, const v4u* __restrict__ y, v4u* __restrict__ dx, long n8) {
  GRID_STRIDE(i, n8) {
    const v4u d = dy[i], v = y[i];
    v4u o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const unsigned lo = lo_bf(v[e]) > 0.f ? (d[e] & 0xffffu) : 0u;
      const unsigned hi = hi_bf(v[e]) > 0.f ? (d[e] & 0xffff0000u) : 0u;
      o[e] = lo | hi;
    }
    dx[i] = o;
  }
}
__global__ void add_kernel(const v4u* __restrict__ a, const v4u* __restrict__ b, v4u* __restrict__ y, long n8) {
  GRID_STRIDE(i, n8) {
    const v4u u = a[i], v = b[i];
    v4u o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2bf(lo_bf(u[e]) + lo_bf(v[e]), hi_bf(u[e]) + hi_bf(v[e]));
    y[i] = o;
  }
}
// tail-safe scalar versions for n % 8 != 0
__global__ void relu_fwd_tail(const bf16_t* x, bf16_t* y, long s, long n) {
  GRID_STRIDE(i, n - s) y[s + i] = f2bf(fmaxf(bf2f(x[s + i]), 0.f));
}
__global__ void relu_bwd_tail(const bf16_t* dy, const bf16_t* y, bf16_t* dx, long s, long n) {
  GRID_STRIDE(i, n - s) dx[s + i] = bf2f(y[s + i]) > 0.f ? dy[s + i] : (bf16_t)0;
}
__global__ void add_tail(const bf16_t* a, const bf16_t* b, bf16_t* y, long s, long n) {
  GRID_STRIDE(i, n - s) y[s + i] = f2bf(bf2f(a[s + i]) + bf2f(b[s + i]));
}

// NCHW fp32 (the user-facing BigDL layout) -> NHWC bf16 with channel padding to Cp (zeros). One thread per
// (pixel, 8-channel group): the C plane reads are coalesced along the pixel axis, the 8 bf16 channels leave
// as one 16-byte store, and blockIdx.y = (image, group) keeps 64-bit division out of the loop.
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                           int N, int C, int H, int W, int Cp) {
  const int HW = H * W, G = Cp >> 3;
  const int hw = blockIdx.x * 256 + threadIdx.x;
  if (hw >= HW) return;
  for (int ng = blockIdx.y; ng < N * G; ng += gridDim.y) {
    const int n = ng / G, g = ng - n * G;
    const float* src = x + ((long)n * C + g * 8) * HW + hw;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (g * 8 + e < C) ? src[(long)e * HW] : 0.f;
    *reinterpret_cast<v4u*>(y + ((long)n * HW + hw) * Cp + g * 8) =
        v4u{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
  }
}
// Column sums of a [P][K] bf16 matrix into fp32 out[K] (+=): bias gradients of GEMM-shaped layers. A lane owns 8
// consecutive columns (one 16-byte load per row), the 4 waves of a block take interleaved rows of the block's row
// chunk, partials meet in LDS and one atomic per column per block lands in out.
__global__ void __launch_bounds__(256) colsum_bf16_kernel(const bf16_t* __restrict__ x, float* __restrict__ out,
                                                         long P, int K, long rows_per_block, long ld) {
  __shared__ float part[4][64][9];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = (blockIdx.x * 64 + lane) * 8;
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = r0 + rows_per_block < P ? r0 + rows_per_block : P;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < K) {
    for (long r = r0 + wave; r < r1; r += 4) {
      const v4u q = *reinterpret_cast<const v4u*>(x + r * ld + c0);
#pragma unroll
      for (int e = 0; e < 4; ++e) { acc[2 * e] += lo_bf(q[e]); acc[2 * e + 1] += hi_bf(q[e]); }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[wave][lane][e] = acc[e];
  __syncthreads();
  if (wave == 0 && c0 < K) {
#pragma unroll
    for (int e = 0; e < 8; ++e) atomicAdd(out + c0 + e, part[0][lane][e] + part[1][lane][e] + part[2][lane][e] +
                                                        part[3][lane][e]);
  }
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, long n) {
  const long n4 = n >> 2;
  GRID_STRIDE(i, n4) {
    const v4f v = reinterpret_cast<const v4f*>(x)[i];
    reinterpret_cast<v2u*>(y)[i] = v2u{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
  }
  GRID_STRIDE(j, n - n4 * 4) y[n4 * 4 + j] = f2bf(x[n4 * 4 + j]);
}
__global__ void cast_bf16_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, long n) {
  GRID_STRIDE(i, n) y[i] = bf2f(x[i]);
}

// ---------------- pooling (NHWC, 8 channels per lane) ----------------
__global__ void maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, uint8_t* __restrict__ idx,
                                   int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh, int sw, int ph,
                                   int pw) {
  const int G = C >> 3;
  const long total = (long)N * OH * OW * G;
  GRID_STRIDE(i, total) {
    const int g = i % G;
    long p = i / G;
    const int ow = p % OW; p /= OW;
    const int oh = p % OH;
    const int n = p / OH;
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
    for (int r = 0; r < kh; ++r) {
      const int ih = oh * sh - ph + r;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int s = 0; s < kw; ++s) {
        const int iw = ow * sw - pw + s;
        if ((unsigned)iw >= (unsigned)W) continue;
        const v4u v = *reinterpret_cast<const v4u*>(x + (((long)n * H + ih) * W + iw) * C + g * 8);
        const uint8_t widx = (uint8_t)(r * kw + s);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float l = lo_bf(v[e]), h = hi_bf(v[e]);
          if (l > best[2 * e] || (l != l)) { best[2 * e] = l; bi[2 * e] = widx; }
          if (h > best[2 * e + 1] || (h != h)) { best[2 * e + 1] = h; bi[2 * e + 1] = widx; }
        }
      }
    }
    v4u o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2bf(best[2 * e], best[2 * e + 1]);
    reinterpret_cast<v4u*>(y)[i] = o;
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((unsigned)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((unsigned)bi[7] << 24);
    reinterpret_cast<uint2*>(idx)[i] = packed;
  }
}

// gather-form backward: deterministic, no atomics
__global__ void maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ idx, bf16_t* __restrict__ dx,
                                   int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh, int sw, int ph,
                                   int pw) {
  const int G = C >> 3;
  const long total = (long)N * H * W * G;
  GRID_STRIDE(i, total) {
    const int g = i % G;
    long p = i / G;
    const int iw = p % W; p /= W;
    const int ih = p % H;
    const int n = p / H;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const int oh_lo = max(0, (ih + ph - kh + sh) / sh), oh_hi = min(OH - 1, (ih + ph) / sh);
    const int ow_lo = max(0, (iw + pw - kw + sw) / sw), ow_hi = min(OW - 1, (iw + pw) / sw);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int r = ih + ph - oh * sh;
      if (r < 0 || r >= kh) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int s = iw + pw - ow * sw;
        if (s < 0 || s >= kw) continue;
        const long o = (((long)n * OH + oh) * OW + ow) * G + g;
        const uint2 ix = reinterpret_cast<const uint2*>(idx)[o];
        const v4u d = reinterpret_cast<const v4u*>(dy)[o];
        const unsigned widx = r * kw + s;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const unsigned b = ((e < 4 ? ix.x : ix.y) >> ((e & 3) * 8)) & 0xff;
          if (b == widx) acc[e] += (e & 1) ? hi_bf(d[e >> 1]) : lo_bf(d[e >> 1]);
        }
      }
    }
    v4u out;
#pragma unroll
    for (int e = 0; e < 4; ++e) out[e] = pack2bf(acc[2 * e], acc[2 * e + 1]);
    reinterpret_cast<v4u*>(dx)[i] = out;
  }
}

// Fixed K x K / stride-S windows (the 3x3 / 2 stem pools of ResNet and Inception): 32-bit index math (the host
// checks the element counts) and every window load issued before the first compare, so a lane keeps K*K
// 16-byte loads in flight instead of walking the window one dependent branch at a time.
// PRE: x is the input of a training BatchNorm + ReLU ([scale C | shift C] in `pre`, ConvArgs::pre semantics): every
// window element is relu(x * scale + shift) rounded to bf16 before the compare (bit-equal to pooling bn_apply's output)
template <int K, int S, bool PRE = false>
__global__ __launch_bounds__(256) void maxpool_fwd_fixed_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                                uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                                int OH, int OW, int ph, int pw,
                                                                const float* __restrict__ pre = nullptr) {
  const int G = C >> 3;
  const int total = N * OH * OW * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int g = i % G;
    float psc[8], psh[8];
    if constexpr (PRE) {
      const v4f s0 = *reinterpret_cast<const v4f*>(pre + g * 8), s1 = *reinterpret_cast<const v4f*>(pre + g * 8 + 4);
      const v4f b0 = *reinterpret_cast<const v4f*>(pre + C + g * 8), b1 = *reinterpret_cast<const v4f*>(pre + C + g * 8 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { psc[e] = s0[e]; psc[e + 4] = s1[e]; psh[e] = b0[e]; psh[e + 4] = b1[e]; }
    }
    int p = i / G;
    const int ow = p % OW; p /= OW;
    const int oh = p % OH;
    const int n = p / OH;
    const int h0 = oh * S - ph, w0 = ow * S - pw;
    v4u v[K * K];
    bool ok[K * K];
#pragma unroll
    for (int r = 0; r < K; ++r)
#pragma unroll
      for (int s = 0; s < K; ++s) {
        const int ih = h0 + r, iw = w0 + s;
        const bool in = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        ok[r * K + s] = in;
        const long off = in ? (long)((n * H + ih) * W + iw) * C + g * 8 : (long)g * 8;
        v[r * K + s] = *reinterpret_cast<const v4u*>(x + off);
      }
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -INFINITY; bi[e] = 0; }
#pragma unroll
    for (int t = 0; t < K * K; ++t) {
      if (!ok[t]) continue;
      if constexpr (PRE) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          v[t][e] = pack2bf(fmaxf(lo_bf(v[t][e]) * psc[2 * e] + psh[2 * e], 0.f),
                            fmaxf(hi_bf(v[t][e]) * psc[2 * e + 1] + psh[2 * e + 1], 0.f));
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float l = lo_bf(v[t][e]), h = hi_bf(v[t][e]);
        if (l > best[2 * e] || (l != l)) { best[2 * e] = l; bi[2 * e] = (uint8_t)t; }
        if (h > best[2 * e + 1] || (h != h)) { best[2 * e + 1] = h; bi[2 * e + 1] = (uint8_t)t; }
      }
    }
    v4u o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2bf(best[2 * e], best[2 * e + 1]);
    reinterpret_cast<v4u*>(y)[i] = o;
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((unsigned)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((unsigned)bi[7] << 24);
    reinterpret_cast<uint2*>(idx)[i] = packed;
  }
}

// gather-form backward of the fixed window: an input pixel is covered by at most ceil(K/S) outputs per axis
template <int K, int S>
__global__ __launch_bounds__(256) void maxpool_bwd_fixed_kernel(const bf16_t* __restrict__ dy,
                                                                const uint8_t* __restrict__ idx,
                                                                bf16_t* __restrict__ dx, int N, int H, int W, int C,
                                                                int OH, int OW, int ph, int pw) {
  constexpr int M = (K + S - 1) / S;
  const int G = C >> 3;
  const int total = N * H * W * G;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int g = i % G;
    int p = i / G;
    const int iw = p % W; p /= W;
    const int ih = p % H;
    const int n = p / H;
    const int ohh = (ih + ph) / S, owh = (iw + pw) / S;
    uint2 ix[M * M];
    v4u d[M * M];
    int widx[M * M];
#pragma unroll
    for (int a = 0; a < M; ++a)
#pragma unroll
      for (int b = 0; b < M; ++b) {
        const int oh = ohh - a, ow = owh - b;
        const int r = ih + ph - oh * S, s = iw + pw - ow * S;
        const bool in = oh >= 0 && oh < OH && ow >= 0 && ow < OW && r < K && s < K;
        const int o = in ? ((n * OH + oh) * OW + ow) * G + g : g;
        ix[a * M + b] = reinterpret_cast<const uint2*>(idx)[o];
        d[a * M + b] = reinterpret_cast<const v4u*>(dy)[o];
        widx[a * M + b] = in ? r * K + s : -1;
      }
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
#pragma unroll
    for (int t = 0; t < M * M; ++t) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int b = (int)(((e < 4 ? ix[t].x : ix[t].y) >> ((e & 3) * 8)) & 0xff);
        if (b == widx[t]) acc[e] += (e & 1) ? hi_bf(d[t][e >> 1]) : lo_bf(d[t][e >> 1]);
      }
    }
    v4u out;
#pragma unroll
    for (int e = 0; e < 4; ++e) out[e] = pack2bf(acc[2 * e], acc[2 * e + 1]);
    reinterpret_cast<v4u*>(dx)[i] = out;
  }
}

// Output-centric backward of the 3x3 / stride-2 / pad-1 window on an input of exactly 2 OH x 2 OW (the ResNet stem
// pool): a thread owns output (oh, ow)'s 8-channel granule and writes the 2 x 2 input block (2 oh + a, 2 ow + b), which
// only outputs (oh, ow), (oh, ow + 1), (oh + 1, ow), (oh + 1, ow + 1) reach: 4 dy / index loads per 4 dx stores,
// instead of 4 per store in the input-centric gather (308 -> ~110 us on the 256 x 64 x 112^2 stem output).
// Window tap t = r * 3 + s of output (oh, ow) is input (2 oh - 1 + r, 2 ow - 1 + s) (maxpool_fwd_fixed_kernel).
// BNR: dx is the gradient of a training BN's (ReLU-fused) output (the ResNet stem's BN feeds this pool): the kernel
// also accumulates that BN's backward reduction (sum dz*m, sum dz*m*(x - mean), m the ReLU mask from the sign bits
// `zm` or from x*scale + shift) into the slotted statistics `red`, so the BN backward skips its chan_reduce pass over
// dz and x (csrc/batchnorm.hip chan_reduce_kernel MODE 1 computes the same sums). Needs 256 % (C/8) == 0 so a
// thread's channel group is fixed over the grid-stride loop.
struct PoolBnRed {
  const bf16_t* x;      // the BN's input, same layout as dx
  const float* mean;
  const float* aff;     // [scale | shift] (mask from x) or nullptr
  const uint8_t* zm;    // [P][C/8] sign bits or nullptr
  float* red;           // [STAT_SLOTS][2][C]
};

template <bool BNR>
__global__ __launch_bounds__(256) void maxpool_bwd_k3s2_kernel(const bf16_t* __restrict__ dy,
                                                               const uint8_t* __restrict__ idx, bf16_t* __restrict__ dx,
                                                               int N, int C, int OH, int OW, PoolBnRed br) {
  const int G = C >> 3;
  const long total = (long)N * OH * OW * G;
  const int W = 2 * OW;
  float s1[8], s2[8], mu[8], sc[8], sf[8];
  const __amdgpu_buffer_rsrc_t rzm = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(br.zm), (short)0, br.zm ? (int)min(total * 4, 0x7fffffffl) : 0, 0x00020000);
  if (BNR) {
    const int g0 = threadIdx.x % G;
    // scale / shift through a buffer resource (0 bytes without aff): a load under `if (aff)` was waited for at the
    // join, one round trip per element before the first row
    const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(br.aff), (short)0,
                                                                        br.aff ? 8 * C : 0, 0x00020000);
    const v4f m0 = *reinterpret_cast<const v4f*>(br.mean + g0 * 8), m1 = *reinterpret_cast<const v4f*>(br.mean + g0 * 8 + 4);
    const v4f a0 = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(ra, (unsigned)(g0 * 32), 0, 0));
    const v4f a1 = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(ra, (unsigned)(g0 * 32 + 16), 0, 0));
    const v4f b0 = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(ra, (unsigned)((C + g0 * 8) * 4), 0, 0));
    const v4f b1 = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(ra, (unsigned)((C + g0 * 8) * 4 + 16), 0, 0));
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s1[e] = s2[e] = s1[e + 4] = s2[e + 4] = 0.f;
      mu[e] = m0[e]; mu[e + 4] = m1[e];
      sc[e] = a0[e]; sc[e + 4] = a1[e];
      sf[e] = b0[e]; sf[e + 4] = b1[e];
    }
  }
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const int g = (int)(i % G);
    long p = i / G;
    const int ow = (int)(p % OW);
    p /= OW;
    const int oh = (int)(p % OH);
    const int n = (int)(p / OH);
    const bool r1 = ow + 1 < OW, d1 = oh + 1 < OH;
    const long o00 = ((long)(n * OH + oh) * OW + ow) * G + g;
    const long o01 = r1 ? o00 + G : o00, o10 = d1 ? o00 + (long)OW * G : o00, o11 = (r1 && d1) ? o10 + G : o00;
    const v4u d00 = reinterpret_cast<const v4u*>(dy)[o00], d01 = reinterpret_cast<const v4u*>(dy)[o01];
    const v4u d10 = reinterpret_cast<const v4u*>(dy)[o10], d11 = reinterpret_cast<const v4u*>(dy)[o11];
    const uint2 x00 = reinterpret_cast<const uint2*>(idx)[o00], x01 = reinterpret_cast<const uint2*>(idx)[o01];
    const uint2 x10 = reinterpret_cast<const uint2*>(idx)[o10], x11 = reinterpret_cast<const uint2*>(idx)[o11];
    // a neighbour past the edge contributes nothing: an impossible tap index
    const unsigned m01 = r1 ? 0u : 0xffffffffu, m10 = d1 ? 0u : 0xffffffffu, m11 = (r1 && d1) ? 0u : 0xffffffffu;
    v4u q[4];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int sh = (e & 3) * 8;
      const unsigned t00 = ((e < 4 ? x00.x : x00.y) >> sh) & 0xff;
      const unsigned t01 = (((e < 4 ? x01.x : x01.y) >> sh) & 0xff) | (m01 & 0x100);
      const unsigned t10 = (((e < 4 ? x10.x : x10.y) >> sh) & 0xff) | (m10 & 0x100);
      const unsigned t11 = (((e < 4 ? x11.x : x11.y) >> sh) & 0xff) | (m11 & 0x100);
      const float v00 = (e & 1) ? hi_bf(d00[e >> 1]) : lo_bf(d00[e >> 1]);
      const float v01 = (e & 1) ? hi_bf(d01[e >> 1]) : lo_bf(d01[e >> 1]);
      const float v10 = (e & 1) ? hi_bf(d10[e >> 1]) : lo_bf(d10[e >> 1]);
      const float v11 = (e & 1) ? hi_bf(d11[e >> 1]) : lo_bf(d11[e >> 1]);
      // input (2oh, 2ow): tap 4 of (oh, ow); (2oh, 2ow+1): 5 of (oh, ow), 3 of (oh, ow+1);
      // (2oh+1, 2ow): 7 of (oh, ow), 1 of (oh+1, ow); (2oh+1, 2ow+1): 8, 6 of (oh, ow+1), 2 of (oh+1, ow), 0 of (oh+1, ow+1)
      const float a00 = t00 == 4 ? v00 : 0.f;
      const float a01 = (t00 == 5 ? v00 : 0.f) + (t01 == 3 ? v01 : 0.f);
      const float a10 = (t00 == 7 ? v00 : 0.f) + (t10 == 1 ? v10 : 0.f);
      const float a11 = (t00 == 8 ? v00 : 0.f) + (t01 == 6 ? v01 : 0.f) + (t10 == 2 ? v10 : 0.f) + (t11 == 0 ? v11 : 0.f);
      const float av[4] = {a00, a01, a10, a11};
      const int ee = e >> 1;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned hb = (unsigned)f2bf(av[k]);
        if (e & 1) q[k][ee] |= hb << 16;
        else q[k][ee] = hb;
      }
    }
    const long row0 = ((long)n * (2 * OH) + 2 * oh) * W + 2 * ow;
    const long pix[4] = {row0, row0 + 1, row0 + W, row0 + W + 1};
    if (BNR) {
      v4u bx[4];
      unsigned zb[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {      // unconditional mask byte (0-byte resource when absent): no wait at a join
        bx[k] = reinterpret_cast<const v4u*>(br.x)[pix[k] * G + g];
        zb[k] = __builtin_amdgcn_raw_buffer_load_b8(rzm, (unsigned)(pix[k] * G + g), 0, 0);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // the gradient as stored (bf16), as the unfused reduction reads it back
          const float d = (e & 1) ? hi_bf(q[k][e >> 1]) : lo_bf(q[k][e >> 1]);
          const float xv = (e & 1) ? hi_bf(bx[k][e >> 1]) : lo_bf(bx[k][e >> 1]);
          const bool on = br.zm ? ((zb[k] >> e) & 1u) != 0u : (xv * sc[e] + sf[e] > 0.f);
          const float dm = on ? d : 0.f;
          s1[e] += dm;
          s2[e] += dm * (xv - mu[e]);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) reinterpret_cast<v4u*>(dx)[pix[k] * G + g] = q[k];
  }
  if (BNR) {
    // per-workgroup sums through LDS, then one atomic per (slot, channel, sum) (rows of threads share a group)
    __shared__ float sm[256 * 16];
#pragma unroll
    for (int e = 0; e < 8; ++e) { sm[threadIdx.x * 16 + e] = s1[e]; sm[threadIdx.x * 16 + 8 + e] = s2[e]; }
    __syncthreads();
    const int rows = 256 / G;
    for (int w = threadIdx.x; w < G * 16; w += 256) {
      const int gg = w >> 4, slot = w & 15;
      float t = 0.f;
      for (int r = 0; r < rows; ++r) t += sm[(r * G + gg) * 16 + slot];
      const int ch = gg * 8 + (slot & 7);
      atomicAdd(br.red + (size_t)(blockIdx.x & (BIGDL_STAT_SLOTS - 1)) * 2 * C + (slot < 8 ? 0 : C) + ch, t);
    }
  }
}

__device__ __forceinline__ int pool_count(int oh, int ow, int H, int W, int kh, int kw, int sh, int sw, int ph, int pw,
                                          int count_pad) {
  int hs = oh * sh - ph, ws = ow * sw - pw;
  int he = min(hs + kh, H + ph), we = min(ws + kw, W + pw);
  const int pool = (he - hs) * (we - ws);
  if (count_pad) return pool;
  hs = max(hs, 0); ws = max(ws, 0); he = min(he, H); we = min(we, W);
  return max((he - hs) * (we - ws), 1);
}

__global__ void avgpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int N, int H, int W, int C,
                                   int OH, int OW, int kh, int kw, int sh, int sw, int ph, int pw, int count_pad) {
  const int G = C >> 3;
  const long total = (long)N * OH * OW * G;
  GRID_STRIDE(i, total) {
    const int g = i % G;
    long p = i / G;
    const int ow = p % OW; p /= OW;
    const int oh = p % OH;
    const int n = p / OH;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int r = 0; r < kh; ++r) {
      const int ih = oh * sh - ph + r;
      if ((unsigned)ih >= (unsigned)H) continue;
      for (int s = 0; s < kw; ++s) {
        const int iw = ow * sw - pw + s;
        if ((unsigned)iw >= (unsigned)W) continue;
        const v4u v = *reinterpret_cast<const v4u*>(x + (((long)n * H + ih) * W + iw) * C + g * 8);
#pragma unroll
        for (int e = 0; e < 4; ++e) { acc[2 * e] += lo_bf(v[e]); acc[2 * e + 1] += hi_bf(v[e]); }
      }
    }
    const float inv = 1.f / (float)pool_count(oh, ow, H, W, kh, kw, sh, sw, ph, pw, count_pad);
    v4u o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2bf(acc[2 * e] * inv, acc[2 * e + 1] * inv);
    reinterpret_cast<v4u*>(y)[i] = o;
  }
}

__global__ void avgpool_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, int N, int H, int W, int C,
                                   int OH, int OW, int kh, int kw, int sh, int sw, int ph, int pw, int count_pad) {
  const int G = C >> 3;
  const long total = (long)N * H * W * G;
  GRID_STRIDE(i, total) {
    const int g = i % G;
    long p = i / G;
    const int iw = p % W; p /= W;
    const int ih = p % H;
    const int n = p / H;
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    const int oh_lo = max(0, (ih + ph - kh + sh) / sh), oh_hi = min(OH - 1, (ih + ph) / sh);
    const int ow_lo = max(0, (iw + pw - kw + sw) / sw), ow_hi = min(OW - 1, (iw + pw) / sw);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int r = ih + ph - oh * sh;
      if (r < 0 || r >= kh) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int s = iw + pw - ow * sw;
        if (s < 0 || s >= kw) continue;
        const float inv = 1.f / (float)pool_count(oh, ow, H, W, kh, kw, sh, sw, ph, pw, count_pad);
        const v4u d = *reinterpret_cast<const v4u*>(dy + (((long)n * OH + oh) * OW + ow) * C + g * 8);
#pragma unroll
        for (int e = 0; e < 4; ++e) { acc[2 * e] += lo_bf(d[e]) * inv; acc[2 * e + 1] += hi_bf(d[e]) * inv; }
      }
    }
    v4u o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2bf(acc[2 * e], acc[2 * e + 1]);
    reinterpret_cast<v4u*>(dx)[i] = o;
  }
}

// ---------------- fused log-softmax + NLL: one wave per row ----------------
// Fused log-softmax + NLL (+ gradient). One wave per row, rows grid-strided; a single online max/sum pass
// (running max with rescaled sum) over 16-byte loads, a second pass writes the gradient. Each block reduces its
// rows' losses in LDS and issues ONE atomic (16k-row LM batches would otherwise serialise on one address).
template <bool VEC>
__global__ __launch_bounds__(256) void softmax_xent_kernel(const bf16_t* __restrict__ lb, const float* __restrict__ lf,
                                                           const float* __restrict__ labels, float* __restrict__ loss,
                                                           bf16_t* __restrict__ db, float* __restrict__ df, int B, int K,
                                                           float label_base, float grad_scale) {
  __shared__ float part[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float my_loss = 0.f;
  for (int row = blockIdx.x * 4 + wave; row < B; row += gridDim.x * 4) {
    const long base = (long)row * K;
    float mx = -INFINITY, se = 0.f;
    auto acc = [&](float v) {
      if (v > mx) { se = se * __expf(mx - v) + 1.f; mx = v; } else { se += __expf(v - mx); }
    };
    if (VEC && lb) {            // 8 bf16 per lane per load
      const v4u* p = (const v4u*)(lb + base);
      for (int q = lane; q < (K >> 3); q += 64) {
        const v4u v = p[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) { acc(lo_bf(v[e])); acc(hi_bf(v[e])); }
      }
    } else if (VEC) {           // 4 fp32 per lane per load
      const float4* p = (const float4*)(lf + base);
      for (int q = lane; q < (K >> 2); q += 64) {
        const float4 v = p[q];
        acc(v.x); acc(v.y); acc(v.z); acc(v.w);
      }
    } else {
      for (int k = lane; k < K; k += 64) acc(lb ? bf2f(lb[base + k]) : lf[base + k]);
    }
    const float m_all = wave_max(mx);
    se = (mx == -INFINITY) ? 0.f : se * __expf(mx - m_all);
    const float s_all = wave_sum(se);
    const float lse = m_all + __logf(s_all);
    const int tgt = (int)(labels[row] - label_base);
    if (lane == 0) {
      const float xt = (tgt >= 0 && tgt < K) ? (lb ? bf2f(lb[base + tgt]) : lf[base + tgt]) : lse;
      my_loss += (lse - xt) * grad_scale;
    }
    if (db || df) {
      const float inv = 1.f / s_all;
      if (VEC && lb && db) {
        const v4u* p = (const v4u*)(lb + base);
        v4u* o = (v4u*)(db + base);
        for (int q = lane; q < (K >> 3); q += 64) {
          const v4u v = p[q];
          v4u w;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int k = q * 8 + 2 * e;
            const float g0 = (__expf(lo_bf(v[e]) - m_all) * inv - (k == tgt ? 1.f : 0.f)) * grad_scale;
            const float g1 = (__expf(hi_bf(v[e]) - m_all) * inv - (k + 1 == tgt ? 1.f : 0.f)) * grad_scale;
            w[e] = pack2bf(g0, g1);
          }
          o[q] = w;
        }
      } else if (VEC && !lb && df) {
        const float4* p = (const float4*)(lf + base);
        float4* o = (float4*)(df + base);
        for (int q = lane; q < (K >> 2); q += 64) {
          const float4 v = p[q];
          const int k = q * 4;
          float4 g;
          g.x = (__expf(v.x - m_all) * inv - (k == tgt ? 1.f : 0.f)) * grad_scale;
          g.y = (__expf(v.y - m_all) * inv - (k + 1 == tgt ? 1.f : 0.f)) * grad_scale;
          g.z = (__expf(v.z - m_all) * inv - (k + 2 == tgt ? 1.f : 0.f)) * grad_scale;
          g.w = (__expf(v.w - m_all) * inv - (k + 3 == tgt ? 1.f : 0.f)) * grad_scale;
          o[q] = g;
        }
      } else {
        for (int k = lane; k < K; k += 64) {
          const float x = lb ? bf2f(lb[base + k]) : lf[base + k];
          const float g = (__expf(x - m_all) * inv - (k == tgt ? 1.f : 0.f)) * grad_scale;
          if (db) db[base + k] = f2bf(g);
          else df[base + k] = g;
        }
      }
    }
  }
  if (loss) {
    if (lane == 0) part[wave] = my_loss;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(loss, part[0] + part[1] + part[2] + part[3]);
  }
}

// ---------------- optimizers on flat fp32 buffers ----------------
// Segment-wise weight decay: the flat buffer is a concatenation of parameter tensors; seg_off[i] is the
// first (global) element of segment i and seg_wd[i] its L2 coefficient (folded layer regularizers).
__device__ __forceinline__ float seg_decay(const long* __restrict__ seg_off, const float* __restrict__ seg_wd,
                                           int nseg, long gi) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (seg_off[mid] <= gi) lo = mid; else hi = mid - 1;
  }
  return seg_wd[lo];
}

__global__ void sgd_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ mom,
                           bf16_t* __restrict__ w16, long n, const float* __restrict__ lr_dev, float lr, float wd,
                           float momentum, float dampening, int nesterov, int first, const long* __restrict__ seg_off,
                           const float* __restrict__ seg_wd, int nseg, long base) {
  const float rate = lr_dev ? lr_dev[0] : lr;
  GRID_STRIDE(i, n) {
    float wi = w[i];
    float decay = wd;
    if (nseg) decay += seg_decay(seg_off, seg_wd, nseg, base + i);
    float d = g[i] + decay * wi;
    if (momentum != 0.f) {
      float b = first ? d : momentum * mom[i] + (1.f - dampening) * d;
      mom[i] = b;
      d = nesterov ? d + momentum * b : b;
    }
    wi -= rate * d;
    w[i] = wi;
    if (w16) w16[i] = f2bf(wi);
  }
}

// 4 elements per lane (16-byte fp32 loads / stores, 8-byte bf16 shadow store); the weight-decay segment is found by
// one binary search per 4 elements and then stepped forward (segments span thousands of elements).
__global__ void sgd4_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ mom,
                            bf16_t* __restrict__ w16, long n4, const float* __restrict__ lr_dev, float lr, float wd,
                            float momentum, float dampening, int nesterov, int first, const long* __restrict__ seg_off,
                            const float* __restrict__ seg_wd, int nseg, long base) {
  const float rate = lr_dev ? lr_dev[0] : lr;
  GRID_STRIDE(i, n4) {
    const v4f wv = reinterpret_cast<const v4f*>(w)[i];
    const v4f gv = reinterpret_cast<const v4f*>(g)[i];
    v4f mv = {0.f, 0.f, 0.f, 0.f};
    if (momentum != 0.f && !first) mv = reinterpret_cast<const v4f*>(mom)[i];
    float dec[4] = {wd, wd, wd, wd};
    if (nseg) {
      const long g0 = base + 4 * i;
      int lo = 0, hi = nseg - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (seg_off[mid] <= g0) lo = mid; else hi = mid - 1;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        while (lo + 1 < nseg && seg_off[lo + 1] <= g0 + e) ++lo;
        dec[e] += seg_wd[lo];
      }
    }
    v4f wo, mo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float d = gv[e] + dec[e] * wv[e];
      if (momentum != 0.f) {
        const float b = first ? d : momentum * mv[e] + (1.f - dampening) * d;
        mo[e] = b;
        d = nesterov ? d + momentum * b : b;
      }
      wo[e] = wv[e] - rate * d;
    }
    reinterpret_cast<v4f*>(w)[i] = wo;
    if (momentum != 0.f) reinterpret_cast<v4f*>(mom)[i] = mo;
    if (w16) reinterpret_cast<v2u*>(w16)[i] = v2u{pack2bf(wo[0], wo[1]), pack2bf(wo[2], wo[3])};
  }
}

__global__ void adam_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, bf16_t* __restrict__ w16, long n, float lr, float b1, float b2,
                            float eps, float wd, float bc1, float bc2) {
  GRID_STRIDE(i, n) {
    float wi = w[i];
    const float gi = g[i] + wd * wi;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi; v[i] = vi;
    // BigDL Adam: x -= lr * sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps)
    wi -= lr * (sqrtf(bc2) / bc1) * mi / (sqrtf(vi) + eps);
    w[i] = wi;
    if (w16) w16[i] = f2bf(wi);
  }
}

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ x, float* __restrict__ out, long n) {
  float acc = 0.f;
  GRID_STRIDE(i, n) { const float v = x[i]; acc += v * v; }
  acc = wave_sum(acc);
  __shared__ float sm[4];
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, sm[0] + sm[1] + sm[2] + sm[3]);
}

// the 128 per-block partials go to a caller-provided workspace (a caching-allocator tensor of the launching stream),
// not a process-global device array: concurrent launches on different streams (the weight-gradient stream, prediction
// replicas) cannot overwrite each other's slots
__global__ __launch_bounds__(256) void sumsq_det_kernel(const float* __restrict__ x, long n, float* __restrict__ slots) {
  float acc = 0.f;
  GRID_STRIDE(i, n) { const float v = x[i]; acc += v * v; }
  acc = wave_sum(acc);
  __shared__ float sm[4];
  if ((threadIdx.x & 63) == 0) sm[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) slots[blockIdx.x] = sm[0] + sm[1] + sm[2] + sm[3];
}
__global__ void sumsq_det_finish_kernel(float* __restrict__ out, const float* __restrict__ slots) {
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int s = 0; s < BIGDL_DET_SLOTS; ++s) t += slots[s];
    out[0] += t;
  }
}

__global__ void scale_kernel(float* __restrict__ x, long n, const float* __restrict__ sdev, float s) {
  const float f = sdev ? sdev[0] : s;
  GRID_STRIDE(i, n) x[i] *= f;
}

// ---------------- LSTM cell pointwise (gate order: input, hidden(cell), forget, output) ----------------
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ void lstm_fwd_kernel(const float* __restrict__ gates, const float* __restrict__ c_prev, float* __restrict__ c,
                                float* __restrict__ h, float* __restrict__ act, int B, int H) {
  const long total = (long)B * H;
  GRID_STRIDE(idx, total) {
    const int b = idx / H, j = idx % H;
    const float* gr = gates + (long)b * 4 * H;
    const float ig = sigm(gr[j]), gg = tanhf(gr[H + j]), fg = sigm(gr[2 * H + j]), og = sigm(gr[3 * H + j]);
    const float cp = c_prev ? c_prev[idx] : 0.f;
    const float cn = fg * cp + ig * gg;
    c[idx] = cn;
    h[idx] = og * tanhf(cn);
    float* ar = act + (long)b * 4 * H;
    ar[j] = ig; ar[H + j] = gg; ar[2 * H + j] = fg; ar[3 * H + j] = og;
  }
}

__global__ void lstm_bwd_kernel(const float* __restrict__ act, const float* __restrict__ c_prev, const float* __restrict__ c,
                                const float* __restrict__ dh, const float* __restrict__ dc_next, float* __restrict__ dgates,
                                float* __restrict__ dc_prev, int B, int H) {
  const long total = (long)B * H;
  GRID_STRIDE(idx, total) {
    const int b = idx / H, j = idx % H;
    const float* ar = act + (long)b * 4 * H;
    const float ig = ar[j], gg = ar[H + j], fg = ar[2 * H + j], og = ar[3 * H + j];
    const float tc = tanhf(c[idx]);
    const float dhv = dh ? dh[idx] : 0.f;
    const float dcv = dhv * og * (1.f - tc * tc) + (dc_next ? dc_next[idx] : 0.f);
    const float cp = c_prev ? c_prev[idx] : 0.f;
    float* dg = dgates + (long)b * 4 * H;
    dg[j] = dcv * gg * ig * (1.f - ig);
    dg[H + j] = dcv * ig * (1.f - gg * gg);
    dg[2 * H + j] = dcv * cp * fg * (1.f - fg);
    dg[3 * H + j] = dhv * tc * og * (1.f - og);
    if (dc_prev) dc_prev[idx] = dcv * fg;
  }
}

}  // namespace

extern "C" {

void bigdl_relu_fwd(const uint16_t* x, uint16_t* y, long n, hipStream_t st) {
  const long n8 = n >> 3;
  if (n8) relu_fwd_kernel<<<grid_cap(n8), 256, 0, st>>>((const v4u*)x, (v4u*)y, n8);
  if (n8 * 8 < n) relu_fwd_tail<<<1, 256, 0, st>>>(x, y, n8 * 8, n);
  HIP_LAUNCH_CHECK();
}
void bigdl_relu_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long n, hipStream_t st) {
  const long n8 = n >> 3;
  if (n8) relu_bwd_kernel<<<grid_cap(n8), 256, 0, st>>>((const v4u*)dy, (const v4u*)y, (v4u*)dx, n8);
  if (n8 * 8 < n) relu_bwd_tail<<<1, 256, 0, st>>>(dy, y, dx, n8 * 8, n);
  HIP_LAUNCH_CHECK();
}
void bigdl_add_bf16(const uint16_t* a, const uint16_t* b, uint16_t* y, long n, hipStream_t st) {
  const long n8 = n >> 3;
  if (n8) add_kernel<<<grid_cap(n8), 256, 0, st>>>((const v4u*)a, (const v4u*)b, (v4u*)y, n8);
  if (n8 * 8 < n) add_tail<<<1, 256, 0, st>>>(a, b, y, n8 * 8, n);
  HIP_LAUNCH_CHECK();
}
void bigdl_nchw_f32_to_nhwc_bf16(const float* x, uint16_t* y, int N, int C, int H, int W, int Cp, hipStream_t st) {
  if (Cp % 8 != 0) return;   // the host pads channels to a multiple of 8
  const dim3 grid((H * W + 255) / 256, std::min(N * (Cp / 8), 65535));
  nchw_to_nhwc_kernel<<<grid, 256, 0, st>>>(x, y, N, C, H, W, Cp);
  HIP_LAUNCH_CHECK();
}
// Deterministic mode (bigdl_set_deterministic): every reduction that lands through float atomics from several
// workgroups is launched so each output element receives exactly ONE atomic (one row block, unique statistics slots),
// or is replaced by a fixed-order pass; training runs are then bitwise reproducible (tests/test_deterministic_gpu.py).
int g_det = -1;
int bigdl_deterministic() {
  if (g_det < 0) {
    const char* e = getenv("BIGDL_DETERMINISTIC");
    g_det = (e && atoi(e) != 0) ? 1 : 0;
  }
  return g_det;
}
void bigdl_set_deterministic(int v) { g_det = v ? 1 : 0; }

void bigdl_colsum_bf16(const uint16_t* x, float* out, long P, int K, hipStream_t st, float* det_ws) {
  bigdl_colsum_bf16_ld(x, out, P, K, K, st, det_ws);
}
// Deterministic column sum: row block y writes its partial to its own slot of the caller's workspace ([by][K] fp32;
// plain stores, no atomics), then one fixed-order pass adds the slots into out (one writer per column).
// Deterministic column sums, pass 1: block (bx, by) sums the channel groups [bx * CGB, + CGB) (8 channels each,
// CGB = min(K / 8, 64)) over its row range into slots[by][.]. A wave covers 64 / CGB rows per trip with every lane
// busy (narrow K no longer idles most of the wave), 4 rows per lane in flight; the block's partials meet in LDS in a
// fixed order.
__global__ void __launch_bounds__(256) colsum_det_kernel(const bf16_t* __restrict__ x, long P, int K,
                                                        long rows_per_block, long ld, float* __restrict__ slots) {
  constexpr int U = 4;
  __shared__ float part[256][9];
  const int Kg = K >> 3;
  const int CGB = Kg < 64 ? Kg : 64, RW = 64 / CGB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cgl = lane % CGB, ro = lane / CGB;
  const int cg = blockIdx.x * CGB + cgl;
  const long r0 = (long)blockIdx.y * rows_per_block;
  const long r1 = r0 + rows_per_block < P ? r0 + rows_per_block : P;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (ro < RW && cg < Kg) {
    const long step = 4L * RW;
    for (long r = r0 + wave * RW + ro; r < r1; r += U * step) {
      v4u q[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long rr = r + u * step;
        q[u] = *reinterpret_cast<const v4u*>(x + (rr < r1 ? rr : r) * ld + cg * 8);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float m = r + u * step < r1 ? 1.f : 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) { acc[2 * e] += m * lo_bf(q[u][e]); acc[2 * e + 1] += m * hi_bf(q[u][e]); }
      }
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[threadIdx.x][e] = acc[e];
  __syncthreads();
  for (int c = threadIdx.x; c < CGB * 8; c += 256) {
    const int g = c >> 3, e = c & 7;
    if (blockIdx.x * CGB + g >= Kg) continue;
    float t = 0.f;
    for (int w = 0; w < 4; ++w)
      for (int rr = 0; rr < RW; ++rr) t += part[w * 64 + rr * CGB + g][e];
    slots[(size_t)blockIdx.y * K + (blockIdx.x * CGB + g) * 8 + e] = t;
  }
}
__global__ void __launch_bounds__(256) colsum_det_finish_kernel(float* __restrict__ out, int K, int nslots,
                                                               const float* __restrict__ slots) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= K) return;
  // 8 interleaved partial sums (slot s into t[s % 8]), combined in a fixed order: deterministic, and the loads of
  // 8 slots are in flight together instead of one dependent chain
  float t[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int s = 0;
  for (; s + 8 <= nslots; s += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] += slots[(size_t)(s + u) * K + c];
  }
  for (; s < nslots; ++s) t[s & 7] += slots[(size_t)s * K + c];
  out[c] += ((t[0] + t[1]) + (t[2] + t[3])) + ((t[4] + t[5]) + (t[6] + t[7]));
}

// out[k] += sum over P rows (row stride ld, ld % 8 == 0) of x[r][k]. Deterministic mode: with det_ws (>= BIGDL_DET_SLOTS
// x K floats) the slotted two-pass form, else one row block (one writer per column, slower).
void bigdl_colsum_bf16_ld(const uint16_t* x, float* out, long P, int K, long ld, hipStream_t st, float* det_ws) {
  const int bx = (K / 8 + 63) / 64;
  long by = (P + 255) / 256;                   // >= 64 rows per wave, ~2048 blocks at most
  if (bigdl_deterministic() && det_ws != nullptr) {
    if (by > BIGDL_DET_SLOTS) by = BIGDL_DET_SLOTS;
    if (by < 1) by = 1;
    const long rpb = (P + by - 1) / by;
    by = (P + rpb - 1) / rpb;
    colsum_det_kernel<<<dim3(bx, (unsigned)by), 256, 0, st>>>(x, P, K, rpb, ld, det_ws);
    colsum_det_finish_kernel<<<(K + 255) / 256, 256, 0, st>>>(out, K, (int)by, det_ws);
    HIP_LAUNCH_CHECK();
    return;
  }
  if ((long)bx * by > 2048) by = (2048 + bx - 1) / bx;
  if (by < 1 || bigdl_deterministic()) by = 1;
  const long rpb = (P + by - 1) / by;
  colsum_bf16_kernel<<<dim3(bx, (unsigned)by), 256, 0, st>>>(x, out, P, K, rpb, ld);
  HIP_LAUNCH_CHECK();
}

// Linear on hipBLASLt (nn/linear.py): the weight-gradient GEMM's B operand is [x | 1 | 0 x 7] (bf16, K + 8 columns)
// so its last useful column is the bias gradient. Pack: one 16-byte granule per thread (K % 8 == 0).
__global__ void ones_col_pack_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xe, long M, int K) {
  const int gpr = K / 8 + 1;
  const long total = M * gpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / gpr;
    const int g = (int)(i - r * gpr);
    v4u v;
    if (g < gpr - 1) v = *reinterpret_cast<const v4u*>(x + r * K + g * 8);
    else v = v4u{0x3f80u, 0u, 0u, 0u};                  // bf16 1.0 then zeros
    *reinterpret_cast<v4u*>(xe + r * (K + 8) + g * 8) = v;
  }
}
// gW[n][k] += sW * gw[n][k], gB[n] += sB * gw[n][K] (gw: [N][K + 8] fp32 from the GEMM)
__global__ void ones_col_acc_kernel(const float* __restrict__ gw, float* __restrict__ gW, float* __restrict__ gB, long N,
                                    int K, float sW, float sB) {
  const int cpr = K / 4 + 1;                           // float4 chunks per row, then one bias word
  const long total = N * cpr;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / cpr;
    const int c = (int)(i - n * cpr);
    if (c < cpr - 1) {
      const v4f g = *reinterpret_cast<const v4f*>(gw + n * (K + 8) + c * 4);
      v4f w = *reinterpret_cast<const v4f*>(gW + n * K + c * 4);
      w += g * sW;
      *reinterpret_cast<v4f*>(gW + n * K + c * 4) = w;
    } else if (gB) {
      gB[n] += sB * gw[n * (K + 8) + K];
    }
  }
}

void bigdl_ones_col_pack(const uint16_t* x, uint16_t* xe, long M, int K, hipStream_t st) {
  ones_col_pack_kernel<<<grid_cap(M * (K / 8 + 1)), 256, 0, st>>>(x, xe, M, K);
  HIP_LAUNCH_CHECK();
}
void bigdl_ones_col_acc(const float* gw, float* gW, float* gB, long N, int K, float sW, float sB, hipStream_t st) {
  ones_col_acc_kernel<<<grid_cap(N * (K / 4 + 1)), 256, 0, st>>>(gw, gW, gB, N, K, sW, sB);
  HIP_LAUNCH_CHECK();
}
void bigdl_cast_f32_bf16(const float* x, uint16_t* y, long n, hipStream_t st) {
  cast_f32_bf16_kernel<<<grid_cap(n / 4 + 1), 256, 0, st>>>(x, y, n);
  HIP_LAUNCH_CHECK();
}
void bigdl_cast_bf16_f32(const uint16_t* x, float* y, long n, hipStream_t st) {
  cast_bf16_f32_kernel<<<grid_cap(n), 256, 0, st>>>(x, y, n);
  HIP_LAUNCH_CHECK();
}
void bigdl_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C, int OH, int OW,
                       int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t st, const float* pre) {
  const long outs = (long)N * OH * OW * (C / 8), ins = (long)N * H * W * C;
  const bool fixed = kh == 3 && kw == 3 && sh == 2 && sw == 2 && outs < (1l << 31) && ins < (1l << 31);
  if (pre) {   // bigdl_maxpool_pre_applies: the fixed window only
    maxpool_fwd_fixed_kernel<3, 2, true><<<grid_cap(outs), 256, 0, st>>>(x, y, idx, N, H, W, C, OH, OW, ph, pw, pre);
  } else if (fixed)
    maxpool_fwd_fixed_kernel<3, 2><<<grid_cap(outs), 256, 0, st>>>(x, y, idx, N, H, W, C, OH, OW, ph, pw);
  else
    maxpool_fwd_kernel<<<grid_cap(outs), 256, 0, st>>>(x, y, idx, N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw);
  HIP_LAUNCH_CHECK();
}
int bigdl_maxpool_pre_applies(int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh, int sw) {
  const long outs = (long)N * OH * OW * (C / 8), ins = (long)N * H * W * C;
  return kh == 3 && kw == 3 && sh == 2 && sw == 2 && outs < (1l << 31) && ins < (1l << 31) && C % 8 == 0;
}
static bool maxpool_k3s2_ok(int H, int W, int C, int OH, int OW, int kh, int kw, int sh, int sw, int ph, int pw,
                            long ins, long outs) {
  static const bool k3s2 = [] { const char* e = getenv("BIGDL_POOL_BWD_K3S2"); return e ? atoi(e) != 0 : true; }();
  return k3s2 && kh == 3 && kw == 3 && sh == 2 && sw == 2 && ph == 1 && pw == 1 && H == 2 * OH && W == 2 * OW &&
         C % 8 == 0 && ins < (1l << 31) && outs < (1l << 31);
}
int bigdl_maxpool_bwd_bnred_applies(int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh, int sw, int ph,
                                    int pw) {
  const long ins = (long)N * H * W * (C / 8), outs = (long)N * OH * OW * C;
  return maxpool_k3s2_ok(H, W, C, OH, OW, kh, kw, sh, sw, ph, pw, ins, outs) && 256 % (C / 8) == 0 &&
         !bigdl_deterministic();
}
// maxpool backward fused with the backward reduction of the BN that produced the pool's input (see PoolBnRed)
void bigdl_maxpool_bwd_bnred(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int C, int OH, int OW,
                             const uint16_t* bx, const float* mean, const float* aff, const uint8_t* zm, float* red,
                             hipStream_t st) {
  const PoolBnRed br{reinterpret_cast<const bf16_t*>(bx), mean, aff, zm, red};
  maxpool_bwd_k3s2_kernel<true><<<grid_cap((long)N * OH * OW * (C / 8), 2048), 256, 0, st>>>(dy, idx, dx, N, C, OH,
                                                                                              OW, br);
  HIP_LAUNCH_CHECK();
}
void bigdl_maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H, int W, int C, int OH,
                       int OW, int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t st) {
  const long ins = (long)N * H * W * (C / 8), outs = (long)N * OH * OW * C;
  if (maxpool_k3s2_ok(H, W, C, OH, OW, kh, kw, sh, sw, ph, pw, ins, outs))
    maxpool_bwd_k3s2_kernel<false><<<grid_cap((long)N * OH * OW * (C / 8)), 256, 0, st>>>(dy, idx, dx, N, C, OH, OW,
                                                                                         PoolBnRed{});
  else if (kh == 3 && kw == 3 && sh == 2 && sw == 2 && ins < (1l << 31) && outs < (1l << 31))
    maxpool_bwd_fixed_kernel<3, 2><<<grid_cap(ins), 256, 0, st>>>(dy, idx, dx, N, H, W, C, OH, OW, ph, pw);
  else
    maxpool_bwd_kernel<<<grid_cap(ins), 256, 0, st>>>(dy, idx, dx, N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw);
  HIP_LAUNCH_CHECK();
}
void bigdl_avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int H, int W, int C, int OH, int OW, int kh, int kw,
                       int sh, int sw, int ph, int pw, int count_pad, hipStream_t st) {
  avgpool_fwd_kernel<<<grid_cap((long)N * OH * OW * (C / 8)), 256, 0, st>>>(x, y, N, H, W, C, OH, OW, kh, kw, sh, sw,
                                                                            ph, pw, count_pad);
  HIP_LAUNCH_CHECK();
}
void bigdl_avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int H, int W, int C, int OH, int OW, int kh, int kw,
                       int sh, int sw, int ph, int pw, int count_pad, hipStream_t st) {
  avgpool_bwd_kernel<<<grid_cap((long)N * H * W * (C / 8)), 256, 0, st>>>(dy, dx, N, H, W, C, OH, OW, kh, kw, sh, sw,
                                                                          ph, pw, count_pad);
  HIP_LAUNCH_CHECK();
}
void bigdl_softmax_xent(const uint16_t* lb, const float* lf, const float* labels, float* loss, uint16_t* db, float* df,
                        int B, int K, float label_base, float grad_scale, hipStream_t st) {
  const int blocks = bigdl_deterministic() ? 1 : std::min((B + 3) / 4, 2048);   // det: one loss atomic
  const bool vec = lb ? (K % 8 == 0) : (K % 4 == 0);   // rows start 16-byte aligned when K is a multiple
  if (vec)
    softmax_xent_kernel<true><<<blocks, 256, 0, st>>>(lb, lf, labels, loss, db, df, B, K, label_base, grad_scale);
  else
    softmax_xent_kernel<false><<<blocks, 256, 0, st>>>(lb, lf, labels, loss, db, df, B, K, label_base, grad_scale);
  HIP_LAUNCH_CHECK();
}
void bigdl_sgd_step(float* w, const float* g, float* mom, uint16_t* w16, long n, const float* lr_dev, float lr,
                    float wd, float momentum, float dampening, int nesterov, int first, const long* seg_off,
                    const float* seg_wd, int nseg, long base, hipStream_t st) {
  const bool vec = (n & 3) == 0 && ((reinterpret_cast<uintptr_t>(w) | reinterpret_cast<uintptr_t>(g) |
                                      reinterpret_cast<uintptr_t>(mom)) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(w16) & 7) == 0;
  if (vec)
    sgd4_kernel<<<grid_cap(n / 4), 256, 0, st>>>(w, g, mom, w16, n / 4, lr_dev, lr, wd, momentum, dampening, nesterov,
                                                 first, seg_off, seg_wd, nseg, base);
  else
    sgd_kernel<<<grid_cap(n), 256, 0, st>>>(w, g, mom, w16, n, lr_dev, lr, wd, momentum, dampening, nesterov, first,
                                            seg_off, seg_wd, nseg, base);
  HIP_LAUNCH_CHECK();
}
void bigdl_adam_step(float* w, const float* g, float* m, float* v, uint16_t* w16, long n, float lr, float beta1,
                     float beta2, float eps, float wd, float bc1, float bc2, hipStream_t st) {
  adam_kernel<<<grid_cap(n), 256, 0, st>>>(w, g, m, v, w16, n, lr, beta1, beta2, eps, wd, bc1, bc2);
  HIP_LAUNCH_CHECK();
}
void bigdl_sumsq(const float* x, float* out, long n, hipStream_t st, float* det_ws) {
  if (bigdl_deterministic()) {   // fixed order: per-block partials into slots, then one ordered sum
    if (det_ws != nullptr) {
      sumsq_det_kernel<<<BIGDL_DET_SLOTS, 256, 0, st>>>(x, n, det_ws);
      sumsq_det_finish_kernel<<<1, 64, 0, st>>>(out, det_ws);
    } else {
      sumsq_kernel<<<1, 256, 0, st>>>(x, out, n);       // one block: one atomic
    }
    HIP_LAUNCH_CHECK();
    return;
  }
  sumsq_kernel<<<grid_cap(n, 2048), 256, 0, st>>>(x, out, n);
  HIP_LAUNCH_CHECK();
}
void bigdl_scale_f32(float* x, long n, const float* sdev, float s, hipStream_t st) {
  scale_kernel<<<grid_cap(n), 256, 0, st>>>(x, n, sdev, s);
  HIP_LAUNCH_CHECK();
}
void bigdl_lstm_cell_fwd(const float* gates, const float* c_prev, float* c, float* h, float* act, int B, int H,
                         hipStream_t st) {
  lstm_fwd_kernel<<<grid_cap((long)B * H), 256, 0, st>>>(gates, c_prev, c, h, act, B, H);
  HIP_LAUNCH_CHECK();
}
void bigdl_lstm_cell_bwd(const float* act, const float* c_prev, const float* c, const float* dh, const float* dc_next,
                         float* dgates, float* dc_prev, int B, int H, hipStream_t st) {
  lstm_bwd_kernel<<<grid_cap((long)B * H), 256, 0, st>>>(act, c_prev, c, dh, dc_next, dgates, dc_prev, B, H);
  HIP_LAUNCH_CHECK();
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Strided-conv data gradient: pixels of stride phases that no tap reaches (a 1x1 stride-2 conv covers one phase in
// four) get zeros, or the residual addend when one is folded in; the phase GEMMs write every other pixel. Replaces
// a full-tensor zero fill / addend copy ahead of the GEMMs (ops/conv.py conv2d_dgrad). NHWC bf16, C % 8 == 0, one
// lane per 8-channel granule, 16-byte loads / stores; `mask` bit ph set = phase ph = (h % sh) * sw + (w % sw) covered.
namespace {
__global__ __launch_bounds__(256) void dgrad_fill_kernel(uint16_t* __restrict__ out, const uint16_t* __restrict__ add,
                                                         long npix, int H, int W, int C8, int sh, int sw,
                                                         unsigned mask) {
  const long total = npix * C8;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long pix = e / C8;
    const int w = (int)(pix % W), h = (int)((pix / W) % H);
    const int ph = (h % sh) * sw + (w % sw);
    if ((mask >> ph) & 1u) continue;
    v4u v = v4u{0u, 0u, 0u, 0u};
    if (add) v = reinterpret_cast<const v4u*>(add)[e];
    reinterpret_cast<v4u*>(out)[e] = v;
  }
}
}  // namespace

namespace {
// Byte fill as a kernel: work captured into a HIP graph must not contain memset nodes — with the one-queue graph
// executor (bigdl_amd/__init__.py) a captured hipMemsetAsync was not ordered with the kernels around it (training
// diverged after a graph trial, tools/_bisect.sh: profiles/r4_memset_node_bisect.txt)
__global__ __launch_bounds__(256) void fill_bytes_kernel(uint8_t* __restrict__ p, unsigned v4, long n16, long bytes) {
  const long stride = (long)gridDim.x * 256;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n16; i += stride)
    reinterpret_cast<v4u*>(p)[i] = v4u{v4, v4, v4, v4};
  for (long b = n16 * 16 + blockIdx.x * 256L + threadIdx.x; b < bytes; b += stride) p[b] = (uint8_t)(v4 & 0xff);
}
}  // namespace

void bigdl_fill_bytes(void* ptr, int value, long bytes, hipStream_t st) {
  if (bytes <= 0) return;
  const unsigned v = (unsigned)(value & 0xff), v4 = v | (v << 8) | (v << 16) | (v << 24);
  const bool al = (reinterpret_cast<uintptr_t>(ptr) & 15) == 0;
  const long n16 = al ? bytes / 16 : 0;
  long g = ((al ? n16 : bytes) + 255) / 256;
  g = g < 1 ? 1 : (g > 4096 ? 4096 : g);
  fill_bytes_kernel<<<(unsigned)g, 256, 0, st>>>(static_cast<uint8_t*>(ptr), v4, n16, bytes);
  HIP_LAUNCH_CHECK();
}

void bigdl_dgrad_fill(uint16_t* out, const uint16_t* add, long npix, int H, int W, int C, int sh, int sw, unsigned mask,
                      hipStream_t st) {
  const long total = npix * (C / 8);
  if (total <= 0) return;
  long g = (total + 255) / 256;
  if (g > 16384) g = 16384;
  dgrad_fill_kernel<<<(unsigned)g, 256, 0, st>>>(out, add, npix, H, W, C / 8, sh, sw, mask);
  HIP_LAUNCH_CHECK();
}
