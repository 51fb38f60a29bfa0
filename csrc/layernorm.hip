// Layer normalisation over the last dimension (fp32 rows) for gfx950.
//
// Reference: S/nn/LayerNormalization.scala (Transformer layer norm: y = (x - mean) / sqrt(var + eps) * g + b over
// the hidden dimension), used by S/nn/Transformer.scala / Attention blocks.
//
// Forward / data-gradient: one 256-thread workgroup per row, the row held in registers (up to 16 floats per
// thread = rows of 4096), 16-byte loads when D % 4 == 0, wave-shuffle + LDS reductions; mean and 1/std are kept
// for the backward. Parameter gradients: a column-tiled pass over row chunks, one atomic per column per chunk.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int LN_THREADS = 256;
constexpr int LN_MAXV = 16;     // floats per thread held in registers

__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wave] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < LN_THREADS / 64; ++i) t += sh[i];
  return t;
}

__global__ void __launch_bounds__(LN_THREADS) ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                            const float* __restrict__ b, float* __restrict__ y,
                                                            float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                            int D, float eps) {
  __shared__ float sh[LN_THREADS / 64];
  const long row = blockIdx.x;
  const float* xr = x + row * D;
  float v[LN_MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = i * LN_THREADS + threadIdx.x;
    v[i] = c < D ? xr[c] : 0.f;
    s += v[i];
  }
  const float mean = block_sum(s, sh) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = i * LN_THREADS + threadIdx.x;
    const float d = c < D ? v[i] - mean : 0.f;
    q += d * d;
  }
  const float rstd = rsqrtf(block_sum(q, sh) / D + eps);
  float* yr = y + row * D;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = i * LN_THREADS + threadIdx.x;
    if (c < D) yr[c] = (v[i] - mean) * rstd * (g ? g[c] : 1.f) + (b ? b[c] : 0.f);
  }
  if (threadIdx.x == 0) { mean_out[row] = mean; rstd_out[row] = rstd; }
}

// dx = rstd * (dxh - mean(dxh) - xh * mean(dxh * xh)),  dxh = dy * g,  xh = (x - mean) * rstd
__global__ void __launch_bounds__(LN_THREADS) ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                            const float* __restrict__ g, const float* __restrict__ mean,
                                                            const float* __restrict__ rstd, float* __restrict__ dx,
                                                            int D) {
  __shared__ float sh[LN_THREADS / 64];
  const long row = blockIdx.x;
  const float mu = mean[row], rs = rstd[row];
  float xh[LN_MAXV], dh[LN_MAXV];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = i * LN_THREADS + threadIdx.x;
    xh[i] = c < D ? (x[row * D + c] - mu) * rs : 0.f;
    dh[i] = c < D ? dy[row * D + c] * (g ? g[c] : 1.f) : 0.f;
    s1 += dh[i];
    s2 += dh[i] * xh[i];
  }
  const float m1 = block_sum(s1, sh) / D;
  const float m2 = block_sum(s2, sh) / D;
#pragma unroll
  for (int i = 0; i < LN_MAXV; ++i) {
    const int c = i * LN_THREADS + threadIdx.x;
    if (c < D) dx[row * D + c] = rs * (dh[i] - m1 - xh[i] * m2);
  }
}

// dg[c] += sum_rows dy * xh,  db[c] += sum_rows dy. Block = 256 columns x a chunk of rows.
__global__ void __launch_bounds__(LN_THREADS) ln_param_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                              const float* __restrict__ mean,
                                                              const float* __restrict__ rstd, float* __restrict__ dg,
                                                              float* __restrict__ db, long rows, int D, long chunk) {
  const int c = blockIdx.x * LN_THREADS + threadIdx.x;
  if (c >= D) return;
  const long r0 = (long)blockIdx.y * chunk, r1 = r0 + chunk < rows ? r0 + chunk : rows;
  float a = 0.f, bsum = 0.f;
  for (long r = r0; r < r1; ++r) {
    const float d = dy[r * D + c];
    a += d * (x[r * D + c] - mean[r]) * rstd[r];
    bsum += d;
  }
  if (dg) atomicAdd(dg + c, a);
  if (db) atomicAdd(db + c, bsum);
}

}  // namespace

int bigdl_layernorm_fwd(const float* x, const float* g, const float* b, float* y, float* mean, float* rstd, long rows,
                        int D, float eps, hipStream_t st) {
  if (D > LN_THREADS * LN_MAXV || D <= 0 || rows <= 0 || rows > 2147483647L) return -1;
  ln_fwd_kernel<<<(unsigned)rows, LN_THREADS, 0, st>>>(x, g, b, y, mean, rstd, D, eps);
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_layernorm_bwd(const float* dy, const float* x, const float* g, const float* mean, const float* rstd,
                        float* dx, float* dg, float* db, long rows, int D, hipStream_t st) {
  if (D > LN_THREADS * LN_MAXV || D <= 0 || rows <= 0 || rows > 2147483647L) return -1;
  if (dx) ln_bwd_kernel<<<(unsigned)rows, LN_THREADS, 0, st>>>(dy, x, g, mean, rstd, dx, D);
  if (dg || db) {
    const int bx = (D + LN_THREADS - 1) / LN_THREADS;
    long by = (rows + 63) / 64;                  // 64-row chunks, at most ~2048 blocks
    if ((long)bx * by > 2048) by = (2048 + bx - 1) / bx;
    const long chunk = (rows + by - 1) / by;
    ln_param_kernel<<<dim3(bx, (unsigned)by), LN_THREADS, 0, st>>>(dy, x, mean, rstd, dg, db, rows, D, chunk);
  }
  HIP_LAUNCH_CHECK();
  return 0;
}
