// Memory-bound NN kernels outside the conv/BN hot path, for gfx950.
//
// Reference counterparts:
//   LRN across channels   S/nn/SpatialCrossMapLRN.scala:43 (fwd), :117 (bwd)        
//   Dropout               S/nn/Dropout.scala:44, RNG S/utils/RandomGenerator.scala  
//   LookupTable           S/nn/LookupTable.scala:47 (gather), accGradParameters      
//   ResizeBilinear        S/nn/ResizeBilinear.scala:35 (TF legacy / align_corners)   
//   LogSoftMax            S/nn/LogSoftMax.scala:49-171                               
//   bf16 truncation       S/parameters/FP16CompressedTensor.scala:271-279           
//
// Design notes (MI355X):
// * LRN: one lane per (n, pixel) column walks the channels with a running window sum, so every
//   channel step is one coalesced 256-B row read per wave and the x^2 window never leaves registers.
// * Dropout: counter-based Philox-4x32-10 keyed by (seed, element/4) -> the backward regenerates the
//   keep-mask instead of storing it (no mask tensor in HBM), and results do not depend on the grid.
// * Embedding: a wave per output row, 16-byte lanes; the backward scatter uses fp32 atomics straight
//   into the gradient table (rows collide rarely for vocab-sized tables; MI355X_MICROARCH global atomics).
// * Row softmax: one wave per row, 4-wide vector loads, wave-shuffle max/sum reductions (no LDS).
#include "common.h"
#include "kernels.h"

namespace {

#define GS_LOOP(i, n) for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (n); i += (long)gridDim.x * blockDim.x)

inline int blocks_for(long work, int threads = 256, int cap = 16384) {
  long g = (work + threads - 1) / threads;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

// ------------------------------------------------------------------------------------------ LRN
__global__ void lrn_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, float* __restrict__ scale, int N,
                               int C, long HW, int size, float alpha_n, float beta, float k) {
  const long cols = (long)N * HW;
  const int pre = (size - 1) / 2;
  GS_LOOP(col, cols) {
    const long n = col / HW, p = col - n * HW;
    const float* xc = x + n * C * HW + p;
    float* yc = y + n * C * HW + p;
    float* sc = scale + n * C * HW + p;
    float win = 0.f;
    // window for channel c covers [c - pre, c - pre + size - 1]
    for (int c = 0; c < size - pre - 1 && c < C; ++c) { const float v = xc[(long)c * HW]; win += v * v; }
    for (int c = 0; c < C; ++c) {
      const int add = c + size - pre - 1, sub = c - pre - 1;
      if (add < C) { const float v = xc[(long)add * HW]; win += v * v; }
      if (sub >= 0) { const float v = xc[(long)sub * HW]; win -= v * v; }
      const float s = k + alpha_n * fmaxf(win, 0.f);
      sc[(long)c * HW] = s;
      yc[(long)c * HW] = xc[(long)c * HW] * __powf(s, -beta);
    }
  }
}

// gx = gy * s^-beta - (2 alpha beta / size) * x * sum_{window'} (gy * y / s)
__global__ void lrn_bwd_kernel(const float* __restrict__ x, const float* __restrict__ y, const float* __restrict__ scale,
                               const float* __restrict__ gy, float* __restrict__ gx, int N, int C, long HW, int size,
                               float alpha_n, float beta) {
  const long cols = (long)N * HW;
  const int pre = (size - 1) / 2;
  const float coef = 2.f * alpha_n * beta;
  GS_LOOP(col, cols) {
    const long base = (col / HW) * C * HW + (col % HW);
    float win = 0.f;
    // the gradient window of channel c is the set of outputs whose forward window contains c:
    // outputs j with j - pre <= c <= j - pre + size - 1  ->  j in [c + pre - size + 1, c + pre]
    auto ratio = [&](int j) { const long o = base + (long)j * HW; return gy[o] * y[o] / scale[o]; };
    for (int j = 0; j <= pre - 1 && j < C; ++j) win += ratio(j);
    for (int c = 0; c < C; ++c) {
      const int add = c + pre, sub = c + pre - size;
      if (add < C) win += ratio(add);
      if (sub >= 0) win -= ratio(sub);
      const long o = base + (long)c * HW;
      gx[o] = gy[o] * __powf(scale[o], -beta) - coef * x[o] * win;
    }
  }
}

// ------------------------------------------------------------------------------------------ Philox dropout
struct U4 { unsigned x, y, z, w; };
__device__ __forceinline__ U4 philox(unsigned long long seed, unsigned long long ctr) {
  unsigned c0 = (unsigned)ctr, c1 = (unsigned)(ctr >> 32), c2 = 0, c3 = 0;
  unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    const unsigned n0 = (unsigned)(p1 >> 32) ^ c1 ^ k0, n2 = (unsigned)(p0 >> 32) ^ c3 ^ k1;
    c1 = (unsigned)p1; c3 = (unsigned)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}
__device__ __forceinline__ float u01(unsigned v) { return (v >> 8) * (1.0f / 16777216.0f); }

// y = x * keep / (1-p) (or x * keep when !scale); mask never stored: bwd calls the same kernel on dy.
template <typename T>
__global__ void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long n, float p, float mul,
                               unsigned long long seed) {
  const long n4 = (n + 3) >> 2;
  GS_LOOP(q, n4) {
    const U4 r = philox(seed, (unsigned long long)q);
    const unsigned rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long i = q * 4 + e;
      if (i < n) {
        const bool keep = u01(rr[e]) >= p;
        if constexpr (sizeof(T) == 4) {
          y[i] = keep ? x[i] * mul : 0.f;
        } else {
          y[i] = keep ? f2bf(bf2f(x[i]) * mul) : (bf16_t)0;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------ embedding
// out[r, :] = W[idx[r], :] (idx < 0 -> paddingValue row of zeros)
__global__ void embedding_fwd_kernel(const float* __restrict__ W, const long* __restrict__ idx, float* __restrict__ out,
                                     long rows, int D, long nIndex) {
  const int lane = threadIdx.x & 63;
  const long wid = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wid; r < rows; r += nw) {
    const long k = idx[r];
    float* o = out + r * D;
    if (k < 0 || k >= nIndex) {
      for (int d = lane; d < D; d += 64) o[d] = 0.f;
      continue;
    }
    const float* w = W + k * D;
    if ((D & 3) == 0) {
      const float4* w4 = (const float4*)w;
      float4* o4 = (float4*)o;
      for (int d = lane; d < (D >> 2); d += 64) o4[d] = w4[d];
    } else {
      for (int d = lane; d < D; d += 64) o[d] = w[d];
    }
  }
}

__global__ void embedding_bwd_kernel(const float* __restrict__ gout, const long* __restrict__ idx,
                                     float* __restrict__ gW, long rows, int D, long nIndex, float scale) {
  const int lane = threadIdx.x & 63;
  const long wid = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wid; r < rows; r += nw) {
    const long k = idx[r];
    if (k < 0 || k >= nIndex) continue;
    const float* g = gout + r * D;
    float* w = gW + k * D;
    for (int d = lane; d < D; d += 64) atomicAdd(w + d, g[d] * scale);
  }
}

// Same gather / scatter-add from the layer's raw 1-based ids (float or int64: LookupTable input), so no index tensor
// is ever materialised: k = id - 1; forward: k < 0 -> zero row if mask_zero else row 0 (the reference's clamp);
// backward: rows with k < 0 or k == pad are skipped; the output gradient is f32 or bf16 (GB: bf16).
template <typename ID>
__device__ __forceinline__ long emb_id(const ID* ids, long r) { return (long)ids[r] - 1; }

template <typename ID>
__global__ void embedding_fwd_ids_kernel(const float* __restrict__ W, const ID* __restrict__ ids, float* __restrict__ out,
                                         long rows, int D, long nIndex, int mask_zero) {
  const int lane = threadIdx.x & 63;
  const long wid = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wid; r < rows; r += nw) {
    long k = emb_id(ids, r);
    if (k < 0 && !mask_zero) k = 0;
    float* o = out + r * D;
    if (k < 0 || k >= nIndex) {
      for (int d = lane; d < D; d += 64) o[d] = 0.f;
      continue;
    }
    const float* w = W + k * D;
    if ((D & 3) == 0) {
      for (int d = lane; d < (D >> 2); d += 64) reinterpret_cast<float4*>(o)[d] = reinterpret_cast<const float4*>(w)[d];
    } else {
      for (int d = lane; d < D; d += 64) o[d] = w[d];
    }
  }
}

template <typename ID, bool GB>
__global__ void embedding_bwd_ids_kernel(const void* __restrict__ gout, const ID* __restrict__ ids,
                                         float* __restrict__ gW, long rows, int D, long nIndex, long pad, float scale) {
  const int lane = threadIdx.x & 63;
  const long wid = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wid; r < rows; r += nw) {
    const long k = emb_id(ids, r);
    if (k < 0 || k >= nIndex || k == pad) continue;
    float* w = gW + k * D;
    if (GB) {
      const bf16_t* g = static_cast<const bf16_t*>(gout) + r * D;
      for (int d = lane; d < D; d += 64) atomicAdd(w + d, __uint_as_float((unsigned)g[d] << 16) * scale);
    } else {
      const float* g = static_cast<const float*>(gout) + r * D;
      for (int d = lane; d < D; d += 64) atomicAdd(w + d, g[d] * scale);
    }
  }
}

// ------------------------------------------------------------------------------------------ bilinear resize (NCHW)
// TF legacy mapping src = dst * scale, scale = in/out (align_corners: (in-1)/(out-1)), clamped at the edge.
__device__ __forceinline__ void bil_src(int o, int in, float scale, int& i0, int& i1, float& f) {
  const float s = o * scale;
  i0 = (int)floorf(s);
  i0 = i0 < in - 1 ? i0 : in - 1;
  i1 = i0 + 1 < in ? i0 + 1 : in - 1;
  f = s - i0;
}

__global__ void resize_bilinear_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, long NC, int H, int W,
                                           int OH, int OW, float sh, float sw) {
  const long total = NC * OH * OW;
  GS_LOOP(i, total) {
    const int ow = i % OW;
    const long t = i / OW;
    const int oh = t % OH;
    const long nc = t / OH;
    int h0, h1, w0, w1;
    float fh, fw;
    bil_src(oh, H, sh, h0, h1, fh);
    bil_src(ow, W, sw, w0, w1, fw);
    const float* p = x + nc * H * W;
    const float top = p[h0 * W + w0] + (p[h0 * W + w1] - p[h0 * W + w0]) * fw;
    const float bot = p[h1 * W + w0] + (p[h1 * W + w1] - p[h1 * W + w0]) * fw;
    y[i] = top + (bot - top) * fh;
  }
}

__global__ void resize_bilinear_bwd_kernel(const float* __restrict__ gy, float* __restrict__ gx, long NC, int H, int W,
                                           int OH, int OW, float sh, float sw) {
  const long total = NC * OH * OW;
  GS_LOOP(i, total) {
    const int ow = i % OW;
    const long t = i / OW;
    const int oh = t % OH;
    const long nc = t / OH;
    int h0, h1, w0, w1;
    float fh, fw;
    bil_src(oh, H, sh, h0, h1, fh);
    bil_src(ow, W, sw, w0, w1, fw);
    float* p = gx + nc * H * W;
    const float g = gy[i];
    atomicAdd(p + h0 * W + w0, g * (1.f - fh) * (1.f - fw));
    atomicAdd(p + h0 * W + w1, g * (1.f - fh) * fw);
    atomicAdd(p + h1 * W + w0, g * fh * (1.f - fw));
    atomicAdd(p + h1 * W + w1, g * fh * fw);
  }
}

// ------------------------------------------------------------------------------------------ log-softmax rows
__global__ void log_softmax_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, long rows, int cols) {
  const int lane = threadIdx.x & 63;
  const long wid = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wid; r < rows; r += nw) {
    const float* xr = x + r * cols;
    float m = -INFINITY;
    for (int c = lane; c < cols; c += 64) m = fmaxf(m, xr[c]);
    m = wave_max(m);
    float s = 0.f;
    for (int c = lane; c < cols; c += 64) s += __expf(xr[c] - m);
    s = wave_sum(s);
    const float lse = m + __logf(s);
    float* yr = y + r * cols;
    for (int c = lane; c < cols; c += 64) yr[c] = xr[c] - lse;
  }
}

// gx = gy - exp(y) * sum(gy)
__global__ void log_softmax_bwd_kernel(const float* __restrict__ y, const float* __restrict__ gy, float* __restrict__ gx,
                                       long rows, int cols) {
  const int lane = threadIdx.x & 63;
  const long wid = (blockIdx.x * (long)blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long r = wid; r < rows; r += nw) {
    const float* g = gy + r * cols;
    float s = 0.f;
    for (int c = lane; c < cols; c += 64) s += g[c];
    s = wave_sum(s);
    const float* yr = y + r * cols;
    float* o = gx + r * cols;
    for (int c = lane; c < cols; c += 64) o[c] = g[c] - __expf(yr[c]) * s;
  }
}

// ------------------------------------------------------------------------------------------ bf16 truncation
// FP16CompressedTensor parity: fp32 -> bf16 by dropping the low 16 bits (round toward zero), 16 B per lane.
__global__ void f32_to_bf16_rtz_kernel(const v4u* __restrict__ x, v2u* __restrict__ y, long n4) {
  GS_LOOP(i, n4) {
    const v4u v = x[i];
    v2u o;
    o[0] = (v[0] >> 16) | (v[1] & 0xffff0000u);
    o[1] = (v[2] >> 16) | (v[3] & 0xffff0000u);
    y[i] = o;
  }
}
__global__ void f32_to_bf16_rtz_tail(const unsigned* x, uint16_t* y, long s, long n) {
  GS_LOOP(i, n - s) y[s + i] = (uint16_t)(x[s + i] >> 16);
}

}  // namespace

// ============================================================================================ C ABI
void bigdl_lrn_fwd(const float* x, float* y, float* scale, int N, int C, long HW, int size, float alpha, float beta,
                   float k, hipStream_t st) {
  const long cols = (long)N * HW;
  lrn_fwd_kernel<<<blocks_for(cols), 256, 0, st>>>(x, y, scale, N, C, HW, size, alpha / size, beta, k);
  HIP_LAUNCH_CHECK();
}
void bigdl_lrn_bwd(const float* x, const float* y, const float* scale, const float* gy, float* gx, int N, int C, long HW,
                   int size, float alpha, float beta, hipStream_t st) {
  const long cols = (long)N * HW;
  lrn_bwd_kernel<<<blocks_for(cols), 256, 0, st>>>(x, y, scale, gy, gx, N, C, HW, size, alpha / size, beta);
  HIP_LAUNCH_CHECK();
}
void bigdl_dropout(const void* x, void* y, int is_bf16, long n, float p, float mul, unsigned long long seed,
                   hipStream_t st) {
  const long n4 = (n + 3) >> 2;
  if (is_bf16)
    dropout_kernel<bf16_t><<<blocks_for(n4), 256, 0, st>>>((const bf16_t*)x, (bf16_t*)y, n, p, mul, seed);
  else
    dropout_kernel<float><<<blocks_for(n4), 256, 0, st>>>((const float*)x, (float*)y, n, p, mul, seed);
  HIP_LAUNCH_CHECK();
}
void bigdl_embedding_fwd(const float* W, const long* idx, float* out, long rows, int D, long nIndex, hipStream_t st) {
  embedding_fwd_kernel<<<blocks_for(rows * 64), 256, 0, st>>>(W, idx, out, rows, D, nIndex);
  HIP_LAUNCH_CHECK();
}
void bigdl_embedding_fwd_ids(const float* W, const void* ids, int ids_long, float* out, long rows, int D, long nIndex,
                             int mask_zero, hipStream_t st) {
  if (ids_long)
    embedding_fwd_ids_kernel<long><<<blocks_for(rows * 64), 256, 0, st>>>(W, (const long*)ids, out, rows, D, nIndex,
                                                                          mask_zero);
  else
    embedding_fwd_ids_kernel<float><<<blocks_for(rows * 64), 256, 0, st>>>(W, (const float*)ids, out, rows, D, nIndex,
                                                                           mask_zero);
  HIP_LAUNCH_CHECK();
}
void bigdl_embedding_bwd_ids(const void* gout, int gout_bf16, const void* ids, int ids_long, float* gW, long rows, int D,
                             long nIndex, long pad, float scale, hipStream_t st) {
  const int g = blocks_for(rows * 64);
  if (ids_long) {
    if (gout_bf16) embedding_bwd_ids_kernel<long, true><<<g, 256, 0, st>>>(gout, (const long*)ids, gW, rows, D, nIndex, pad, scale);
    else embedding_bwd_ids_kernel<long, false><<<g, 256, 0, st>>>(gout, (const long*)ids, gW, rows, D, nIndex, pad, scale);
  } else {
    if (gout_bf16) embedding_bwd_ids_kernel<float, true><<<g, 256, 0, st>>>(gout, (const float*)ids, gW, rows, D, nIndex, pad, scale);
    else embedding_bwd_ids_kernel<float, false><<<g, 256, 0, st>>>(gout, (const float*)ids, gW, rows, D, nIndex, pad, scale);
  }
  HIP_LAUNCH_CHECK();
}
void bigdl_embedding_bwd(const float* gout, const long* idx, float* gW, long rows, int D, long nIndex, float scale,
                         hipStream_t st) {
  embedding_bwd_kernel<<<blocks_for(rows * 64), 256, 0, st>>>(gout, idx, gW, rows, D, nIndex, scale);
  HIP_LAUNCH_CHECK();
}
void bigdl_resize_bilinear_fwd(const float* x, float* y, long NC, int H, int W, int OH, int OW, float sh, float sw,
                               hipStream_t st) {
  resize_bilinear_fwd_kernel<<<blocks_for(NC * OH * OW), 256, 0, st>>>(x, y, NC, H, W, OH, OW, sh, sw);
  HIP_LAUNCH_CHECK();
}
void bigdl_resize_bilinear_bwd(const float* gy, float* gx, long NC, int H, int W, int OH, int OW, float sh, float sw,
                               hipStream_t st) {
  resize_bilinear_bwd_kernel<<<blocks_for(NC * OH * OW), 256, 0, st>>>(gy, gx, NC, H, W, OH, OW, sh, sw);
  HIP_LAUNCH_CHECK();
}
void bigdl_log_softmax_fwd(const float* x, float* y, long rows, int cols, hipStream_t st) {
  log_softmax_fwd_kernel<<<blocks_for(rows * 64), 256, 0, st>>>(x, y, rows, cols);
  HIP_LAUNCH_CHECK();
}
void bigdl_log_softmax_bwd(const float* y, const float* gy, float* gx, long rows, int cols, hipStream_t st) {
  log_softmax_bwd_kernel<<<blocks_for(rows * 64), 256, 0, st>>>(y, gy, gx, rows, cols);
  HIP_LAUNCH_CHECK();
}
void bigdl_f32_to_bf16_rtz(const float* x, uint16_t* y, long n, hipStream_t st) {
  const long n4 = n >> 2;
  if (n4) f32_to_bf16_rtz_kernel<<<blocks_for(n4), 256, 0, st>>>((const v4u*)x, (v2u*)y, n4);
  if (n4 * 4 < n) f32_to_bf16_rtz_tail<<<1, 64, 0, st>>>((const unsigned*)x, y, n4 * 4, n);
  HIP_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------------
// Device-side delay: one wave spins on the constant-rate real-time counter (s_memrealtime, 100 MHz on gfx950) for
// `us` microseconds, capped at 5 s so a bad argument cannot hang the queue. Injects a compute straggler for the
// straggler-drop tests (optim/optimizer.py _StragglerDrop) without touching the host.
namespace {
__global__ __launch_bounds__(64) void spin_us_kernel(long ticks, int* done) {
  const unsigned long t0 = wall_clock64();
  while ((long)(wall_clock64() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0) done[0] = 1;
}
// CU hog: a one-wave workgroup that declares the whole 160 KiB LDS (one per CU) and spins, so no other workgroup with
// LDS can be co-resident on that CU meanwhile. Tests use it to take CUs away from a persistent launch on another
// stream (csrc/lstm_seq.hip residency / timeout tests). Capped at 5 s.
__global__ __launch_bounds__(64) void hog_cu_kernel(long ticks, int* done) {
  __shared__ int pad[160 * 1024 / 4];
  pad[threadIdx.x * 640] = threadIdx.x;
  const unsigned long t0 = wall_clock64();
  while ((long)(wall_clock64() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (threadIdx.x == 0) done[blockIdx.x] = pad[(threadIdx.x + 1) * 640 % 40960] + 1;
}
}  // namespace

void bigdl_hog_cus(int n, double us, int* done, hipStream_t st) {
  double t = us < 0 ? 0 : (us > 5e6 ? 5e6 : us);
  if (n < 1) return;
  hog_cu_kernel<<<n, 64, 0, st>>>((long)(t * 100.0), done);
  HIP_LAUNCH_CHECK();
}

void bigdl_spin_us(double us, int* done, hipStream_t st) {
  double t = us < 0 ? 0 : (us > 5e6 ? 5e6 : us);
  spin_us_kernel<<<1, 64, 0, st>>>((long)(t * 100.0), done);   // wall_clock64 ticks at 100 MHz
  HIP_LAUNCH_CHECK();
}
