// Generic N-d (1D / 2D / 3D) window pooling and nearest-neighbour up-sampling for gfx950, forward and backward.
//
// Reference: S/nn/VolumetricMaxPooling.scala, VolumetricAveragePooling.scala, TemporalMaxPooling.scala (window
// loops of NNPrimitive.scala:654-1051 extended to a depth axis), S/nn/UpSampling1D.scala, UpSampling2D.scala,
// UpSampling3D.scala (the long-tail pooling and resize layers that the 2D NHWC kernels of
// elementwise.hip do not cover).
//
// Every layout is seen as a dense [B][D][H][W][C] array with C innermost: an NCDHW / NCHW tensor is B = N*C, C = 1
// (W innermost), a (batch, frames, features) sequence is B = N, D = H = 1, W = frames, C = features, a channels-last
// tensor is B = N with its real C. One thread owns one output (forward) or one input (backward) element, so
// consecutive lanes walk the innermost axis and every access is coalesced; the backward passes are gathers over the
// windows that cover the element (no atomics, deterministic sums, overlapping windows accumulate correctly).
// fp32 math for bf16 tensors; max pooling stores the winning input position (d*H + h)*W + w as int32.
#include "common.h"
#include "kernels.h"

namespace {

__device__ __forceinline__ float ldf(const float* p, long i) { return p[i]; }
__device__ __forceinline__ float ldf(const bf16_t* p, long i) { return bf2f(p[i]); }
__device__ __forceinline__ void stf(float* p, long i, float v) { p[i] = v; }
__device__ __forceinline__ void stf(bf16_t* p, long i, float v) { p[i] = f2bf(v); }

// window [lo, hi) of axis `o` clipped to the input, plus the unclipped (pad-bounded) extent for count_include_pad
struct Win { int lo, hi, full; };
__device__ __forceinline__ Win win(int o, int s, int p, int k, int n) {
  int lo = o * s - p;
  int hi = min(lo + k, n + p);
  const int full = hi - lo;
  lo = max(lo, 0);
  hi = min(hi, n);
  return {lo, hi, full};
}

// output range of axis o whose windows cover input position i: [olo, ohi]
__device__ __forceinline__ void cover(int i, int s, int p, int k, int on, int& olo, int& ohi) {
  const int t = i + p;
  olo = t < k ? 0 : (t - k) / s + 1;
  ohi = min(t / s, on - 1);
}

template <typename T, bool MAX>
__global__ __launch_bounds__(256) void poolnd_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                         int* __restrict__ idx, PoolNdGeo g, int count_pad) {
  const long total = (long)g.B * g.OD * g.OH * g.OW * g.C;
  for (long e = blockIdx.x * 256l + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    long r = e;
    const int c = r % g.C; r /= g.C;
    const int ow = r % g.OW; r /= g.OW;
    const int oh = r % g.OH; r /= g.OH;
    const int od = r % g.OD;
    const long b = r / g.OD;
    const Win wd = win(od, g.sd, g.pd, g.kd, g.D), wh = win(oh, g.sh, g.ph, g.kh, g.H),
              ww = win(ow, g.sw, g.pw, g.kw, g.W);
    const long base = b * g.D * g.H * g.W;
    float acc = MAX ? -INFINITY : 0.f;
    int arg = -1;
    for (int d = wd.lo; d < wd.hi; ++d)
      for (int h = wh.lo; h < wh.hi; ++h)
        for (int w = ww.lo; w < ww.hi; ++w) {
          const int pos = (d * g.H + h) * g.W + w;
          const float v = ldf(x, (base + pos) * g.C + c);
          if (MAX) {
            if (v > acc || arg < 0 || v != v) { acc = v; arg = pos; }   // NaN propagates, like the reference max
          } else {
            acc += v;
          }
        }
    if (MAX) {
      if (idx) idx[e] = arg;
      if (arg < 0) acc = 0.f;
    } else {
      const int cnt = count_pad ? wd.full * wh.full * ww.full
                                : (wd.hi - wd.lo) * (wh.hi - wh.lo) * (ww.hi - ww.lo);
      acc = cnt > 0 ? acc / (float)cnt : 0.f;
    }
    stf(y, e, acc);
  }
}

template <typename T, bool MAX>
__global__ __launch_bounds__(256) void poolnd_bwd_kernel(const T* __restrict__ dy, const int* __restrict__ idx,
                                                         T* __restrict__ dx, PoolNdGeo g, int count_pad) {
  const long total = (long)g.B * g.D * g.H * g.W * g.C;
  for (long e = blockIdx.x * 256l + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    long r = e;
    const int c = r % g.C; r /= g.C;
    const int w = r % g.W; r /= g.W;
    const int h = r % g.H; r /= g.H;
    const int d = r % g.D;
    const long b = r / g.D;
    const int pos = (d * g.H + h) * g.W + w;
    int d0, d1, h0, h1, w0, w1;
    cover(d, g.sd, g.pd, g.kd, g.OD, d0, d1);
    cover(h, g.sh, g.ph, g.kh, g.OH, h0, h1);
    cover(w, g.sw, g.pw, g.kw, g.OW, w0, w1);
    const long obase = b * g.OD * g.OH * g.OW;
    float acc = 0.f;
    for (int od = d0; od <= d1; ++od)
      for (int oh = h0; oh <= h1; ++oh)
        for (int ow = w0; ow <= w1; ++ow) {
          const long o = (obase + ((long)od * g.OH + oh) * g.OW + ow) * g.C + c;
          if (MAX) {
            if (idx[o] == pos) acc += ldf(dy, o);
          } else {
            const Win wd = win(od, g.sd, g.pd, g.kd, g.D), wh = win(oh, g.sh, g.ph, g.kh, g.H),
                      ww = win(ow, g.sw, g.pw, g.kw, g.W);
            const int cnt = count_pad ? wd.full * wh.full * ww.full
                                      : (wd.hi - wd.lo) * (wh.hi - wh.lo) * (ww.hi - ww.lo);
            if (cnt > 0) acc += ldf(dy, o) / (float)cnt;
          }
        }
    stf(dx, e, acc);
  }
}

// nearest up-sampling by integer factors (kd, kh, kw): y[b][d][h][w][c] = x[b][d/kd][h/kh][w/kw][c]
template <typename T>
__global__ __launch_bounds__(256) void upsample_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, PoolNdGeo g) {
  const long total = (long)g.B * g.OD * g.OH * g.OW * g.C;
  for (long e = blockIdx.x * 256l + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    long r = e;
    const int c = r % g.C; r /= g.C;
    const int ow = r % g.OW; r /= g.OW;
    const int oh = r % g.OH; r /= g.OH;
    const int od = r % g.OD;
    const long b = r / g.OD;
    const long src = (((b * g.D + od / g.kd) * g.H + oh / g.kh) * g.W + ow / g.kw) * g.C + c;
    y[e] = x[src];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void upsample_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx, PoolNdGeo g) {
  const long total = (long)g.B * g.D * g.H * g.W * g.C;
  for (long e = blockIdx.x * 256l + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    long r = e;
    const int c = r % g.C; r /= g.C;
    const int w = r % g.W; r /= g.W;
    const int h = r % g.H; r /= g.H;
    const int d = r % g.D;
    const long b = r / g.D;
    float acc = 0.f;
    for (int i = 0; i < g.kd; ++i)
      for (int j = 0; j < g.kh; ++j) {
        const long row = ((b * g.OD + (long)d * g.kd + i) * g.OH + (long)h * g.kh + j) * g.OW + (long)w * g.kw;
        for (int k = 0; k < g.kw; ++k) acc += ldf(dy, (row + k) * g.C + c);
      }
    stf(dx, e, acc);
  }
}

int grid_for(long total) {
  const long b = (total + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

bool geo_ok(const PoolNdGeo& g, bool pool) {
  if (g.B < 0 || g.C < 1 || g.D < 1 || g.H < 1 || g.W < 1 || g.OD < 1 || g.OH < 1 || g.OW < 1) return false;
  if (g.kd < 1 || g.kh < 1 || g.kw < 1) return false;
  if (!pool) return g.OD == g.D * g.kd && g.OH == g.H * g.kh && g.OW == g.W * g.kw;
  if (g.sd < 1 || g.sh < 1 || g.sw < 1 || g.pd < 0 || g.ph < 0 || g.pw < 0) return false;
  // every output window starts inside input + padding (what the reference's ceil-mode rule guarantees)
  return (g.OD - 1) * g.sd < g.D + g.pd && (g.OH - 1) * g.sh < g.H + g.ph && (g.OW - 1) * g.sw < g.W + g.pw;
}

}  // namespace

extern "C" {

int bigdl_poolnd_fwd(const void* x, void* y, int* idx, const PoolNdGeo* g, int max_mode, int count_pad, int bf16,
                     hipStream_t st) {
  if (!geo_ok(*g, true)) return -1;
  const long total = (long)g->B * g->OD * g->OH * g->OW * g->C;
  if (total == 0) return 0;
  const int grid = grid_for(total);
  if (bf16) {
    if (max_mode) poolnd_fwd_kernel<bf16_t, true><<<grid, 256, 0, st>>>((const bf16_t*)x, (bf16_t*)y, idx, *g, count_pad);
    else poolnd_fwd_kernel<bf16_t, false><<<grid, 256, 0, st>>>((const bf16_t*)x, (bf16_t*)y, nullptr, *g, count_pad);
  } else {
    if (max_mode) poolnd_fwd_kernel<float, true><<<grid, 256, 0, st>>>((const float*)x, (float*)y, idx, *g, count_pad);
    else poolnd_fwd_kernel<float, false><<<grid, 256, 0, st>>>((const float*)x, (float*)y, nullptr, *g, count_pad);
  }
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_poolnd_bwd(const void* dy, const int* idx, void* dx, const PoolNdGeo* g, int max_mode, int count_pad,
                     int bf16, hipStream_t st) {
  if (!geo_ok(*g, true) || (max_mode && idx == nullptr)) return -1;
  const long total = (long)g->B * g->D * g->H * g->W * g->C;
  if (total == 0) return 0;
  const int grid = grid_for(total);
  if (bf16) {
    if (max_mode) poolnd_bwd_kernel<bf16_t, true><<<grid, 256, 0, st>>>((const bf16_t*)dy, idx, (bf16_t*)dx, *g, count_pad);
    else poolnd_bwd_kernel<bf16_t, false><<<grid, 256, 0, st>>>((const bf16_t*)dy, nullptr, (bf16_t*)dx, *g, count_pad);
  } else {
    if (max_mode) poolnd_bwd_kernel<float, true><<<grid, 256, 0, st>>>((const float*)dy, idx, (float*)dx, *g, count_pad);
    else poolnd_bwd_kernel<float, false><<<grid, 256, 0, st>>>((const float*)dy, nullptr, (float*)dx, *g, count_pad);
  }
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_upsample_nearest(const void* src, void* dst, const PoolNdGeo* g, int backward, int bf16, hipStream_t st) {
  if (!geo_ok(*g, false)) return -1;
  const long total = backward ? (long)g->B * g->D * g->H * g->W * g->C : (long)g->B * g->OD * g->OH * g->OW * g->C;
  if (total == 0) return 0;
  const int grid = grid_for(total);
  if (backward) {
    if (bf16) upsample_bwd_kernel<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)src, (bf16_t*)dst, *g);
    else upsample_bwd_kernel<float><<<grid, 256, 0, st>>>((const float*)src, (float*)dst, *g);
  } else {
    if (bf16) upsample_fwd_kernel<bf16_t><<<grid, 256, 0, st>>>((const bf16_t*)src, (bf16_t*)dst, *g);
    else upsample_fwd_kernel<float><<<grid, 256, 0, st>>>((const float*)src, (float*)dst, *g);
  }
  HIP_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
