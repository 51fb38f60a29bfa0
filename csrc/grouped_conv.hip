// Direct grouped / depthwise convolution for gfx950 (fp32 NCHW), one launch per pass for ALL groups.
//
// Reference: S/nn/SpatialConvolution.scala (nGroup), S/nn/SpatialSeparableConvolution.scala:54 (depthwise
// + pointwise), S/nn/mkldnn/SpatialConvolution.scala group handling.
//
// Groups with few input channels per group (depthwise = 1, ResNeXt-style 4-16) carry too little reduction
// depth for an MFMA GEMM (K = cin_g * R * S is 9-144) and the round-1 path launched one GEMM per group and
// concatenated the results. Here every pass is ONE launch over all groups:
//   forward  : one thread per output element (ow fastest: coalesced x reads, wave-uniform weight reads)
//   dgrad    : one thread per input element, gathering the taps that hit it (stride phases by divisibility)
//   wgrad    : one workgroup per (output channel, input channel of its group, tap) reducing over N*OH*OW,
//              plus one per output channel for the bias
// These layers are memory-bound (9-144 FMAs per output), so fp32 NCHW in place of bf16 NHWC costs nothing on
// the hot path and avoids any layout conversion.
#include "common.h"
#include "kernels.h"

namespace {

struct GConv {
  int N, C, H, W, K, OH, OW, R, S, sh, sw, ph, pw, dh, dw, G;
};

__global__ void __launch_bounds__(256) gconv_fwd_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ b, float* __restrict__ y, GConv g) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)g.N * g.K * g.OH * g.OW;
  if (idx >= total) return;
  const int ow = idx % g.OW;
  const int oh = (idx / g.OW) % g.OH;
  const int k = (idx / ((long)g.OW * g.OH)) % g.K;
  const int n = idx / ((long)g.OW * g.OH * g.K);
  const int cin_g = g.C / g.G, cout_g = g.K / g.G;
  const int c0 = (k / cout_g) * cin_g;
  float acc = b ? b[k] : 0.f;
  const float* wk = w + (long)k * cin_g * g.R * g.S;
  for (int cl = 0; cl < cin_g; ++cl) {
    const float* xc = x + ((long)n * g.C + c0 + cl) * g.H * g.W;
    for (int r = 0; r < g.R; ++r) {
      const int ih = oh * g.sh - g.ph + r * g.dh;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int s = 0; s < g.S; ++s) {
        const int iw = ow * g.sw - g.pw + s * g.dw;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        acc += xc[(long)ih * g.W + iw] * wk[(cl * g.R + r) * g.S + s];
      }
    }
  }
  y[idx] = acc;
}

__global__ void __launch_bounds__(256) gconv_dgrad_kernel(const float* __restrict__ dy, const float* __restrict__ w,
                                                          float* __restrict__ dx, GConv g) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)g.N * g.C * g.H * g.W;
  if (idx >= total) return;
  const int iw = idx % g.W;
  const int ih = (idx / g.W) % g.H;
  const int c = (idx / ((long)g.W * g.H)) % g.C;
  const int n = idx / ((long)g.W * g.H * g.C);
  const int cin_g = g.C / g.G, cout_g = g.K / g.G;
  const int grp = c / cin_g, cl = c % cin_g;
  float acc = 0.f;
  for (int m = 0; m < cout_g; ++m) {
    const int k = grp * cout_g + m;
    const float* dyk = dy + ((long)n * g.K + k) * g.OH * g.OW;
    const float* wk = w + ((long)k * cin_g + cl) * g.R * g.S;
    for (int r = 0; r < g.R; ++r) {
      const int th = ih + g.ph - r * g.dh;
      if (th < 0 || th % g.sh) continue;
      const int oh = th / g.sh;
      if (oh >= g.OH) continue;
      for (int s = 0; s < g.S; ++s) {
        const int tw = iw + g.pw - s * g.dw;
        if (tw < 0 || tw % g.sw) continue;
        const int ow = tw / g.sw;
        if (ow >= g.OW) continue;
        acc += dyk[(long)oh * g.OW + ow] * wk[r * g.S + s];
      }
    }
  }
  dx[idx] = acc;
}

// blockIdx.x = k * cin_g + cl (weight row), blockIdx.y = tap (r * S + s), or tap == R*S: bias of channel k (cl 0)
__global__ void __launch_bounds__(256) gconv_wgrad_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                          float* __restrict__ dw, float* __restrict__ db, GConv g) {
  __shared__ float red[4];
  const int cin_g = g.C / g.G, cout_g = g.K / g.G;
  const int k = blockIdx.x / cin_g, cl = blockIdx.x % cin_g;
  const int tap = blockIdx.y;
  const bool bias = tap == g.R * g.S;
  if (bias && (cl != 0 || !db)) return;
  const int r = bias ? 0 : tap / g.S, s = bias ? 0 : tap % g.S;
  const int c = (k / cout_g) * cin_g + cl;
  const long P = (long)g.N * g.OH * g.OW;
  float acc = 0.f;
  for (long p = threadIdx.x; p < P; p += 256) {
    const int ow = p % g.OW;
    const int oh = (p / g.OW) % g.OH;
    const int n = p / ((long)g.OW * g.OH);
    const float d = dy[((long)n * g.K + k) * g.OH * g.OW + (long)oh * g.OW + ow];
    if (bias) { acc += d; continue; }
    const int ih = oh * g.sh - g.ph + r * g.dh, iw = ow * g.sw - g.pw + s * g.dw;
    if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
      acc += d * x[((long)n * g.C + c) * g.H * g.W + (long)ih * g.W + iw];
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    const float t = red[0] + red[1] + red[2] + red[3];
    if (bias) db[k] += t;
    else dw[((long)k * cin_g + cl) * g.R * g.S + tap] += t;
  }
}

unsigned blocks(long n) { return (unsigned)((n + 255) / 256); }

}  // namespace

int bigdl_gconv(const GConvCall* c, int pass, hipStream_t st) {
  GConv g{c->N, c->C, c->H, c->W, c->K, c->OH, c->OW, c->R, c->S, c->sh, c->sw, c->ph, c->pw, c->dh, c->dw, c->G};
  if (g.G <= 0 || g.C % g.G || g.K % g.G || g.N <= 0 || g.OH <= 0 || g.OW <= 0) return -1;
  if (pass == 0) {
    gconv_fwd_kernel<<<blocks((long)g.N * g.K * g.OH * g.OW), 256, 0, st>>>(c->x, c->w, c->b, c->y, g);
  } else if (pass == 1) {
    gconv_dgrad_kernel<<<blocks((long)g.N * g.C * g.H * g.W), 256, 0, st>>>(c->dy, c->w, c->dx, g);
  } else {
    dim3 grid(g.K * (g.C / g.G), g.R * g.S + 1);
    gconv_wgrad_kernel<<<grid, 256, 0, st>>>(c->dy, c->x, c->dwt, c->db, g);
  }
  HIP_LAUNCH_CHECK();
  return 0;
}
