// Fused flat-buffer updates of the adaptive OptimMethods for gfx950: Adagrad, RMSprop, Adadelta, Adamax, Ftrl.
//
// Reference: S/optim/Adagrad.scala, RMSprop.scala, Adadelta.scala, Adamax.scala, Ftrl.scala:39 (each a sequence of
// element-wise tensor ops over the flattened parameters). Here each update is ONE memory-bound pass over
// the (ZeRO-1 shard of the) flat fp32 buffer: 4 elements per lane with 16-byte loads, the state tensors updated in
// place and the bf16 compute shadow of the weights written in the same pass (the SGD / Adam kernels of
// elementwise.hip do the same), so an update never re-reads the parameters.
#include "common.h"
#include "kernels.h"

namespace {

enum Method { M_ADAGRAD = 0, M_RMSPROP, M_ADADELTA, M_ADAMAX, M_FTRL };

// per-method scalars: ADAGRAD (clr, wd); RMSPROP (clr, rho, eps); ADADELTA (rho, eps); ADAMAX (lr/(1-b1^t), b1, b2,
// eps); FTRL (lr, power, l1, l2, l2shrink)
__device__ __forceinline__ void update1(int k, const OptimHP& h, float& x, float g, float& s1, float& s2) {
  switch (k) {
    case M_ADAGRAD: {
      g += h.b * x;
      s1 += g * g;
      x -= h.a * g / (sqrtf(s1) + 1e-10f);
      break;
    }
    case M_RMSPROP: {
      s1 = h.b * s1 + (1.f - h.b) * g * g;
      x -= h.a * g / (sqrtf(s1) + h.c);
      break;
    }
    case M_ADADELTA: {
      s1 = h.a * s1 + (1.f - h.a) * g * g;
      const float d = sqrtf(s2 + h.b) / sqrtf(s1 + h.b) * g;
      x -= d;
      s2 = h.a * s2 + (1.f - h.a) * d * d;
      break;
    }
    case M_ADAMAX: {
      s1 = h.b * s1 + (1.f - h.b) * g;
      s2 = fmaxf(h.c * s2, fabsf(g) + h.d);
      x -= h.a * s1 / s2;
      break;
    }
    case M_FTRL: {
      const float gs = h.e > 0.f ? g + 2.f * h.e * x : g;
      const float acc_new = s1 + g * g;
      float sigma, quad;
      if (h.b == -0.5f) {
        sigma = (sqrtf(acc_new) - sqrtf(s1)) / h.a;
        quad = sqrtf(acc_new) / h.a + 2.f * h.d;
      } else {
        sigma = (powf(acc_new, -h.b) - powf(s1, -h.b)) / h.a;
        quad = powf(acc_new, -h.b) / h.a + 2.f * h.d;
      }
      s2 += gs - sigma * x;
      const float l1 = (s2 > 0.f ? 1.f : (s2 < 0.f ? -1.f : 0.f)) * h.c;
      x = fabsf(s2) > h.c ? (l1 - s2) / quad : 0.f;
      s1 = acc_new;
      break;
    }
  }
}

__global__ void optim4_kernel(int k, OptimHP h, float* __restrict__ x, const float* __restrict__ g,
                              float* __restrict__ s1, float* __restrict__ s2, bf16_t* __restrict__ w16, long n4) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    v4f xv = reinterpret_cast<v4f*>(x)[i];
    const v4f gv = reinterpret_cast<const v4f*>(g)[i];
    v4f a = reinterpret_cast<v4f*>(s1)[i];
    v4f b = s2 ? reinterpret_cast<v4f*>(s2)[i] : v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float xe = xv[e], ae = a[e], be = b[e];
      update1(k, h, xe, gv[e], ae, be);
      xv[e] = xe; a[e] = ae; b[e] = be;
    }
    reinterpret_cast<v4f*>(x)[i] = xv;
    reinterpret_cast<v4f*>(s1)[i] = a;
    if (s2) reinterpret_cast<v4f*>(s2)[i] = b;
    if (w16) reinterpret_cast<v2u*>(w16)[i] = v2u{pack2bf(xv[0], xv[1]), pack2bf(xv[2], xv[3])};
  }
}

__global__ void optim1_kernel(int k, OptimHP h, float* __restrict__ x, const float* __restrict__ g,
                              float* __restrict__ s1, float* __restrict__ s2, bf16_t* __restrict__ w16, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float xe = x[i], ae = s1[i], be = s2 ? s2[i] : 0.f;
    update1(k, h, xe, g[i], ae, be);
    x[i] = xe;
    s1[i] = ae;
    if (s2) s2[i] = be;
    if (w16) w16[i] = f2bf(xe);
  }
}

}  // namespace

extern "C" {

int bigdl_optim_step(int method, const OptimHP* hp, float* x, const float* g, float* s1, float* s2, uint16_t* w16,
                     long n, hipStream_t st) {
  if (method < M_ADAGRAD || method > M_FTRL) return -1;
  const bool vec = (n & 3) == 0 && ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(g) |
                                     reinterpret_cast<uintptr_t>(s1) | reinterpret_cast<uintptr_t>(s2)) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(w16) & 7) == 0;
  const long work = vec ? n / 4 : n;
  long blocks = (work + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  if (vec) optim4_kernel<<<(int)blocks, 256, 0, st>>>(method, *hp, x, g, s1, s2, w16, n / 4);
  else optim1_kernel<<<(int)blocks, 256, 0, st>>>(method, *hp, x, g, s1, s2, w16, n);
  HIP_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
