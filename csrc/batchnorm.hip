// BatchNorm for NHWC bf16 activations with fp32 statistics (gfx950).
//
// Replaces S/nn/SpatialBatchNormalization.scala (NCHW train fwd :1211, bwd :1048, NHWC :299-640) and
// the MKL-DNN BN primitive (S/nn/mkldnn/SpatialBatchNormalization.scala:212-344). MI355X design:
//  * two-phase reduce: every workgroup reduces a slab of rows for all channels in registers (16-byte
//    loads = 8 channels per lane), combines rows through LDS, then one fp32 atomic per channel;
//  * the stats phase is usually skipped entirely: the conv epilogue (conv_igemm.hip) already emits
//    sum / sum-of-squares for the BN that follows it;
//  * apply phase fuses the affine transform, the residual add of a ResNet block (CAddTable) and the
//    trailing ReLU into one pass; backward fuses the ReLU mask and emits the residual-branch gradient.
// Cross-replica sync-BN (S/utils/ParameterSynchronizer.scala) plugs in between reduce and finalize: the
// [2][C] fp32 stats buffer is all-reduced over RCCL by the Python layer.
#include "common.h"
#include "kernels.h"
#include <stdlib.h>

#define STAT_SLOTS BIGDL_STAT_SLOTS

namespace {

// Generic per-channel reduction over P rows of C channels (C % 8 == 0).
// MODE 0: stats     -> out[c] += x,          out[C+c] += x*x
// MODE 1: bwd       -> out[c] += dy,         out[C+c] += dy*(x-mean)  with dy = dz * (z>0 ? 1 : 0 if z)
// MODE 1 with z == nullptr and aff != nullptr: the ReLU mask is recomputed from x as x*scale + shift > 0 (the
// exact fp32 expression of bn_apply_kernel), so the post-ReLU output is never read back (one pass less).
template <int MODE, int U>
__global__ __launch_bounds__(256) void chan_reduce_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dz,
                                                          const bf16_t* __restrict__ z, const float* __restrict__ mean,
                                                          float* __restrict__ out, long P, int C, long rows_per_block,
                                                          const float* __restrict__ aff, const uint8_t* __restrict__ zm) {
  __shared__ float sm[256 * 16];
  const int G = C >> 3;
  const int tid = threadIdx.x;
  const long rbeg = blockIdx.x * rows_per_block;
  const long rend = min(P, rbeg + rows_per_block);
  for (int gbase = 0; gbase < G; gbase += 256) {
    const int gcount = min(256, G - gbase);
    const int rpi = 256 / gcount;          // rows per iteration
    const int g = gbase + tid % gcount, rsub = tid / gcount;
    float a1[8], a2[8], mu[8], sc[8], sh[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { a1[e] = 0.f; a2[e] = 0.f; mu[e] = 0.f; sc[e] = 0.f; sh[e] = 0.f; }
    const bool xmask = MODE == 1 && z == nullptr && zm == nullptr && aff != nullptr;
    const __amdgpu_buffer_rsrc_t rzm = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(zm), (short)0, zm ? (int)min((long)P * C / 8, 0x7fffffffl) : 0, 0x00020000);
    const bf16_t* zp = (z && !zm) ? z : x;
    if (MODE == 1 && rsub < rpi) {
#pragma unroll
      for (int e = 0; e < 8; ++e) mu[e] = mean[g * 8 + e];
      if (xmask) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { sc[e] = aff[g * 8 + e]; sh[e] = aff[C + g * 8 + e]; }
      }
    }
    if (rsub < rpi) {
      // U rows per trip, all loads issued before the first use: a lane keeps U (x, dz[, z]) granules in flight,
      // which is what lets a streaming reduction approach HBM bandwidth (one load in flight per lane is
      // latency-bound at ~2.5 TB/s). Rows past the block end re-read row rbeg and contribute zero.
      for (long r0 = rbeg + rsub; r0 < rend; r0 += (long)U * rpi) {
        v4u vx[U], vd[U], vz[U];
        unsigned zb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long r = r0 + (long)u * rpi;
          const size_t off = (size_t)(r < rend ? r : rbeg) * C + g * 8;
          vx[u] = *reinterpret_cast<const v4u*>(x + off);
          if (MODE == 1) {
            // unconditional loads (no branch, no phi): a load under `if (zm)` / `if (z)` made the compiler wait
            // for it at the join (vmcnt(0) per row), serialising the U rows. Absent masks read x (a cache hit)
            // or a 0-byte buffer resource, and are ignored below.
            vd[u] = *reinterpret_cast<const v4u*>(dz + off);
            zb[u] = __builtin_amdgcn_raw_buffer_load_b8(rzm, (unsigned)(off >> 3), 0, 0);
            vz[u] = *reinterpret_cast<const v4u*>(zp + off);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (MODE == 1 && zm) vz[u] = mask8_to_bf(zb[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool ok = r0 + (long)u * rpi < rend;
          if (MODE == 0) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float l = ok ? lo_bf(vx[u][e]) : 0.f, h = ok ? hi_bf(vx[u][e]) : 0.f;
              a1[2 * e] += l; a1[2 * e + 1] += h;
              a2[2 * e] += l * l; a2[2 * e + 1] += h * h;
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float dl = ok ? lo_bf(vd[u][e]) : 0.f, dh = ok ? hi_bf(vd[u][e]) : 0.f;
              const float xl = lo_bf(vx[u][e]), xh = hi_bf(vx[u][e]);
              if (z || zm) { if (!(lo_bf(vz[u][e]) > 0.f)) dl = 0.f; if (!(hi_bf(vz[u][e]) > 0.f)) dh = 0.f; }
              if (xmask) {
                if (!(xl * sc[2 * e] + sh[2 * e] > 0.f)) dl = 0.f;
                if (!(xh * sc[2 * e + 1] + sh[2 * e + 1] > 0.f)) dh = 0.f;
              }
              a1[2 * e] += dl; a1[2 * e + 1] += dh;
              a2[2 * e] += dl * (xl - mu[2 * e]);
              a2[2 * e + 1] += dh * (xh - mu[2 * e + 1]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) { sm[tid * 16 + e] = a1[e]; sm[tid * 16 + 8 + e] = a2[e]; }
    __syncthreads();
    // reduce over rsub for each (g, e, which)
    for (int w = tid; w < gcount * 16; w += 256) {
      const int gg = w >> 4, slot = w & 15;
      float t = 0.f;
      for (int rs = 0; rs < rpi; ++rs) t += sm[(rs * gcount + gg) * 16 + slot];
      const int ch = (gbase + gg) * 8 + (slot & 7);
      // spread over STAT_SLOTS copies: thousands of workgroups adding into the same 2C words serialise at
      // the memory-side atomic unit (MI355X_MICROARCH "contention"); finalize sums the slots.
      atomicAdd(out + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * 2 * C + (slot < 8 ? 0 : C) + ch, t);
    }
    __syncthreads();
  }
}

// Row unroll of the streaming BN passes (BIGDL_BN_UNROLL=1|2|4|8 for A/B runs; default 4).
int bn_unroll() {
  static int u = [] {
    const char* e = getenv("BIGDL_BN_UNROLL");
    const int v = e ? atoi(e) : 4;
    return (v == 1 || v == 2 || v == 8) ? v : 4;
  }();
  return u;
}

// Slot sums for one channel by 32 lanes (one slot each) + shuffle reduction: the per-layer finalize / coefficient
// kernels sit on the critical path between the big passes, and a serial 32-slot loop per thread made them
// latency-bound (~12 us each, 100+ per ResNet-50 step). Two channels per wave, lanes 0-31 and 32-63.
__device__ __forceinline__ void slot_sums(const float* __restrict__ red, int nslots, int C, int c, int sl, double& s1,
                                          double& s2) {
  s1 = 0.0;
  s2 = 0.0;
  for (int k = sl; k < nslots; k += 32) {
    s1 += red[(size_t)k * 2 * C + c];
    s2 += red[(size_t)k * 2 * C + C + c];
  }
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
}

__global__ void bn_finalize_kernel(const float* __restrict__ stats, int nslots, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float* run_mean, float* run_var, float* save_mean,
                                   float* save_invstd, float* scale, float* shift, long P, int C, float eps,
                                   float momentum, int training) {
  const int lane = threadIdx.x & 63, sl = lane & 31;
  const int c = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  if (c >= C) return;
  float mean, invstd;
  if (training) {
    double s1, s2;
    slot_sums(stats, nslots, C, c, sl, s1, s2);
    if (sl != 0) return;
    mean = (float)(s1 / (double)P);
    const float var = fmaxf((float)(s2 / (double)P - (double)mean * mean), 0.f);
    invstd = rsqrtf(var + eps);
    save_mean[c] = mean;
    save_invstd[c] = invstd;
    if (run_mean) {
      const float unbiased = P > 1 ? var * (float)P / (float)(P - 1) : var;
      run_mean[c] = momentum * mean + (1.f - momentum) * run_mean[c];
      run_var[c] = momentum * unbiased + (1.f - momentum) * run_var[c];
    }
  } else {
    if (sl != 0) return;
    mean = run_mean[c];
    invstd = rsqrtf(run_var[c] + eps);
    if (save_mean) { save_mean[c] = mean; save_invstd[c] = invstd; }
  }
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * invstd;
  shift[c] = b - mean * g * invstd;
}

// Channel-stationary mapping (also bn_bwd_apply_kernel): a thread owns one 8-channel group for its whole row
// range, so its per-channel coefficients are loaded once instead of once per 16-byte granule, and the loop has
// no 64-bit modulo. blockIdx.y walks channel groups in chunks of 256; rows of a block are [rbeg, rend).
template <int U>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ x, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, const bf16_t* __restrict__ res,
                                                       bf16_t* __restrict__ y, long P, int C, long rpb, int relu,
                                                       uint8_t* __restrict__ zm) {
  const int G = C >> 3;
  const int gbase = blockIdx.y * 256;
  const int gcount = min(256, G - gbase);
  const int rpi = 256 / gcount;
  const int g = gbase + threadIdx.x % gcount, rsub = threadIdx.x / gcount;
  if (rsub >= rpi) return;
  const long rbeg = blockIdx.x * rpb, rend = min(P, rbeg + rpb);
  const int c0 = g * 8;
  const v4f s0 = *reinterpret_cast<const v4f*>(scale + c0), s1 = *reinterpret_cast<const v4f*>(scale + c0 + 4);
  const v4f b0 = *reinterpret_cast<const v4f*>(shift + c0), b1 = *reinterpret_cast<const v4f*>(shift + c0 + 4);
  const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
  const float sh[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
  for (long r0 = rbeg + rsub; r0 < rend; r0 += (long)U * rpi) {
    v4u vx[U], vr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {     // all U rows' loads in flight before the first store
      const long r = r0 + (long)u * rpi;
      const long i = (r < rend ? r : rbeg) * G + g;
      vx[u] = reinterpret_cast<const v4u*>(x)[i];
      vr[u] = v4u{0u, 0u, 0u, 0u};
      if (res) vr[u] = reinterpret_cast<const v4u*>(res)[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = r0 + (long)u * rpi;
      v4u o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float l = lo_bf(vx[u][e]) * sc[2 * e] + sh[2 * e];
        float h = hi_bf(vx[u][e]) * sc[2 * e + 1] + sh[2 * e + 1];
        if (res) { l += lo_bf(vr[u][e]); h += hi_bf(vr[u][e]); }
        if (relu) { l = fmaxf(l, 0.f); h = fmaxf(h, 0.f); }
        o[e] = pack2bf(l, h);
      }
      if (r < rend) {
        reinterpret_cast<v4u*>(y)[r * G + g] = o;
        if (zm) zm[r * G + g] = (uint8_t)bf_to_mask8(o);   // 1 byte per 8 channels: the backward's ReLU mask
      }
    }
  }
}

// Per-channel backward coefficients: dx = A*dy + B*x + D (dy = dz masked by the fused ReLU), with
//   A = g*is, B = -g*is^2*mean(dy*xhat)/... , D = g*is*(mean*is*m_dyx - m_dy); param grads folded in.
__global__ void bn_bwd_coeff_kernel(const float* __restrict__ red, int nslots, const float* __restrict__ mean,
                                    const float* __restrict__ invstd, const float* __restrict__ gamma,
                                    float* __restrict__ coef, float* dgamma, float* dbeta, long P, int C, int training) {
  const int lane = threadIdx.x & 63, sl = lane & 31;
  const int c = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  if (c >= C) return;
  double sdy = 0.0, sdyx = 0.0;
  if (training) slot_sums(red, nslots, C, c, sl, sdy, sdyx);
  if (sl != 0) return;
  const float is = invstd[c];
  const float g = gamma ? gamma[c] : 1.f;
  float A = g * is, B = 0.f, D = 0.f;
  if (training) {
    const float mdy = (float)(sdy / (double)P);
    const float mdyx = (float)(sdyx / (double)P) * is;     // mean(dy * xhat)
    B = -g * is * is * mdyx;
    D = g * is * (mean[c] * is * mdyx - mdy);
    if (dgamma) dgamma[c] += (float)sdyx * is;
    if (dbeta) dbeta[c] += (float)sdy;
  }
  coef[c] = A; coef[C + c] = B; coef[2 * C + c] = D;
}

__global__ void bn_slot_reduce_kernel(const float* __restrict__ in, int nslots, int C, float* __restrict__ out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 2 * C) return;
  float t = 0.f;
  for (int k = 0; k < nslots; ++k) t += in[(size_t)k * 2 * C + c];
  out[c] = t;
}

__device__ __forceinline__ void load8(const float* p, float* v) {
  const v4f a = *reinterpret_cast<const v4f*>(p), b = *reinterpret_cast<const v4f*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}

// R2: the residual-branch gradient dres (= masked dz) is also the output gradient of a second training BN without
// ReLU (the projection shortcut's BN of a ResNet downsampling block, input x2 / mean2): its backward reduction
// (sum dres, sum dres*(x2 - mean2), over dres as stored in bf16) is accumulated here into the slotted `red2`, which
// saves that BN a chan_reduce pass re-reading dres and x2 (nn/fusion.py residual_backward).
template <int U, bool R2>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16_t* __restrict__ dz, const bf16_t* __restrict__ z,
                                                           const bf16_t* __restrict__ x, const float* __restrict__ coef,
                                                           bf16_t* __restrict__ dx, bf16_t* __restrict__ dres, long P,
                                                           int C, long rpb, const float* __restrict__ aff,
                                                           const uint8_t* __restrict__ zm, const bf16_t* __restrict__ x2,
                                                           const float* __restrict__ mean2, float* __restrict__ red2) {
  const int G = C >> 3;
  const bool xmask = z == nullptr && zm == nullptr && aff != nullptr;   // ReLU mask from x*scale + shift (see chan_reduce_kernel)
  const __amdgpu_buffer_rsrc_t rzm = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(zm), (short)0, zm ? (int)min(P * C / 8, 0x7fffffffl) : 0, 0x00020000);
  const bf16_t* zp = (z && !zm) ? z : x;
  const int gbase = blockIdx.y * 256;
  const int gcount = min(256, G - gbase);
  const int rpi = 256 / gcount;
  const int g = gbase + threadIdx.x % gcount, rsub = threadIdx.x / gcount;
  if (!R2 && rsub >= rpi) return;
  const long rbeg = blockIdx.x * rpb, rend = rsub < rpi ? min(P, rbeg + rpb) : rbeg;   // idle threads: no rows
  const int c0 = g * 8;
  float A[8], B[8], D[8], S[8], T[8], M2[8], a1[8], a2[8];
  load8(coef + c0, A);
  load8(coef + C + c0, B);
  load8(coef + 2 * C + c0, D);
  if (xmask) {
    load8(aff + c0, S);
    load8(aff + C + c0, T);
  }
  if (R2) {
    load8(mean2 + c0, M2);
#pragma unroll
    for (int e = 0; e < 8; ++e) { a1[e] = 0.f; a2[e] = 0.f; }
  }
  for (long r0 = rbeg + rsub; r0 < rend; r0 += (long)U * rpi) {
    v4u vd[U], vz[U], vx[U], vx2[U];
    unsigned zb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = r0 + (long)u * rpi;
      const long i = (r < rend ? r : rbeg) * G + g;
      vd[u] = reinterpret_cast<const v4u*>(dz)[i];
      // unconditional mask loads (see chan_reduce_kernel): absent masks read x (a cache hit) / a 0-byte resource
      zb[u] = __builtin_amdgcn_raw_buffer_load_b8(rzm, (unsigned)i, 0, 0);
      vz[u] = reinterpret_cast<const v4u*>(zp)[i];
      vx[u] = reinterpret_cast<const v4u*>(x)[i];
      if (R2) vx2[u] = reinterpret_cast<const v4u*>(x2)[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      vz[u] = zm ? mask8_to_bf(zb[u]) : z ? vz[u] : v4u{0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long r = r0 + (long)u * rpi;
      v4u o, od;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float d0 = lo_bf(vd[u][e]), d1 = hi_bf(vd[u][e]);
        const float x0 = lo_bf(vx[u][e]), x1 = hi_bf(vx[u][e]);
        if (z || zm) { if (!(lo_bf(vz[u][e]) > 0.f)) d0 = 0.f; if (!(hi_bf(vz[u][e]) > 0.f)) d1 = 0.f; }
        if (xmask) {
          if (!(x0 * S[2 * e] + T[2 * e] > 0.f)) d0 = 0.f;
          if (!(x1 * S[2 * e + 1] + T[2 * e + 1] > 0.f)) d1 = 0.f;
        }
        const float r0v = A[2 * e] * d0 + B[2 * e] * x0 + D[2 * e];
        const float r1v = A[2 * e + 1] * d1 + B[2 * e + 1] * x1 + D[2 * e + 1];
        o[e] = pack2bf(r0v, r1v);
        od[e] = pack2bf(d0, d1);
        if (R2 && r < rend) {
          const float q0 = lo_bf(od[e]), q1 = hi_bf(od[e]);
          a1[2 * e] += q0; a1[2 * e + 1] += q1;
          a2[2 * e] += q0 * (lo_bf(vx2[u][e]) - M2[2 * e]);
          a2[2 * e + 1] += q1 * (hi_bf(vx2[u][e]) - M2[2 * e + 1]);
        }
      }
      if (r < rend) {
        if (dx) reinterpret_cast<v4u*>(dx)[r * G + g] = o;
        if (dres) reinterpret_cast<v4u*>(dres)[r * G + g] = od;
      }
    }
  }
  if (R2) {
    // per-workgroup sums through LDS (threads of one channel group sit gcount apart), one atomic per value
    __shared__ float sm[256 * 16];
#pragma unroll
    for (int e = 0; e < 8; ++e) { sm[threadIdx.x * 16 + e] = a1[e]; sm[threadIdx.x * 16 + 8 + e] = a2[e]; }
    __syncthreads();
    for (int w = threadIdx.x; w < gcount * 16; w += 256) {
      const int gg = w >> 4, slot = w & 15;
      float t = 0.f;
      for (int rs = 0; rs < rpi; ++rs) t += sm[(rs * gcount + gg) * 16 + slot];
      const int ch = (gbase + gg) * 8 + (slot & 7);
      atomicAdd(red2 + (size_t)(blockIdx.x & (STAT_SLOTS - 1)) * 2 * C + (slot < 8 ? 0 : C) + ch, t);
    }
  }
}

// Grid of a channel-stationary elementwise pass: (row blocks, channel-group chunks); ~8 rows per thread.
dim3 stationary_grid(long P, int C, long* rpb_out) {
  const int G = C >> 3;
  const int rpi = 256 / (G < 256 ? G : 256);
  const int gy = (G + 255) / 256;
  long rpb = (long)rpi * 8;
  long bx = (P + rpb - 1) / rpb;
  const long cap = 8192 / gy;
  if (bx > cap) {
    bx = cap;
    rpb = (P + bx - 1) / bx;
  }
  if (bx < 1) bx = 1;
  *rpb_out = rpb;
  return dim3((unsigned)bx, (unsigned)gy);
}

int grid_for(long work, int per_block, int cap) {
  long g = (work + per_block - 1) / per_block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

void launch_reduce(int mode, const bf16_t* x, const bf16_t* dz, const bf16_t* z, const float* mean, float* out, long P,
                   int C, hipStream_t st, const float* aff = nullptr, const uint8_t* zm = nullptr) {
  const int G = C >> 3;
  const int rpi = 256 / (G < 256 ? G : 256);
  long blocks = (P + rpi * 16 - 1) / (rpi * 16);   // >= 16 rows per thread
  if (blocks > 2048) blocks = 2048;
  // deterministic mode: at most two blocks per statistics slot, so every slot word receives at most two atomics
  // onto zero — fl(0 + a + b) is the same in either arrival order (IEEE addition commutes; only a third addend
  // makes the order visible) — and the reduction keeps one workgroup per CU instead of half the chip
  if (bigdl_deterministic() && blocks > 2 * STAT_SLOTS) blocks = 2 * STAT_SLOTS;
  if (blocks < 1) blocks = 1;
  const long rpb = (P + blocks - 1) / blocks;
  blocks = (P + rpb - 1) / rpb;
#define BN_RED(M, U) chan_reduce_kernel<M, U><<<(int)blocks, 256, 0, st>>>(x, dz, z, mean, out, P, C, rpb, aff, zm)
  if (mode == 0) { aff = nullptr; zm = nullptr; }
  switch (bn_unroll()) {
    case 1: if (mode == 0) BN_RED(0, 1); else BN_RED(1, 1); break;
    case 2: if (mode == 0) BN_RED(0, 2); else BN_RED(1, 2); break;
    case 8: if (mode == 0) BN_RED(0, 8); else BN_RED(1, 8); break;
    default: if (mode == 0) BN_RED(0, 4); else BN_RED(1, 4); break;
  }
#undef BN_RED
}

}  // namespace

extern "C" {

void bigdl_bn_stats(const uint16_t* x, float* stats, long P, int C, hipStream_t st) {
  launch_reduce(0, x, nullptr, nullptr, nullptr, stats, P, C, st);
  HIP_LAUNCH_CHECK();
}

void bigdl_bn_finalize(const float* stats, int nslots, const float* gamma, const float* beta, float* run_mean,
                       float* run_var, float* save_mean, float* save_invstd, float* scale, float* shift, long P, int C,
                       float eps, float momentum, int training, hipStream_t st) {
  bn_finalize_kernel<<<(C + 7) / 8, 256, 0, st>>>(stats, nslots, gamma, beta, run_mean, run_var, save_mean,
                                                   save_invstd, scale, shift, P, C, eps, momentum, training);
  HIP_LAUNCH_CHECK();
}

void bigdl_bn_slot_reduce(const float* in, int nslots, int C, float* out, hipStream_t st) {
  bn_slot_reduce_kernel<<<(2 * C + 255) / 256, 256, 0, st>>>(in, nslots, C, out);
  HIP_LAUNCH_CHECK();
}

void bigdl_bn_apply(const uint16_t* x, const float* scale, const float* shift, const uint16_t* res, uint16_t* y,
                    long P, int C, int relu, hipStream_t st, uint8_t* zm) {
  long rpb = 0;
  const dim3 grid = stationary_grid(P, C, &rpb);
  switch (bn_unroll()) {
    case 1: bn_apply_kernel<1><<<grid, 256, 0, st>>>(x, scale, shift, res, y, P, C, rpb, relu, zm); break;
    case 2: bn_apply_kernel<2><<<grid, 256, 0, st>>>(x, scale, shift, res, y, P, C, rpb, relu, zm); break;
    case 8: bn_apply_kernel<8><<<grid, 256, 0, st>>>(x, scale, shift, res, y, P, C, rpb, relu, zm); break;
    default: bn_apply_kernel<4><<<grid, 256, 0, st>>>(x, scale, shift, res, y, P, C, rpb, relu, zm); break;
  }
  HIP_LAUNCH_CHECK();
}

void bigdl_bn_bwd_reduce(const uint16_t* dz, const uint16_t* z, const uint16_t* x, const float* mean, float* red,
                         long P, int C, const float* aff, hipStream_t st, const uint8_t* zm) {
  launch_reduce(1, x, dz, z, mean, red, P, C, st, aff, zm);
  HIP_LAUNCH_CHECK();
}

void bigdl_bn_bwd_apply(const uint16_t* dz, const uint16_t* z, const uint16_t* x, const float* mean,
                        const float* invstd, const float* gamma, const float* red, int nslots, float* coef,
                        uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta, long P, int C, int training,
                        const float* aff, hipStream_t st, const uint8_t* zm, const uint16_t* x2u,
                        const float* mean2, float* red2) {
  const bf16_t* x2 = reinterpret_cast<const bf16_t*>(x2u);
  bn_bwd_coeff_kernel<<<(C + 7) / 8, 256, 0, st>>>(red, nslots, mean, invstd, gamma, coef, dgamma, dbeta, P, C,
                                                    training);
  if (dx || dres) {
    long rpb = 0;
    const dim3 grid = stationary_grid(P, C, &rpb);
    if (red2) {        // second BN's reduction over dres (needs dres)
#define BWD2(UU) bn_bwd_apply_kernel<UU, true><<<grid, 256, 0, st>>>(dz, z, x, coef, dx, dres, P, C, rpb, aff, zm, x2, mean2, red2)
      switch (bn_unroll()) {
        case 1: BWD2(1); break;
        case 2: BWD2(2); break;
        case 8: BWD2(8); break;
        default: BWD2(4); break;
      }
#undef BWD2
    } else {
#define BWD1(UU) bn_bwd_apply_kernel<UU, false><<<grid, 256, 0, st>>>(dz, z, x, coef, dx, dres, P, C, rpb, aff, zm, nullptr, nullptr, nullptr)
      switch (bn_unroll()) {
        case 1: BWD1(1); break;
        case 2: BWD1(2); break;
        case 8: BWD1(8); break;
        default: BWD1(4); break;
      }
#undef BWD1
    }
  }
  HIP_LAUNCH_CHECK();
}

}  // extern "C"
