// Int8 inference path for gfx950: dynamic per-sample activation quantization and an implicit-GEMM
// convolution / linear on the i8 matrix cores (v_mfma_i32_16x16x64_i8: twice the bf16 MACs per cycle).
//
// Reference: S/nn/quantized/{Quantization.scala:27-180 (symmetric max-abs / 127 scaling, per output row for
// weights), SpatialConvolution.scala:197-203 + Linear.scala:79-90 (BigQuant ConvDataInit / FCDataInit:
// on-the-fly input quantization; MixPrecisionGEMM: int8 x int8 -> int32, dequantized to fp32)}.
//
// Design: activations are quantized once per layer call into an NHWC int8 image with one scale per sample
// (amax reduction + quantize: two memory-bound kernels), weights are quantized offline per output channel
// into a KRSC int8 matrix. The conv kernel is the bf16 NT kernel's structure with 16 int8 per 16-byte granule
// (BK = 128 elements = 128 bytes per LDS row, same XOR-swizzled image), int32 accumulation, and a dequantizing
// epilogue y = acc * s_x[image] * s_w[channel] + bias (+ReLU) written as bf16 NHWC.
#include "common.h"
#include "kernels.h"
#include <stdlib.h>

namespace {


__device__ __attribute__((aligned(64))) uint8_t g_zero16[64];

constexpr int QBK = 128;   // int8 elements per LDS row (8 granules of 16 B)

// ---------------------------------------------------------------------------------- quantize activations
template <typename T>
__device__ __forceinline__ float ldf(const T* p, long i);
template <>
__device__ __forceinline__ float ldf<float>(const float* p, long i) { return p[i]; }
template <>
__device__ __forceinline__ float ldf<uint16_t>(const uint16_t* p, long i) { return bf2f(p[i]); }

// amax per sample: grid (blocks_per_sample, N); positive floats order like their bit patterns.
// bf16 rows whose length is a multiple of 8 are read 16 bytes per lane (the activations of a 256-image batch
// are 100+ MB: a 2-byte-per-lane scan was the int8 path's largest kernel).
template <typename T>
__global__ void amax_kernel(const T* __restrict__ x, long per_sample, float* __restrict__ amax) {
  const int n = blockIdx.y;
  const T* xs = x + (long)n * per_sample;
  float m = 0.f;
  if (sizeof(T) == 2 && (per_sample & 7) == 0) {
    const v4u* v = reinterpret_cast<const v4u*>(xs);
    const long n8 = per_sample >> 3;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
      const v4u u = v[i];
#pragma unroll
      for (int e = 0; e < 4; ++e) m = fmaxf(m, fmaxf(fabsf(lo_bf(u[e])), fabsf(hi_bf(u[e]))));
    }
  } else {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < per_sample; i += (long)gridDim.x * blockDim.x)
      m = fmaxf(m, fabsf(ldf<T>(xs, i)));
  }
  m = wave_max(m);
  __shared__ float red[16];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t = fmaxf(t, red[i]);
    atomicMax(reinterpret_cast<unsigned*>(amax) + n, __float_as_uint(t));
  }
}

// x [N][P][C] (NHWC-contiguous) -> q [N][P][Cp] int8 (channel pad zero), scale = amax / 127
template <typename T>
__global__ void quantize_kernel(const T* __restrict__ x, int8_t* __restrict__ q, const float* __restrict__ amax,
                                float* __restrict__ scale, long P, int C, int Cp, int N) {
  const long total = (long)N * P * Cp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % Cp);
    const long pix = i / Cp;
    const int n = (int)(pix / P);
    const float a = amax[n];
    const float inv = a > 0.f ? 127.f / a : 0.f;
    int v = 0;
    if (c < C) v = __float2int_rn(ldf<T>(x, pix * C + c) * inv);
    q[i] = (int8_t)max(-127, min(127, v));
    if (i < N) scale[i] = amax[i] / 127.f;
  }
}

// C == Cp, C % 8 == 0, bf16: 8 channels per lane, one 16-byte load and one 8-byte store.
__global__ void quantize8_bf16_kernel(const v4u* __restrict__ x, v2u* __restrict__ q, const float* __restrict__ amax,
                                      float* __restrict__ scale, long per8, int N) {
  const long total = (long)N * per8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int n = (int)(i / per8);
    const float a = amax[n];
    const float inv = a > 0.f ? 127.f / a : 0.f;
    const v4u u = x[i];
    unsigned packed[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int v0 = max(-127, min(127, __float2int_rn(lo_bf(u[e]) * inv)));
      const int v1 = max(-127, min(127, __float2int_rn(hi_bf(u[e]) * inv)));
      packed[e >> 1] |= ((unsigned)(v0 & 0xff) | ((unsigned)(v1 & 0xff) << 8)) << (16 * (e & 1));
    }
    v2u o;
    o[0] = packed[0];
    o[1] = packed[1];
    q[i] = o;
    if (i < N) scale[i] = amax[i] / 127.f;
  }
}

// ---------------------------------------------------------------------------------- int8 conv
// LDS-DMA implicit GEMM on v_mfma_i32_16x16x64_i8. The LDS image, fragment reads and XOR swizzle are byte-for-byte
// those of the bf16 conv_nt_glds_kernel (conv_igemm.hip): a 16-byte granule is 16 int8 channels instead of 8 bf16,
// a 128-byte K stage is 128 int8 taps*channels instead of 64, and one i8 MFMA consumes a 16-byte fragment per lane
// exactly like the bf16 one — so the int8 kernel moves half the operand bytes per MAC and issues half the MFMAs.
// Operands go global -> LDS with global_load_lds_dwordx4 (no VGPR staging); a K stage lies in one tap when
// Cs % 128 == 0 (FASTK), otherwise every lane resolves the tap of its own granule.
// Epilogue (through the idle staging LDS, one pixel row of 8 channels per lane): y = acc * s_x * s_w[n] + bias
// (+ReLU), stored as bf16 / fp32, or requantized to int8 with the consumer's static scale (y * out_inv, round,
// clamp +-127) — the int8 output path lets the next quantized layer (or a concat slice it reads) consume it
// directly, with no separate quantize pass. Output rows are `ldo` apart, so a concat slice is just an offset.
__device__ __forceinline__ void glds16(const void* g, LDS_PTR(void) l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g, l, 16, 0, 0);
}

// I8Epi (the int8 epilogue's scales / output mode / residual addend): csrc/kernels.h

//
// Tiles: 128 x 128 (2 x 2 waves) by default; narrow layers (Ncol <= 64 / <= 32 — the 147x147 / 73x73 stem convs
// and the 64-, 48-, 32-channel branch convs of Inception) use 256 x 64 / 256 x 32 tiles with the four waves stacked
// along M, so no MFMA is spent on the empty half (or three quarters) of a 128-wide tile.
template <int BM, int BN, int WM, bool FASTK>
__global__ __launch_bounds__(256, 2) void conv_i8_glds_kernel(ConvArgs a, I8Epi ep) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int AI = BM / 32, BI = BN / 32;
  constexpr int STAGE = (BM + BN) * QBK;          // bytes
  __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * STAGE];
  const uint8_t* src = reinterpret_cast<const uint8_t*>(a.src);
  const uint8_t* wt = reinterpret_cast<const uint8_t*>(a.wt);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (a.Ncol + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // DMA lane geometry (as conv_nt_glds_kernel): instruction i of wave w fills rows (i*4 + w)*8 .. +8; lane ->
  // row += lane>>3, LDS slot lane&7 holds source granule (lane ^ (lane>>3)) & 7.
  const int rsub = lane >> 3;
  const int gsrc = (lane ^ rsub) & 7;
  int a_pix[AI], a_h[AI], a_w[AI];
  const int ohw = a.OH * a.OW;
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + (i * 4 + wave) * 8 + rsub;
    if (m < a.M) {
      const int nb = m / ohw, rem = m - nb * ohw;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      a_pix[i] = nb * a.Hs * a.Ws;
      a_h[i] = oh * a.mul_h;
      a_w[i] = ow * a.mul_w;
    } else {
      a_pix[i] = 0; a_h[i] = -(1 << 28); a_w[i] = -(1 << 28);
    }
  }
  const uint8_t* wrow[BI];
  bool bvalid[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int n = n0 + (i * 4 + wave) * 8 + rsub;
    bvalid[i] = n < a.Ncol;
    wrow[i] = wt + (size_t)(bvalid[i] ? n : 0) * a.ldw;
  }
  auto issue = [&](int kt, int buf) {
    const int k0 = kt * QBK;
    int th, tw, c, wk;
    bool kv = true;
    if constexpr (FASTK) {
      const int t = k0 / a.Cs;
      c = k0 - t * a.Cs + gsrc * 16;
      th = a.tap_h[t]; tw = a.tap_w[t];
      wk = a.tap_k[t] * a.Cs + c;
    } else {
      const int kk = k0 + gsrc * 16;
      kv = kk < a.Kdim;
      const int kc = kv ? kk : 0;
      const int t = kc / a.Cs;
      c = kc - t * a.Cs;
      th = a.tap_h[t]; tw = a.tap_w[t];
      wk = a.tap_k[t] * a.Cs + c;
    }
    uint8_t* A = lds + buf * STAGE;
    uint8_t* B = A + BM * QBK;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int ch = a_h[i] + th, cw = a_w[i] + tw;
      const bool ok = kv && (unsigned)ch < (unsigned)a.Hs && (unsigned)cw < (unsigned)a.Ws;
      const uint8_t* g = ok ? src + (size_t)(a_pix[i] + ch * a.Ws + cw) * a.Cs + c : g_zero16;
      glds16(g, (LDS_PTR(void))(A + (i * 4 + wave) * 8 * QBK));
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const uint8_t* g = (bvalid[i] && kv) ? wrow[i] + wk : g_zero16;
      glds16(g, (LDS_PTR(void))(B + (i * 4 + wave) * 8 * QBK));
    }
  };
  auto swz = [](int row, int g) { return row * QBK + ((g ^ (row & 7)) << 4); };

  v4i acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  const int nk = (a.Kdim + QBK - 1) / QBK;
  issue(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) issue(kt + 1, cur ^ 1);
    const uint8_t* A = lds + cur * STAGE;
    const uint8_t* B = A + BM * QBK;
#pragma unroll
    for (int ks = 0; ks < QBK / 64; ++ks) {
      v4i fa[MI], fb[NI];
      const int g = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const v4i*>(A + swz(wm * TM + i * 16 + (lane & 15), g));
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[j] = *reinterpret_cast<const v4i*>(B + swz(wn * TN + j * 16 + (lane & 15), g));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    __syncthreads();   // retires the stage-(k+1) DMA and the stage-k fragment reads
  }

  // ---- epilogue: park the wave's int32 tile (as fp32, exact to 2^24 relative rounding) in its LDS slice,
  // XOR-swizzled by pixel, then re-read one pixel row of 8 channels per lane.
  constexpr int GR = TN / 4, LPR = TN / 8, PPI = 64 / LPR, NR = TM / PPI;
  float* wl = reinterpret_cast<float*>(lds) + wave * TM * TN;
  auto gpos = [](int p, int g) { return (p * GR + (g ^ (p & (GR - 1)))) * 4; };
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const v4i v = acc[i][j];
      *reinterpret_cast<v4f*>(wl + gpos(i * 16 + (lane & 15), j * 4 + (lane >> 4))) =
          v4f{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
    }
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes landed (wave-private slice)
  const int q = lane % LPR;
  const int mbase = m0 + wm * TM, n = n0 + wn * TN + q * 8;
  if (n >= a.Ncol) return;
  const bool full8 = n + 8 <= a.Ncol;
  float wsc[8], bs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const bool ok = n + e < a.Ncol;
    wsc[e] = ok ? ep.wscale[n + e] : 0.f;
    bs[e] = (ok && a.bias) ? a.bias[n + e] : 0.f;
  }
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int p = r * PPI + lane / LPR;
    const int m = mbase + p;
    if (m >= a.M) continue;
    const v4f lo = *reinterpret_cast<const v4f*>(wl + gpos(p, 2 * q));
    const v4f hi = *reinterpret_cast<const v4f*>(wl + gpos(p, 2 * q + 1));
    const float xs = ep.xscale ? ep.xscale[m / ohw] : ep.xs_const;
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    float ad[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (ep.add8) {          // residual (conv + sum, then ReLU): the shortcut's int8 tensor in its own scale
      const int8_t* ap = ep.add8 + (size_t)m * ep.add_ld + n;
      if (full8 && ((reinterpret_cast<uintptr_t>(ap) & 7) == 0)) {
        const v2u u = *reinterpret_cast<const v2u*>(ap);
#pragma unroll
        for (int e = 0; e < 8; ++e) ad[e] = (float)(int8_t)((u[e >> 2] >> (8 * (e & 3))) & 0xff) * ep.add_scale;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) ad[e] = n + e < a.Ncol ? (float)ap[e] * ep.add_scale : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = v[e] * xs * wsc[e] + bs[e] + ad[e];
      if (a.relu) v[e] = fmaxf(v[e], 0.f);
    }
    const size_t off = (size_t)m * a.ldo + n;
    if (ep.out_mode == 2) {
      int8_t* o = reinterpret_cast<int8_t*>(a.out) + off;
      unsigned pk[2] = {0u, 0u};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int qv = max(-127, min(127, __float2int_rn(v[e] * ep.out_inv)));
        pk[e >> 2] |= (unsigned)(qv & 0xff) << (8 * (e & 3));
      }
      if (full8 && (off & 7) == 0) {
        *reinterpret_cast<v2u*>(o) = v2u{pk[0], pk[1]};
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (n + e < a.Ncol) o[e] = (int8_t)((pk[e >> 2] >> (8 * (e & 3))) & 0xff);
      }
    } else if (ep.out_mode == 1) {
      float* o = reinterpret_cast<float*>(a.out) + off;
      if (full8 && (off & 3) == 0) {
        *reinterpret_cast<v4f*>(o) = v4f{v[0], v[1], v[2], v[3]};
        *reinterpret_cast<v4f*>(o + 4) = v4f{v[4], v[5], v[6], v[7]};
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (n + e < a.Ncol) o[e] = v[e];
      }
    } else {
      bf16_t* o = a.out + off;
      if (full8 && (off & 7) == 0) {
        *reinterpret_cast<v4u*>(o) = v4u{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (n + e < a.Ncol) o[e] = f2bf(v[e]);
      }
    }
  }
}

// int8 conv epilogue of one wave's TM x TN accumulator tile, in NH row chunks through the wave-private LDS slice wl:
// dequantize (x scale per sample x per-channel weight scale), bias, int8 residual addend, ReLU, then int8 (requantized
// with the consumer's scale), fp32 or bf16 stores; each lane finishes CPL channels of one pixel (CPL = 16: one
// 16-byte int8 store / addend load per lane instead of two 8-byte ones).
template <int MI, int NI, int TM, int TN, int NH, int CPL>
__device__ __forceinline__ void i8_tile_epilogue(const ConvArgs& a, const I8Epi& ep, v4i (&acc)[MI][NI], int mbase,
                                                 int nbase, int lane, float* wl) {
  constexpr int GR = TN / 4, LPR = TN / CPL, PPI = 64 / LPR, NR = TM / PPI, MIH = MI / NH, NRH = NR / NH;
  const int ohw = a.OH * a.OW;
  constexpr int GPL = CPL / 4;   // fp32 granules per lane
  auto gpos = [](int p, int g) { return (p * GR + (g ^ (p & (GR - 1)))) * 4; };
  const int q = lane % LPR;
  const int n = nbase + q * CPL;
  const bool nok = n < a.Ncol;
  const bool full = n + CPL <= a.Ncol;
  float wsc[CPL], bs[CPL];
#pragma unroll
  for (int e = 0; e < CPL; ++e) {
    const bool ok = n + e < a.Ncol;
    wsc[e] = ok ? ep.wscale[n + e] : 0.f;
    bs[e] = (ok && a.bias) ? a.bias[n + e] : 0.f;
  }
#pragma unroll
  for (int h = 0; h < NH; ++h) {
#pragma unroll
    for (int i = 0; i < MIH; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const v4i v = acc[h * MIH + i][j];
        *reinterpret_cast<v4f*>(wl + gpos(i * 16 + (lane & 15), j * 4 + (lane >> 4))) =
            v4f{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes landed (wave-private slice)
#pragma unroll
    for (int r = 0; r < NRH; ++r) {
      const int p = r * PPI + lane / LPR;
      const int m = mbase + h * (TM / NH) + p;
      float v[CPL];
#pragma unroll
      for (int g = 0; g < GPL; ++g) {
        const v4f t = *reinterpret_cast<const v4f*>(wl + gpos(p, GPL * q + g));
        v[4 * g] = t[0]; v[4 * g + 1] = t[1]; v[4 * g + 2] = t[2]; v[4 * g + 3] = t[3];
      }
      if (m >= a.M || !nok) continue;
      const float xs = ep.xscale ? ep.xscale[m / ohw] : ep.xs_const;
      float ad[CPL];
#pragma unroll
      for (int e = 0; e < CPL; ++e) ad[e] = 0.f;
      if (ep.add8) {
        const int8_t* ap = ep.add8 + (size_t)m * ep.add_ld + n;
        if (full && ((reinterpret_cast<uintptr_t>(ap) & (CPL - 1)) == 0)) {
          unsigned u[CPL / 4];
          if constexpr (CPL == 16) {
            const v4u w = *reinterpret_cast<const v4u*>(ap);
            u[0] = w[0]; u[1] = w[1]; u[2] = w[2]; u[3] = w[3];
          } else {
            const v2u w = *reinterpret_cast<const v2u*>(ap);
            u[0] = w[0]; u[1] = w[1];
          }
#pragma unroll
          for (int e = 0; e < CPL; ++e) ad[e] = (float)(int8_t)((u[e >> 2] >> (8 * (e & 3))) & 0xff) * ep.add_scale;
        } else {
#pragma unroll
          for (int e = 0; e < CPL; ++e) ad[e] = n + e < a.Ncol ? (float)ap[e] * ep.add_scale : 0.f;
        }
      }
#pragma unroll
      for (int e = 0; e < CPL; ++e) {
        v[e] = v[e] * xs * wsc[e] + bs[e] + ad[e];
        if (a.relu) v[e] = fmaxf(v[e], 0.f);
      }
      const size_t off = (size_t)m * a.ldo + n;
      if (ep.out_mode == 2) {
        int8_t* o = reinterpret_cast<int8_t*>(a.out) + off;
        unsigned pk[CPL / 4];
#pragma unroll
        for (int g = 0; g < CPL / 4; ++g) pk[g] = 0u;
#pragma unroll
        for (int e = 0; e < CPL; ++e) {
          const int qv = max(-127, min(127, __float2int_rn(v[e] * ep.out_inv)));
          pk[e >> 2] |= (unsigned)(qv & 0xff) << (8 * (e & 3));
        }
        if (full && (reinterpret_cast<uintptr_t>(o) & (CPL - 1)) == 0) {
          if constexpr (CPL == 16) *reinterpret_cast<v4u*>(o) = v4u{pk[0], pk[1], pk[2], pk[3]};
          else *reinterpret_cast<v2u*>(o) = v2u{pk[0], pk[1]};
        } else {
#pragma unroll
          for (int e = 0; e < CPL; ++e)
            if (n + e < a.Ncol) o[e] = (int8_t)((pk[e >> 2] >> (8 * (e & 3))) & 0xff);
        }
      } else if (ep.out_mode == 1) {
        float* o = reinterpret_cast<float*>(a.out) + off;
        if (full && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
#pragma unroll
          for (int g = 0; g < CPL / 4; ++g)
            *reinterpret_cast<v4f*>(o + 4 * g) = v4f{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]};
        } else {
#pragma unroll
          for (int e = 0; e < CPL; ++e)
            if (n + e < a.Ncol) o[e] = v[e];
        }
      } else {
        bf16_t* o = a.out + off;
        if (full && (reinterpret_cast<uintptr_t>(o) & 15) == 0) {
#pragma unroll
          for (int g = 0; g < CPL / 8; ++g)
            *reinterpret_cast<v4u*>(o + 8 * g) = v4u{pack2bf(v[8 * g], v[8 * g + 1]), pack2bf(v[8 * g + 2], v[8 * g + 3]),
                                                     pack2bf(v[8 * g + 4], v[8 * g + 5]), pack2bf(v[8 * g + 6], v[8 * g + 7])};
        } else {
#pragma unroll
          for (int e = 0; e < CPL; ++e)
            if (n + e < a.Ncol) o[e] = f2bf(v[e]);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // the slice is rewritten by the next half
  }
}

// Register-direct variant of i8_tile_epilogue: the i8 MFMA's D[n][m] layout already gives a lane 4 consecutive
// channels of one pixel per 16 x 16 tile, so each tile is finished in registers and stored as one 4-byte int8 group
// (8-byte bf16 / 16-byte fp32) per lane — no LDS round trip, no barrier — with the per-channel factors folded once:
// q = rn(acc * (xs * wsc * out_inv) + bias * out_inv + add * add_scale * out_inv). Needs Ncol % 4 == 0 and
// ldo % 4 == 0 (4-byte aligned groups); the caller checks (i8_direct_ok).
template <int MI, int NI>
__device__ __forceinline__ void i8_tile_epilogue_direct(const ConvArgs& a, const I8Epi& ep, v4i (&acc)[MI][NI],
                                                        int mbase, int nbase, int lane) {
  const int ohw = a.OH * a.OW;
  const int nl = 4 * (lane >> 4), ml = lane & 15;
  const bool q8 = ep.out_mode == 2;
  const float oi = q8 ? ep.out_inv : 1.f;
  float ws[NI][4], bs[NI][4];
#pragma unroll
  for (int j = 0; j < NI; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int n = nbase + j * 16 + nl + e;
      const bool ok = n < a.Ncol;
      ws[j][e] = ok ? ep.wscale[n] * oi : 0.f;
      bs[j][e] = (ok && a.bias) ? a.bias[n] * oi : 0.f;
    }
  const float as = ep.add_scale * oi;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int m = mbase + i * 16 + ml;
    if (m >= a.M) continue;
    const float xs = ep.xscale ? ep.xscale[m / ohw] : ep.xs_const;
    unsigned addw[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) {     // residual groups first, all in flight before the first store
      const int n = nbase + j * 16 + nl;
      addw[j] = (ep.add8 && n < a.Ncol) ? *reinterpret_cast<const unsigned*>(ep.add8 + (size_t)m * ep.add_ld + n) : 0u;
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int n = nbase + j * 16 + nl;
      if (n >= a.Ncol) continue;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = (float)acc[i][j][e] * (xs * ws[j][e]) + bs[j][e];
        if (ep.add8) v[e] += (float)(int8_t)((addw[j] >> (8 * e)) & 0xff) * as;
        if (a.relu) v[e] = fmaxf(v[e], 0.f);
      }
      const size_t off = (size_t)m * a.ldo + n;
      if (q8) {
        unsigned pk = 0u;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk |= (unsigned)(max(-127, min(127, __float2int_rn(v[e]))) & 0xff) << (8 * e);
        *reinterpret_cast<unsigned*>(reinterpret_cast<int8_t*>(a.out) + off) = pk;
      } else if (ep.out_mode == 1) {
        *reinterpret_cast<v4f*>(reinterpret_cast<float*>(a.out) + off) = v4f{v[0], v[1], v[2], v[3]};
      } else {
        *reinterpret_cast<v2u*>(a.out + off) = v2u{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      }
    }
  }
}

// 128 x 128 int8 tile with the counted-vmcnt pipeline of conv_nt_g4_kernel (conv_igemm.hip): 64-byte LDS rows (one
// i8 MFMA K-step of 64 = four 16-byte granules, slot g ^ ((r >> 1) & 3)), THREE stages of 16 KB with two K-steps in
// flight across every raw s_barrier (the 2-stage kernel above drains its DMA queue with __syncthreads every
// 128-byte step), 3 workgroups per CU. Tap table behind the stages. Fast-K only (Cs % 64 == 0: a K-step lies in one
// tap). The epilogue is conv_i8_glds_kernel's, run in two row halves so a wave's fp32 slice fits the stages.
// Tiles: 128 x 128 (2 x 2 waves) or, for the narrow layers (Ncol <= 64 / <= 32), 256 x 64 / 256 x 32 with the four
// waves stacked along M (as conv_i8_glds_kernel).
// FASTK = false (Cs % 64 != 0: Inception's 48 / 80 / 96 / 160 / ...-channel inputs, padded to 16): every lane resolves
// the tap of its own 16-channel granule from the LDS tap table; the K tail past Kdim loads zeros.
// NS_ = 2 (short-K variant, Kdim <= 128: at most two K-steps, no ring): two 16 KB stages and the epilogue in four row
// chunks, so 4 workgroups share a CU instead of 3 — these layers are one or two K-steps per tile and latency-bound.
template <int BM, int BN, int WGM, int WGN, bool FASTK = true, int CPL = 8, bool DIRECT = false, int NS_ = 3>
__global__ __launch_bounds__(256, NS_ == 2 ? 4 : ((BM + (BN + 63) / 64 * 64) * 64 * 3 <= 52 * 1024 ? 3 : 2)) void
conv_i8_g3_kernel(ConvArgs a, I8Epi ep) {
  constexpr int BKB = 64, NS = NS_;
  constexpr int TM = BM / WGM, TN = BN / WGN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int AI = BM / 64, BI = (BN + 63) / 64;   // DMA instructions per thread per stage (4 waves x 16 rows)
  constexpr int STAGE = (BM + BI * 64) * BKB;         // bytes (B region rounded up to the 64 rows one DMA pass fills)
  constexpr int L = AI + BI;
  constexpr int NH = NS == 2 ? 4 : 2;
  static_assert(NS == 2 || NS == 3, "stage ring of three, or the short-K pair");
  static_assert(4 * (TM / NH) * TN * 4 <= NS * STAGE, "epilogue chunk must fit the stages");
  __shared__ __attribute__((aligned(1024))) uint8_t lds[NS * STAGE + 6 * CONV_MAX_TAPS];
  short* taps = reinterpret_cast<short*>(lds + NS * STAGE);
  const uint8_t* src = reinterpret_cast<const uint8_t*>(a.src);
  const uint8_t* wt = reinterpret_cast<const uint8_t*>(a.wt);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int tiles_n = (a.Ncol + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (a.Kdim + BKB - 1) / BKB;

  const int rsub = lane >> 2;
  const int gsrc = (lane & 3) ^ ((rsub >> 1) & 3);
  int a_pix[AI], a_h[AI], a_w[AI];
  const int ohw = a.OH * a.OW;
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int m = m0 + (j * 4 + wave) * 16 + rsub;
    if (m < a.M) {
      const int nb = m / ohw, rem = m - nb * ohw;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      a_pix[j] = nb * a.Hs * a.Ws;
      a_h[j] = oh * a.mul_h;
      a_w[j] = ow * a.mul_w;
    } else {
      a_pix[j] = 0; a_h[j] = -(1 << 28); a_w[j] = -(1 << 28);
    }
  }
  const uint8_t* wrow[BI];
  bool bvalid[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int nl = (j * 4 + wave) * 16 + rsub;     // tile row; rows past BN (BN = 32) load into a spare slot
    const int n = n0 + nl;
    bvalid[j] = nl < BN && n < a.Ncol;
    wrow[j] = wt + (size_t)(bvalid[j] ? n : 0) * a.ldw + (FASTK ? gsrc * 16 : 0);
  }
  if (tid < a.ntaps) {
    taps[tid] = a.tap_h[tid];
    taps[CONV_MAX_TAPS + tid] = a.tap_w[tid];
    taps[2 * CONV_MAX_TAPS + tid] = a.tap_k[tid];
  }
  __syncthreads();   // tap table visible (no DMA outstanding yet)

  auto issue = [&](int kt, int buf) {
    const int k0 = kt * BKB;
    int th, tw, wk, c;
    bool kv = true;
    if constexpr (FASTK) {
      const int t = k0 / a.Cs;
      const int cin = k0 - t * a.Cs;
      th = taps[t]; tw = taps[CONV_MAX_TAPS + t];
      wk = taps[2 * CONV_MAX_TAPS + t] * a.Cs + cin;
      c = cin + gsrc * 16;
    } else {
      const int kk = k0 + gsrc * 16;
      kv = kk < a.Kdim;
      const int kc = kv ? kk : 0;
      const int t = kc / a.Cs;
      c = kc - t * a.Cs;
      th = taps[t]; tw = taps[CONV_MAX_TAPS + t];
      wk = taps[2 * CONV_MAX_TAPS + t] * a.Cs + c;
    }
    uint8_t* A = lds + buf * STAGE;
    uint8_t* B = A + BM * BKB;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int ch = a_h[j] + th, cw = a_w[j] + tw;
      const bool ok = kv && (unsigned)ch < (unsigned)a.Hs && (unsigned)cw < (unsigned)a.Ws;
      const uint8_t* g = ok ? src + (size_t)(a_pix[j] + ch * a.Ws + cw) * a.Cs + c : g_zero16;
      glds16(g, (LDS_PTR(void))(A + (j * 4 + wave) * 16 * BKB));
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const uint8_t* g = (bvalid[j] && kv) ? wrow[j] + wk : g_zero16;
      glds16(g, (LDS_PTR(void))(B + (j * 4 + wave) * 16 * BKB));
    }
  };
  const int foff = (lane & 15) * BKB + ((((lane >> 4) ^ ((lane >> 1) & 3))) << 4);

  v4i acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4i{0, 0, 0, 0};

  issue(0, 0);
  if (nk > 1) {
    issue(1, 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    const bool more2 = NS == 3 && kt + 2 < nk;   // NS == 2: the caller guarantees nk <= 2
    if (more2) issue(kt + 2, cur == 0 ? 2 : cur - 1);
    const uint8_t* A = lds + cur * STAGE;
    const uint8_t* B = A + BM * BKB;
    v4i fa[MI], fb[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) fb[j] = *reinterpret_cast<const v4i*>(B + (wn * TN + j * 16) * BKB + foff);
#pragma unroll
    for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const v4i*>(A + (wm * TM + i * 16) * BKB + foff);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fb[j], fa[i], acc[i][j], 0, 0, 0);
    if (more2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(L) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }

  // ---- epilogue: in registers (DIRECT), or conv_i8_glds_kernel's in NH row halves through a wave-private LDS slice
  if constexpr (DIRECT)
    i8_tile_epilogue_direct<MI, NI>(a, ep, acc, m0 + wm * TM, n0 + wn * TN, lane);
  else
    i8_tile_epilogue<MI, NI, TM, TN, NH, CPL>(a, ep, acc, m0 + wm * TM, n0 + wn * TN, lane,
                                             reinterpret_cast<float*>(lds) + wave * (TM / NH) * TN);
}

// 256 x 256 int8 tile on the phase-interleaved schedule of conv_nt_p8_kernel (conv_igemm.hip: pieces, phases, counted
// waits, wave-group stagger — see there): 8 waves of 128 x 64, two 64 KB LDS buffers of four 16 KB pieces of 128 rows
// x 128 B. A 128-byte row is one K-tile of 128 int8 = two i8 MFMA K-steps of 64, so the byte-level schedule is the bf16
// kernel's unchanged; the MFMA is v_mfma_i32_16x16x64_i8 and the epilogue i8_tile_epilogue (4 row chunks through the
// buffers). Fast-K only (Cs % 128 == 0: a K-tile lies in one tap).
template <bool DIRECT>
__global__ __launch_bounds__(512, 2) void conv_i8_p8_kernel(ConvArgs a, I8Epi ep) {
  constexpr int BM = 256, BN = 256, BKB = 128;
  constexpr int WGM = 2, WGN = 4;
  constexpr int TM = BM / WGM, TN = BN / WGN;      // 128 x 64 per wave
  constexpr int MI = TM / 16, NI = TN / 16;        // 8 x 4 MFMA tiles
  constexpr int PIECE = 128 * BKB;                 // bytes (16 KB)
  constexpr int BUF = 4 * PIECE;                   // 64 KB
  constexpr int NH = 4;
  static_assert(8 * (TM / NH) * TN * 4 <= 2 * BUF, "epilogue chunk must fit the buffers");
  __shared__ __attribute__((aligned(1024))) uint8_t lds[2 * BUF + 6 * CONV_MAX_TAPS];
  short* taps = reinterpret_cast<short*>(lds + 2 * BUF);
  const uint8_t* src8 = reinterpret_cast<const uint8_t*>(a.src);
  const uint8_t* wt8 = reinterpret_cast<const uint8_t*>(a.wt);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int tiles_n = (a.Ncol + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = a.Kdim / BKB;

  // DMA geometry as conv_nt_p8_kernel: instruction j of wave w fills piece rows (j * 8 + w) * 8 .. +8; lane -> row
  // + (lane >> 3), slot lane & 7 holding granule (lane & 7) ^ (lane >> 3)
  const int gsrc = (lane & 7) ^ (lane >> 3);
  const int ohw = a.OH * a.OW;
  int a_pix[4], a_h[4], a_w[4];
  const uint8_t* wrow[4];
  bool bvalid[4];
#pragma unroll
  for (int q2 = 0; q2 < 4; ++q2) {
    const int q = q2 >> 1, lr = ((q2 & 1) * 8 + wave) * 8 + (lane >> 3);
    const int m = m0 + (lr >> 6) * 128 + q * 64 + (lr & 63);
    if (m < a.M) {
      const int nb = m / ohw, rem = m - nb * ohw;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      a_pix[q2] = nb * a.Hs * a.Ws;
      a_h[q2] = oh * a.mul_h;
      a_w[q2] = ow * a.mul_w;
    } else {
      a_pix[q2] = 0; a_h[q2] = -(1 << 28); a_w[q2] = -(1 << 28);
    }
    const int n = n0 + (lr >> 5) * 64 + q * 32 + (lr & 31);
    bvalid[q2] = n < a.Ncol;
    wrow[q2] = wt8 + (size_t)(bvalid[q2] ? n : 0) * a.ldw + gsrc * 16;
  }
  if (tid < a.ntaps) {
    taps[tid] = a.tap_h[tid];
    taps[CONV_MAX_TAPS + tid] = a.tap_w[tid];
    taps[2 * CONV_MAX_TAPS + tid] = a.tap_k[tid];
  }
  __syncthreads();

  auto issue = [&](int kt, int buf, int P) {
    const int k0 = kt * BKB;
    const int t = k0 / a.Cs;
    const int cin = k0 - t * a.Cs;
    uint8_t* base = lds + buf * BUF + P * PIECE;
    const int q = P >> 1;
    if ((P & 1) == 0) {
      const int th = taps[t], tw = taps[CONV_MAX_TAPS + t];
      const int c = cin + gsrc * 16;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q2 = q * 2 + j;
        const int ch = a_h[q2] + th, cw = a_w[q2] + tw;
        const bool ok = (unsigned)ch < (unsigned)a.Hs && (unsigned)cw < (unsigned)a.Ws;
        const uint8_t* g = ok ? src8 + (size_t)(a_pix[q2] + ch * a.Ws + cw) * a.Cs + c : g_zero16;
        glds16(g, (LDS_PTR(void))(base + (j * 8 + wave) * 8 * BKB));
      }
    } else {
      const int wk = taps[2 * CONV_MAX_TAPS + t] * a.Cs + cin;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q2 = q * 2 + j;
        const uint8_t* g = bvalid[q2] ? wrow[q2] + wk : g_zero16;
        glds16(g, (LDS_PTR(void))(base + (j * 8 + wave) * 8 * BKB));
      }
    }
  };
  // fragment of K-step kh (64 int8 = 4 granules): granule kh * 4 + (lane >> 4) of row (lane & 15) at slot ^ (lane & 7)
  const int fo0 = (lane & 15) * BKB + (((lane >> 4)) ^ (lane & 7)) * 16;
  const int fo1 = (lane & 15) * BKB + ((4 + (lane >> 4)) ^ (lane & 7)) * 16;
  const int a_row = wm * 64 * BKB;
  const int b_row = wn * 32 * BKB;

  v4i acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  v4i fa[4][2], fb[NI][2];
  auto quad = [&](int ib, int jb) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ib + i][jb + j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fb[jb + j][kh], fa[i][kh], acc[ib + i][jb + j], 0, 0, 0);
  };
  auto read_a = [&](const uint8_t* P) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i][0] = *reinterpret_cast<const v4i*>(P + a_row + i * 16 * BKB + fo0);
      fa[i][1] = *reinterpret_cast<const v4i*>(P + a_row + i * 16 * BKB + fo1);
    }
  };
  auto read_b = [&](const uint8_t* P, int jb) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fb[jb + j][0] = *reinterpret_cast<const v4i*>(P + b_row + j * 16 * BKB + fo0);
      fb[jb + j][1] = *reinterpret_cast<const v4i*>(P + b_row + j * 16 * BKB + fo1);
    }
  };
  auto compute = [&](int ib, int jb) {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    quad(ib, jb);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  };

  if (nk > 0) {
    issue(0, 0, 0); issue(0, 0, 1); issue(0, 0, 3); issue(0, 0, 2);
  }
  if (nk > 1) {
    issue(1, 1, 0); issue(1, 1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();   // stagger

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const uint8_t* L = lds + cur * BUF;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    if (n1) issue(kt + 1, cur ^ 1, 3);
    read_a(L); read_b(L + PIECE, 0);
    if (n1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    compute(0, 0);
    if (n1) issue(kt + 1, cur ^ 1, 2);
    read_b(L + 3 * PIECE, 2);
    if (n1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    compute(0, 2);
    if (n2) issue(kt + 2, cur, 0);
    read_a(L + 2 * PIECE);
    compute(4, 2);
    if (n2) issue(kt + 2, cur, 1);
    if (n2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    compute(4, 0);
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();   // balance the stagger
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (DIRECT) {
    i8_tile_epilogue_direct<MI, NI>(a, ep, acc, m0 + wm * TM, n0 + wn * TN, lane);
  } else {
    __syncthreads();                          // every wave is done with the buffers before the epilogue reuses them
    i8_tile_epilogue<MI, NI, TM, TN, NH, 16>(a, ep, acc, m0 + wm * TM, n0 + wn * TN, lane,
                                             reinterpret_cast<float*>(lds) + wave * (TM / NH) * TN);
  }
}

// int8 rows [rows][C] from src (row stride lds) into dst (row stride ldd): a concat input that was not produced in place
__global__ __launch_bounds__(256) void copy_rows_i8_kernel(const int8_t* __restrict__ src, int8_t* __restrict__ dst,
                                                           long rows, int C, long lds, long ldd) {
  const long total = rows * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / C;
    const int c = (int)(i - r * C);
    dst[r * ldd + c] = src[r * lds + c];
  }
}

// ---------------------------------------------------------------------------------- int8 pooling / quantize
// NHWC int8 max / average pooling over [N][H][W][Cp] -> [N][OH][OW][ldo] (rows `ldo` apart, so a pooling branch
// of an int8 concat writes its slice in place). One lane = 16 channels of one output pixel (16-byte loads); the
// scale is unchanged (max of int8 values / rounded mean stay in [-127, 127]). Average: count_pad selects whether
// padded taps count in the divisor (Caffe / BigDL default) or not.
// K3 (3x3 windows, Inception's branch pools and reductions): the nine window granules are loaded unconditionally
// (out-of-image taps read a zero granule) before any is used, so a lane keeps nine L2/HBM requests in flight
// instead of nine dependent round trips.
template <bool K3>
__global__ void pool_i8_kernel(const int8_t* __restrict__ x, int8_t* __restrict__ y, int N, int H, int W, int Cp,
                               int OH, int OW, int kh, int kw, int sh, int sw, int ph, int pw, int avg, int count_pad,
                               long ldo) {
  const int G = Cp >> 4;
  if constexpr (K3) {
    const long total = (long)N * OH * OW * G;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
      const int g = (int)(i % G);
      const long pix = i / G;
      const int ow = (int)(pix % OW), oh = (int)((pix / OW) % OH), nb = (int)(pix / ((long)OW * OH));
      const int h0 = oh * sh - ph, w0 = ow * sw - pw;
      v4u u[9];
      int cnt = 0;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int hh = h0 + t / 3, ww = w0 + t % 3;
        const bool inb = (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
        cnt += (avg && count_pad) ? (hh < H + ph && ww < W + pw) : inb;
        const int8_t* src = inb ? x + (((size_t)nb * H + hh) * W + ww) * Cp + g * 16
                                : reinterpret_cast<const int8_t*>(g_zero16);
        u[t] = *reinterpret_cast<const v4u*>(src);
        if (!avg && !inb) u[t] = v4u{0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u};   // -128: never the max
      }
      v4u o = {0u, 0u, 0u, 0u};
      const float inv = cnt > 0 ? 1.f / (float)cnt : 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        int acc = avg ? 0 : -128;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int v = (int)(int8_t)((u[t][e >> 2] >> (8 * (e & 3))) & 0xff);
          acc = avg ? acc + v : max(acc, v);
        }
        int v = avg ? __float2int_rn((float)acc * inv) : (cnt > 0 ? acc : 0);
        v = max(-127, min(127, v));
        o[e >> 2] |= (unsigned)(v & 0xff) << (8 * (e & 3));
      }
      *reinterpret_cast<v4u*>(y + pix * ldo + g * 16) = o;
    }
    return;
  }
  const long total = (long)N * OH * OW * G;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int g = (int)(i % G);
    const long pix = i / G;
    const int ow = (int)(pix % OW), oh = (int)((pix / OW) % OH), nb = (int)(pix / ((long)OW * OH));
    const int h0 = oh * sh - ph, w0 = ow * sw - pw;
    int acc[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[e] = avg ? 0 : -128;
    int cnt = 0;
    for (int r = 0; r < kh; ++r) {
      const int hh = h0 + r;
      for (int s = 0; s < kw; ++s) {
        const int ww = w0 + s;
        const bool inb = (unsigned)hh < (unsigned)H && (unsigned)ww < (unsigned)W;
        if (avg && count_pad) {
          if (hh < H + ph && ww < W + pw) ++cnt;
        } else if (inb) {
          ++cnt;
        }
        if (!inb) continue;
        const v4u u = *reinterpret_cast<const v4u*>(x + (((size_t)nb * H + hh) * W + ww) * Cp + g * 16);
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int v = (int)(int8_t)((u[e >> 2] >> (8 * (e & 3))) & 0xff);
          acc[e] = avg ? acc[e] + v : max(acc[e], v);
        }
      }
    }
    v4u o = {0u, 0u, 0u, 0u};
    const float inv = cnt > 0 ? 1.f / (float)cnt : 0.f;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      int v = avg ? __float2int_rn((float)acc[e] * inv) : (cnt > 0 ? acc[e] : 0);
      v = max(-127, min(127, v));
      o[e >> 2] |= (unsigned)(v & 0xff) << (8 * (e & 3));
    }
    *reinterpret_cast<v4u*>(y + pix * ldo + g * 16) = o;
  }
}

// fp32 NCHW image batch -> int8 NHWC [N][H][W][Cp] with a static scale (graph input of an int8 plan); pad channels 0.
__global__ void quantize_nchw_f32_kernel(const float* __restrict__ x, int8_t* __restrict__ q, int N, int C, int HW,
                                         int Cp, float inv) {
  const long total = (long)N * HW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long nb = i / HW, p = i - nb * HW;
    const float* xs = x + nb * C * (long)HW + p;
    int8_t* o = q + i * Cp;
    for (int c0 = 0; c0 < Cp; c0 += 16) {
      v4u u = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int c = c0 + e;
        const int v = c < C ? max(-127, min(127, __float2int_rn(xs[(long)c * HW] * inv))) : 0;
        u[e >> 2] |= (unsigned)(v & 0xff) << (8 * (e & 3));
      }
      *reinterpret_cast<v4u*>(o + c0) = u;
    }
  }
}

// int8 stem (C <= 4 channels, width stride sw, S <= 8 width taps): the image is quantized straight into its width
// im2col, y[n][h][ow][e*4 + c] = q(x[n][c][h][ow*sw + e - pw]) (0 for e >= S, c >= C or outside the image), so one
// 32-byte row holds every width tap of output column ow and the stem becomes an R x 1 convolution over 32 int8
// "channels": a reduction of R * 32 instead of R * S * 16 (7x7: 224 vs 784; the bf16 stem's pixel pairs,
// stem.hip, do the same for 16-bit data).
__global__ __launch_bounds__(256) void quantize_wim2col_f32_kernel(const float* __restrict__ x, int8_t* __restrict__ y,
                                                                   int N, int C, int H, int W, int OW, int S, int sw,
                                                                   int pw, float inv) {
  const long total = (long)N * H * OW;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ow = (int)(i % OW);
    const long t = i / OW;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    const float* xb = x + ((size_t)n * C * H + h) * W;
    unsigned u[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      u[e] = 0u;
      const int w = ow * sw + e - pw;
      if (e < S && (unsigned)w < (unsigned)W) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (c < C) {
            const int v = max(-127, min(127, __float2int_rn(xb[(size_t)c * H * W + w] * inv)));
            u[e] |= (unsigned)(v & 0xff) << (8 * c);
          }
      }
    }
    v4u* o = reinterpret_cast<v4u*>(y + (size_t)i * 32);
    o[0] = v4u{u[0], u[1], u[2], u[3]};
    o[1] = v4u{u[4], u[5], u[6], u[7]};
  }
}

// bf16 NHWC [P][C] -> int8 [P][ldq] (written at a channel offset of a wider int8 buffer), static scale
__global__ void quantize_rows_bf16_kernel(const bf16_t* __restrict__ x, int8_t* __restrict__ q, long P, int C,
                                          long ldq, float inv) {
  const int G = C >> 3;
  const long total = P * G;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / G;
    const int g = (int)(i - p * G);
    const v4u u = *reinterpret_cast<const v4u*>(x + p * C + g * 8);
    unsigned pk[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int v0 = max(-127, min(127, __float2int_rn(lo_bf(u[e]) * inv)));
      const int v1 = max(-127, min(127, __float2int_rn(hi_bf(u[e]) * inv)));
      pk[e >> 1] |= ((unsigned)(v0 & 0xff) | ((unsigned)(v1 & 0xff) << 8)) << (16 * (e & 1));
    }
    *reinterpret_cast<v2u*>(q + p * ldq + g * 8) = v2u{pk[0], pk[1]};
  }
}

// int8 NHWC [P][ld] -> bf16 [P][C] (dequantize, for a float consumer of an int8 tensor)
__global__ void dequantize_rows_kernel(const int8_t* __restrict__ q, bf16_t* __restrict__ y, long P, int C, long ld,
                                       float scale) {
  const long total = P * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long p = i / C;
    const int c = (int)(i - p * C);
    y[i] = f2bf((float)q[p * ld + c] * scale);
  }
}

}  // namespace

namespace {
// BIGDL_I8_CPL (default 16): channels per lane in the int8 3-stage kernel's epilogue (16 = 16-byte int8 stores)
int g_i8_cpl = -1;
int i8_cpl() {
  if (g_i8_cpl < 0) {
    const char* e = getenv("BIGDL_I8_CPL");
    g_i8_cpl = e ? atoi(e) : 16;   // 16: ResNet-50 int8 4.19 -> 3.90 ms (profiles/r3_int8_epilogue_ab.txt)
  }
  return g_i8_cpl;
}

// BIGDL_I8_EPI (default 0): 1 = register-direct int8 epilogue where the output groups are 4-byte aligned. Measured
// slower: ResNet-50 int8 3.83 -> 5.11 ms (4-byte groups scattered over 16 pixel rows per store instruction vs the
// LDS-staged 16-byte rows; profiles/r4_int8_epilogue_direct_ab.txt)
int g_i8_epi = -1;
bool i8_direct_ok(const ConvArgs& a, const I8Epi& ep) {
  if (g_i8_epi < 0) {
    const char* e = getenv("BIGDL_I8_EPI");
    g_i8_epi = e ? atoi(e) : 0;
  }
  return g_i8_epi != 0 && a.Ncol % 4 == 0 && a.ldo % 4 == 0 && (ep.add8 == nullptr || ep.add_ld % 4 == 0) &&
         (ep.out_mode != 1 || a.ldo % 4 == 0);
}

// BIGDL_I8_SHORTK (default 0): 1 = the two-stage, 4-workgroups-per-CU 128 x 128 variant when Kdim <= 128 (fast-K);
// 2: that variant with the 8-channel epilogue (106 VGPRs, no spill, vs 16 spilled VGPRs with 16 channels per lane).
// Measured: 1 slower (ResNet-50 int8 3.83 -> 4.22 ms), 2 neutral (3.85 ms) — the one-K-step layers are not
// occupancy-bound (profiles/r4_shortk_ab.txt)
int g_i8_shortk = -1;
bool i8_shortk() {
  if (g_i8_shortk < 0) {
    const char* e = getenv("BIGDL_I8_SHORTK");
    g_i8_shortk = e ? atoi(e) : 0;
  }
  return g_i8_shortk != 0;
}

// Streaming 1x1 int8 kernel: the structure of conv_nt_s1_kernel (conv_igemm.hip) on v_mfma_i32_16x16x64_i8 for the
// one-tap int8 GEMMs of the static int8 plan (identity pixel mapping, Kdim = Cs in {64, 128, 256} int8 channels,
// Ncol % 64 == 0, identity output rows). Persistent workgroups (2 per CU) stride over pixel tiles of one channel
// block; a wave's weights stay in VGPRs as i8 MFMA fragments for the whole launch (K 256: 64 VGPRs); operand tiles
// come straight from HBM into VGPRs two tiles ahead; the int32 tile is parked as fp32 in a wave-private LDS slice
// (16-byte granules XOR-swizzled by pixel) and re-read as 16 channels of one pixel per lane, so the epilogue
// (y = acc * s_x * s_w[n] + bias (+ int8 residual * s_add), ReLU, bf16 / fp32 / requantized int8) runs once per
// 16 outputs with the per-channel factors held in registers for the whole launch, and stores whole 16-byte groups.
// Semantics are i8_tile_epilogue's (CPL = 16).
template <int K, int CG, int BMW, int OUT, bool ADD>
__global__ __launch_bounds__(256, 2) void conv_i8_s1_kernel(ConvArgs a, I8Epi ep) {
  constexpr int KF = K / 64, MI = BMW / 16, PGN = 4 / CG, BM = BMW * PGN;
  constexpr int NR = BMW / 16;                     // row passes: 16 pixels x 4 lanes (16 channels each)
  __shared__ __attribute__((aligned(16))) float lds[4 * BMW * 64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cg = wave % CG, pg = wave / CG;
  const int nchb = a.Ncol / (64 * CG);
  const int chb = blockIdx.x % nchb, wgi = blockIdx.x / nchb, ngr = gridDim.x / nchb;
  const int c0 = (chb * CG + cg) * 64;
  const int ntiles = (a.M + BM - 1) / BM;
  float* wl = lds + wave * BMW * 64;
  const int q = lane & 3;                          // row phase: channels c0 + 16 q .. + 15
  const int n = c0 + 16 * q;
  const int8_t* W8 = reinterpret_cast<const int8_t*>(a.wt);
  const int8_t* X8 = reinterpret_cast<const int8_t*>(a.src);
  const int ohw = a.OH * a.OW;

  v4i wf[4][KF];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int kk = 0; kk < KF; ++kk)
      wf[j][kk] = *reinterpret_cast<const v4i*>(W8 + (size_t)(c0 + 16 * j + (lane & 15)) * a.ldw + 64 * kk +
                                                16 * (lane >> 4));
  const float oi = OUT == 2 ? ep.out_inv : 1.f;
  // 16-byte loads, the bias through a buffer resource (0 bytes without one): per-element `a.bias ? a.bias[..] : 0`
  // was 16 waited round trips at the start of every workgroup
  float wsc[16], bs[16];
  {
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.bias), (short)0,
                                                                        a.bias ? a.Ncol * 4 : 0, 0x00020000);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const v4f w = *reinterpret_cast<const v4f*>(ep.wscale + n + 4 * g);
      const v4f b = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rb, (unsigned)((n + 4 * g) * 4), 0, 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        wsc[4 * g + e] = w[e] * oi;
        bs[4 * g + e] = b[e] * oi;
      }
    }
  }
  const float as = ep.add_scale * oi;
  const __amdgpu_buffer_rsrc_t rxs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ep.xscale), (short)0,
                                                                       ep.xscale ? a.Nb * 4 : 0, 0x00020000);
  const float xs0 = ep.xscale ? 0.f : ep.xs_const;
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
      a.out, (short)0, (int)(((size_t)(a.M - 1) * a.ldo + a.Ncol) * (OUT == 2 ? 1 : OUT == 1 ? 4 : 2)), 0x00020000);

  auto load = [&](v4i (&af)[MI][KF], int t) {
    const int p0 = t * BM + pg * BMW;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = min(p0 + 16 * i + (lane & 15), a.M - 1);
#pragma unroll
      for (int kk = 0; kk < KF; ++kk)
        af[i][kk] = *reinterpret_cast<const v4i*>(X8 + (size_t)m * K + 64 * kk + 16 * (lane >> 4));
    }
  };

  auto compute_store = [&](v4i (&af)[MI][KF], int t) {
    const int p0 = t * BM + pg * BMW;
    v4u pad[ADD ? NR : 1];
    if constexpr (ADD) {
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) {
        const int m = min(p0 + rr * 16 + (lane >> 2), a.M - 1);
        pad[rr] = *reinterpret_cast<const v4u*>(ep.add8 + (size_t)m * ep.add_ld + n);
      }
    }
    v4i acc[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < KF; ++kk)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(wf[j][kk], af[i][kk], acc[i][j], 0, 0, 0);
    // D[n][m]: lane holds channels 16 j + 4 (lane >> 4) + e of pixel 16 i + (lane & 15): fp32 granule g = 4 j + qq
    // of a 16-granule (64-channel) row, at slot g ^ (p & 15)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = 16 * i + (lane & 15), g = 4 * j + (lane >> 4);
        const v4i v = acc[i][j];
        *reinterpret_cast<v4f*>(wl + (p * 16 + (g ^ (p & 15))) * 4) = v4f{(float)v[0], (float)v[1], (float)v[2], (float)v[3]};
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): wave-private slice
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int p = rr * 16 + (lane >> 2);
      const int m = p0 + p;
      float v[16];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const v4f t4 = *reinterpret_cast<const v4f*>(wl + (p * 16 + ((4 * q + g) ^ (p & 15))) * 4);
        v[4 * g] = t4[0]; v[4 * g + 1] = t4[1]; v[4 * g + 2] = t4[2]; v[4 * g + 3] = t4[3];
      }
      // branch-free row: per-sample scale through a buffer resource, tail rows stored out of range (a skipped row
      // or `xscale ? xscale[..] : c` was a wait at each join)
      const bool ok = m < a.M;
      const float xl = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                     rxs, ok ? (unsigned)(m / ohw * 4) : 0x7ffffff0u, 0, 0));
      const float xs = xl + xs0;         // xl reads 0 without per-sample scales: no select for the load to sink into
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        float y = v[e] * (xs * wsc[e]) + bs[e];
        if constexpr (ADD) y += (float)(int8_t)((pad[rr][e >> 2] >> (8 * (e & 3))) & 0xff) * as;
        if (a.relu) y = fmaxf(y, 0.f);
        v[e] = y;
      }
      constexpr int ESZ = OUT == 2 ? 1 : OUT == 1 ? 4 : 2;
      const unsigned off = ok ? (unsigned)(((size_t)m * a.ldo + n) * ESZ) : 0x7ffffff0u;
      if constexpr (OUT == 2) {
        unsigned pk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int e = 0; e < 16; ++e) pk[e >> 2] |= (unsigned)(max(-127, min(127, __float2int_rn(v[e]))) & 0xff) << (8 * (e & 3));
        __builtin_amdgcn_raw_buffer_store_b128(v4u{pk[0], pk[1], pk[2], pk[3]}, ro, off, 0, 0);
      } else if constexpr (OUT == 1) {
#pragma unroll
        for (int g = 0; g < 4; ++g)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v4f{v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]}),
                                                 ro, off, 16 * g, 0);
      } else {
#pragma unroll
        for (int g = 0; g < 2; ++g)
          __builtin_amdgcn_raw_buffer_store_b128(v4u{pack2bf(v[8 * g], v[8 * g + 1]), pack2bf(v[8 * g + 2], v[8 * g + 3]),
                                                     pack2bf(v[8 * g + 4], v[8 * g + 5]), pack2bf(v[8 * g + 6], v[8 * g + 7])},
                                                 ro, off, 16 * g, 0);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // the slice is rewritten by the next tile
  };

  v4i a0[MI][KF], a1[MI][KF], a2[MI][KF];
  int t = wgi;
  if (t < ntiles) load(a0, t);
  if (t + ngr < ntiles) load(a1, t + ngr);
  for (; t < ntiles; t += 3 * ngr) {
    if (t + 2 * ngr < ntiles) load(a2, t + 2 * ngr);
    compute_store(a0, t);
    if (t + ngr >= ntiles) break;
    if (t + 3 * ngr < ntiles) load(a0, t + 3 * ngr);
    compute_store(a1, t + ngr);
    if (t + 2 * ngr >= ntiles) break;
    if (t + 4 * ngr < ntiles) load(a1, t + 4 * ngr);
    compute_store(a2, t + 2 * ngr);
  }
}

int g_i8_s1 = -1;   // BIGDL_I8_S1 (default 1): the streaming 1x1 int8 kernel wherever it applies
bool i8_s1_applies(const ConvArgs& a, const I8Epi& ep) {
  if (g_i8_s1 < 0) {
    const char* e = getenv("BIGDL_I8_S1");
    g_i8_s1 = e ? atoi(e) : 1;
  }
  if (!g_i8_s1 || !a.ident_out || a.ntaps != 1 || a.tap_h[0] || a.tap_w[0] || a.tap_k[0]) return false;
  if (a.mul_h != 1 || a.mul_w != 1 || a.Hs != a.OH || a.Ws != a.OW) return false;
  if ((a.Kdim != 64 && a.Kdim != 128 && a.Kdim != 256) || a.Cs != a.Kdim || (a.Ncol % 64) || (a.ldw % 16)) return false;
  const int osz = ep.out_mode == 2 ? 1 : ep.out_mode == 1 ? 4 : 2;
  if ((a.ldo * osz) % 16 || (ep.add8 && (ep.add_ld % 16))) return false;
  // stores through a 32-bit buffer offset, below the out-of-range offset used for tail rows
  if (((size_t)(a.M - 1) * a.ldo + a.Ncol) * osz >= 0x7ff00000u) return false;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return al(a.src) && al(a.wt) && al(a.out) && al(ep.add8);
}

template <int K, int CG, int BMW, int OUT>
void launch_i8_s1_o(const ConvArgs& a, const I8Epi& ep, hipStream_t st) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int nchb = a.Ncol / (64 * CG);
  const int tiles = (a.M + BMW * (4 / CG) - 1) / (BMW * (4 / CG));
  int per = std::max(1, (2 * cus) / nchb);
  per = std::min(per, tiles);
  if (ep.add8) conv_i8_s1_kernel<K, CG, BMW, OUT, true><<<dim3(per * nchb), dim3(256), 0, st>>>(a, ep);
  else conv_i8_s1_kernel<K, CG, BMW, OUT, false><<<dim3(per * nchb), dim3(256), 0, st>>>(a, ep);
}

template <int K, int CG>
void launch_i8_s1_cg(const ConvArgs& a, const I8Epi& ep, hipStream_t st) {
  constexpr int BW = K == 256 ? 16 : 32;
  if (ep.out_mode == 2) launch_i8_s1_o<K, CG, BW, 2>(a, ep, st);
  else if (ep.out_mode == 1) launch_i8_s1_o<K, CG, BW, 1>(a, ep, st);
  else launch_i8_s1_o<K, CG, BW, 0>(a, ep, st);
}

void launch_i8_s1(const ConvArgs& a, const I8Epi& ep, hipStream_t st) {
  const int cg = (a.Ncol % 256 == 0) ? 4 : (a.Ncol % 128 == 0) ? 2 : 1;
#define I8S1_K(KK)                                 \
  if (cg == 4) launch_i8_s1_cg<KK, 4>(a, ep, st);   \
  else if (cg == 2) launch_i8_s1_cg<KK, 2>(a, ep, st); \
  else launch_i8_s1_cg<KK, 1>(a, ep, st);
  if (a.Kdim == 64) { I8S1_K(64) }
  else if (a.Kdim == 128) { I8S1_K(128) }
  else { I8S1_K(256) }
#undef I8S1_K
}

template <int BM, int BN, int WGM, int WGN>
void launch_i8_g3(int g, bool fk, const ConvArgs& a, const I8Epi& ep, hipStream_t st) {
  if constexpr (BM == 128 && BN == 128) {
    if (fk && a.Kdim <= 128 && i8_shortk() && !i8_direct_ok(a, ep)) {
      if (i8_cpl() == 16 && g_i8_shortk != 2) conv_i8_g3_kernel<BM, BN, WGM, WGN, true, 16, false, 2><<<g, 256, 0, st>>>(a, ep);
      else conv_i8_g3_kernel<BM, BN, WGM, WGN, true, 8, false, 2><<<g, 256, 0, st>>>(a, ep);
      return;
    }
  }
  if (fk && i8_direct_ok(a, ep)) {
    conv_i8_g3_kernel<BM, BN, WGM, WGN, true, 16, true><<<g, 256, 0, st>>>(a, ep);
    return;
  }
  if (i8_cpl() == 16 && BN / WGN >= 16) {
    if (fk) conv_i8_g3_kernel<BM, BN, WGM, WGN, true, 16><<<g, 256, 0, st>>>(a, ep);
    else conv_i8_g3_kernel<BM, BN, WGM, WGN, false, 16><<<g, 256, 0, st>>>(a, ep);
  } else {
    if (fk) conv_i8_g3_kernel<BM, BN, WGM, WGN, true, 8><<<g, 256, 0, st>>>(a, ep);
    else conv_i8_g3_kernel<BM, BN, WGM, WGN, false, 8><<<g, 256, 0, st>>>(a, ep);
  }
}

}  // namespace

extern "C" {

int bigdl_quantize_act(const void* x, int is_bf16, int8_t* q, float* amax, float* scale, int N, long P, int C,
                       int Cp, int static_amax, hipStream_t st) {
  const long per = P * C;
  if (!static_amax) {            // dynamic per-sample range; with static_amax the caller filled amax (calibrated)
    bigdl_fill_bytes(amax, 0, (long)sizeof(float) * N, st);
    const int bx = (int)std::min<long>((per / (is_bf16 && (per & 7) == 0 ? 8 : 1) + 255) / 256, 256);
    dim3 g1(bx > 0 ? bx : 1, N);
    if (is_bf16) amax_kernel<uint16_t><<<g1, 256, 0, st>>>((const uint16_t*)x, per, amax);
    else amax_kernel<float><<<g1, 256, 0, st>>>((const float*)x, per, amax);
  }
  if (is_bf16 && C == Cp && (C & 7) == 0) {
    const long per8 = per >> 3, total8 = (long)N * per8;
    const int blocks = (int)std::min<long>((total8 + 255) / 256, 16384);
    quantize8_bf16_kernel<<<blocks, 256, 0, st>>>((const v4u*)x, (v2u*)q, amax, scale, per8, N);
    HIP_LAUNCH_CHECK();
    return 0;
  }
  const long total = (long)N * P * Cp;
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  if (is_bf16) quantize_kernel<uint16_t><<<blocks, 256, 0, st>>>((const uint16_t*)x, q, amax, scale, P, C, Cp, N);
  else quantize_kernel<float><<<blocks, 256, 0, st>>>((const float*)x, q, amax, scale, P, C, Cp, N);
  HIP_LAUNCH_CHECK();
  return 0;
}

int g_i8_g3 = -1;
// BIGDL_I8_G3 (default 1): the 3-stage counted-vmcnt 128 x 128 int8 kernel for Ncol > 64, Cs % 64 == 0.
// 2: also the 256 x 128 tile (2 x 2 waves of 128 x 64: 32 i8 MFMAs per wave between barriers instead of 16, 2
// workgroups per CU) when its grid still fills two workgroups per CU; 3: the 256 x 128 tile always (tests).
static bool i8_g3() {
  if (g_i8_g3 < 0) {
    const char* e = getenv("BIGDL_I8_G3");
    g_i8_g3 = e ? atoi(e) : 1;
  }
  return g_i8_g3 != 0;
}
void bigdl_set_i8_g3(int v) { g_i8_g3 = v; }
// BIGDL_I8_P8 (default 1): the 256 x 256 phase-interleaved int8 kernel for Cs % 128 == 0, Kdim >= 1024, Ncol >= 256
// and >= 160 tiles (the bf16 kernel's rule); 2: whenever the shape allows (tests); 0: off
int g_i8_p8 = -1;
static bool i8_p8() {
  if (g_i8_p8 < 0) {
    const char* e = getenv("BIGDL_I8_P8");
    g_i8_p8 = e ? atoi(e) : 1;
  }
  return g_i8_p8 != 0;
}
void bigdl_set_i8_p8(int v) { g_i8_p8 = v; }
void bigdl_set_i8_s1(int v) { g_i8_s1 = v; }
void bigdl_set_i8_epi(int v) { g_i8_epi = v; }
void bigdl_set_i8_shortk(int v) { g_i8_shortk = v; }
void bigdl_set_i8_cpl(int v) { g_i8_cpl = v; }
int bigdl_get_i8_cpl() { return i8_cpl(); }
int bigdl_get_i8_g3() { return i8_g3() ? g_i8_g3 : 0; }

int bigdl_conv_i8(const ConvArgs* a, const float* xscale, float xs_const, const float* wscale, int out_mode,
                  float out_inv, const int8_t* add8, float add_scale, long add_ld, hipStream_t st) {
  if (a->Cs % 16 != 0 || a->Kdim != a->ntaps * a->Cs || a->ntaps < 1 || a->ntaps > CONV_MAX_TAPS) return -1;
  if (a->M <= 0) return 0;
  const int nwg = ((a->M + 127) / 128) * ((a->Ncol + 127) / 128);
  const I8Epi ep{xscale, xs_const, wscale, out_mode, out_inv, add8, add_scale, add_ld};
  const bool fk = a->Cs % QBK == 0;
  const bool g3fk = a->Cs % 64 == 0;
  const long p8_tiles = (long)((a->M + 255) / 256) * ((a->Ncol + 255) / 256);
  if (bigdl_stem_i8_applies(a, &ep) && bigdl_stem_i8(a, &ep, st) == 0) {
    // the 7x7/2 image stem over its width im2col: staged-row kernel (conv_halo.hip stem_i8_kernel)
  } else if (bigdl_conv_halo_i8_applies(a, &ep) && bigdl_conv_halo_i8(a, &ep, st) == 0) {
    // 3x3 / stride-1 / pad-1: the halo-tile kernel on the i8 matrix cores (conv_halo.hip)
  } else if (i8_s1_applies(*a, ep)) {
    launch_i8_s1(*a, ep, st);
  } else if (i8_p8() && fk && a->Kdim >= 1024 && a->Ncol >= 256 && a->Ncol % 16 == 0 &&
      (g_i8_p8 == 2 || p8_tiles >= 160)) {
    if (i8_direct_ok(*a, ep)) conv_i8_p8_kernel<true><<<dim3((unsigned)p8_tiles), dim3(512), 0, st>>>(*a, ep);
    else conv_i8_p8_kernel<false><<<dim3((unsigned)p8_tiles), dim3(512), 0, st>>>(*a, ep);
  } else if (a->Ncol <= 64 && i8_g3()) {
    const int bn = a->Ncol <= 32 ? 32 : 64;
    const int g = ((a->M + 255) / 256) * ((a->Ncol + bn - 1) / bn);
    if (bn == 32) launch_i8_g3<256, 32, 4, 1>(g, g3fk, *a, ep, st);
    else launch_i8_g3<256, 64, 4, 1>(g, g3fk, *a, ep, st);
  } else if (a->Ncol <= 32) {
    const int g = ((a->M + 255) / 256) * ((a->Ncol + 31) / 32);
    if (fk) conv_i8_glds_kernel<256, 32, 4, true><<<g, 256, 0, st>>>(*a, ep);
    else conv_i8_glds_kernel<256, 32, 4, false><<<g, 256, 0, st>>>(*a, ep);
  } else if (a->Ncol <= 64) {
    const int g = ((a->M + 255) / 256) * ((a->Ncol + 63) / 64);
    if (fk) conv_i8_glds_kernel<256, 64, 4, true><<<g, 256, 0, st>>>(*a, ep);
    else conv_i8_glds_kernel<256, 64, 4, false><<<g, 256, 0, st>>>(*a, ep);
  } else if (i8_g3() && (g_i8_g3 == 3 || (g_i8_g3 == 2 && ((a->M + 255) / 256) * ((a->Ncol + 127) / 128) >= 512))) {
    const int g = ((a->M + 255) / 256) * ((a->Ncol + 127) / 128);
    launch_i8_g3<256, 128, 2, 2>(g, g3fk, *a, ep, st);
  } else if (i8_g3()) {
    launch_i8_g3<128, 128, 2, 2>(nwg, g3fk, *a, ep, st);
  } else if (fk) {
    conv_i8_glds_kernel<128, 128, 2, true><<<nwg, 256, 0, st>>>(*a, ep);
  } else {
    conv_i8_glds_kernel<128, 128, 2, false><<<nwg, 256, 0, st>>>(*a, ep);
  }
  HIP_LAUNCH_CHECK();
  return 0;
}

void bigdl_copy_rows_i8(const int8_t* src, int8_t* dst, long rows, int C, long lds, long ldd, hipStream_t st) {
  const long total = rows * C;
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  copy_rows_i8_kernel<<<blocks > 0 ? blocks : 1, 256, 0, st>>>(src, dst, rows, C, lds, ldd);
  HIP_LAUNCH_CHECK();
}

void bigdl_pool_i8(const int8_t* x, int8_t* y, int N, int H, int W, int Cp, int OH, int OW, int kh, int kw, int sh,
                   int sw, int ph, int pw, int avg, int count_pad, long ldo, hipStream_t st) {
  const long total = (long)N * OH * OW * (Cp >> 4);
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  if (kh == 3 && kw == 3)
    pool_i8_kernel<true><<<blocks > 0 ? blocks : 1, 256, 0, st>>>(x, y, N, H, W, Cp, OH, OW, kh, kw, sh, sw, ph, pw,
                                                                  avg, count_pad, ldo);
  else
    pool_i8_kernel<false><<<blocks > 0 ? blocks : 1, 256, 0, st>>>(x, y, N, H, W, Cp, OH, OW, kh, kw, sh, sw, ph, pw,
                                                                   avg, count_pad, ldo);
  HIP_LAUNCH_CHECK();
}

void bigdl_quantize_nchw_f32(const float* x, int8_t* q, int N, int C, int HW, int Cp, float inv, hipStream_t st) {
  const long total = (long)N * HW;
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  quantize_nchw_f32_kernel<<<blocks > 0 ? blocks : 1, 256, 0, st>>>(x, q, N, C, HW, Cp, inv);
  HIP_LAUNCH_CHECK();
}

void bigdl_quantize_wim2col_f32(const float* x, int8_t* y, int N, int C, int H, int W, int OW, int S, int sw, int pw,
                                float inv, hipStream_t st) {
  const long total = (long)N * H * OW;
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  quantize_wim2col_f32_kernel<<<blocks > 0 ? blocks : 1, 256, 0, st>>>(x, y, N, C, H, W, OW, S, sw, pw, inv);
  HIP_LAUNCH_CHECK();
}

void bigdl_quantize_rows_bf16(const uint16_t* x, int8_t* q, long P, int C, long ldq, float inv, hipStream_t st) {
  const long total = P * (C >> 3);
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  quantize_rows_bf16_kernel<<<blocks > 0 ? blocks : 1, 256, 0, st>>>(x, q, P, C, ldq, inv);
  HIP_LAUNCH_CHECK();
}

void bigdl_dequantize_rows(const int8_t* q, uint16_t* y, long P, int C, long ld, float scale, hipStream_t st) {
  const long total = P * C;
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  dequantize_rows_kernel<<<blocks > 0 ? blocks : 1, 256, 0, st>>>(q, y, P, C, ld, scale);
  HIP_LAUNCH_CHECK();
}

}  // extern "C"
