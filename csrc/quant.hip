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

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));

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
__device__ __forceinline__ v4u qload16(const uint8_t* p, bool ok) {
  return *reinterpret_cast<const v4u*>(ok ? p : g_zero16);
}

template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void conv_i8_kernel(ConvArgs a, const float* __restrict__ xscale,
                                                         const float* __restrict__ wscale, int out_f32) {
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int AROWS = BM / 32, BROWS = BN / 32;
  constexpr int STAGE = (BM + BN) * QBK;        // bytes per stage
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * STAGE];
  const uint8_t* src = reinterpret_cast<const uint8_t*>(a.src);
  const uint8_t* wt = reinterpret_cast<const uint8_t*>(a.wt);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (a.Ncol + BN - 1) / BN;
  const int nwg = ((a.M + BM - 1) / BM) * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int lrow = tid >> 3, lg = tid & 7;
  const int ohw = a.OH * a.OW;
  int a_pix[AROWS], a_h[AROWS], a_w[AROWS];
#pragma unroll
  for (int i = 0; i < AROWS; ++i) {
    const int m = m0 + lrow + 32 * i;
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
  v4u ra[AROWS], rb[BROWS];
  auto gload = [&](int kt) {
    const int kk = kt * QBK + lg * 16;
    const bool kvalid = kk < a.Kdim;
    const int kc = kvalid ? kk : 0;
    const int t = kc / a.Cs, c = kc - t * a.Cs;
    const int th = a.tap_h[t], tw = a.tap_w[t];
    const int wk = a.tap_k[t] * a.Cs + c;
#pragma unroll
    for (int i = 0; i < AROWS; ++i) {
      const int ch = a_h[i] + th, cw = a_w[i] + tw;
      const bool ok = kvalid && (unsigned)ch < (unsigned)a.Hs && (unsigned)cw < (unsigned)a.Ws;
      ra[i] = qload16(src + (size_t)(a_pix[i] + ch * a.Ws + cw) * a.Cs + c, ok);
    }
#pragma unroll
    for (int i = 0; i < BROWS; ++i) {
      const int n = n0 + lrow + 32 * i;
      rb[i] = qload16(wt + (size_t)(n < a.Ncol ? n : 0) * a.ldw + wk, kvalid && n < a.Ncol);
    }
  };
  auto swz = [](int row, int g) { return row * QBK + ((g ^ (row & 7)) << 4); };
  auto swrite = [&](int buf) {
    uint8_t* A = lds + buf * STAGE;
    uint8_t* B = A + BM * QBK;
#pragma unroll
    for (int i = 0; i < AROWS; ++i) *reinterpret_cast<v4u*>(A + swz(lrow + 32 * i, lg)) = ra[i];
#pragma unroll
    for (int i = 0; i < BROWS; ++i) *reinterpret_cast<v4u*>(B + swz(lrow + 32 * i, lg)) = rb[i];
  };
  v4i acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  const int nk = (a.Kdim + QBK - 1) / QBK;
  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);
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
    if (kt + 1 < nk) swrite(cur ^ 1);
    __syncthreads();
  }
  // epilogue: lane owns channels 4*(lane>>4)+e of pixel lane&15 (weights were the MFMA A operand)
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int nb = n0 + wn * TN + j * 16 + (lane >> 4) * 4;
    float ws[4], bs[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool ok = nb + e < a.Ncol;
      ws[e] = ok ? wscale[nb + e] : 0.f;
      bs[e] = (ok && a.bias) ? a.bias[nb + e] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = m0 + wm * TM + i * 16 + (lane & 15);
      if (m >= a.M) continue;
      const int img = m / ohw;
      const float xs = xscale[img];
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = (float)acc[i][j][e] * xs * ws[e] + bs[e];
        if (a.relu) t = fmaxf(t, 0.f);
        v[e] = t;
      }
      if (out_f32) {
        float* o = reinterpret_cast<float*>(a.out) + (size_t)m * a.ldo + nb;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (nb + e < a.Ncol) o[e] = v[e];
      } else {
        bf16_t* o = a.out + (size_t)m * a.ldo + nb;
        if ((a.ldo & 3) == 0 && nb + 3 < a.Ncol) {
          *reinterpret_cast<v2u*>(o) = v2u{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (nb + e < a.Ncol) o[e] = f2bf(v[e]);
        }
      }
    }
  }
}

}  // namespace

extern "C" {

int bigdl_quantize_act(const void* x, int is_bf16, int8_t* q, float* amax, float* scale, int N, long P, int C,
                       int Cp, int static_amax, hipStream_t st) {
  const long per = P * C;
  if (!static_amax) {            // dynamic per-sample range; with static_amax the caller filled amax (calibrated)
    (void)hipMemsetAsync(amax, 0, sizeof(float) * N, st);
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

int bigdl_conv_i8(const ConvArgs* a, const float* xscale, const float* wscale, int out_f32, hipStream_t st) {
  if (a->Cs % 16 != 0 || a->Kdim != a->ntaps * a->Cs || a->ntaps < 1 || a->ntaps > CONV_MAX_TAPS) return -1;
  if (a->M <= 0) return 0;
  const int nwg = ((a->M + 127) / 128) * ((a->Ncol + 127) / 128);
  conv_i8_kernel<128, 128><<<nwg, 256, 0, st>>>(*a, xscale, wscale, out_f32);
  HIP_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
