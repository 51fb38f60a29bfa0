// bigdl_amd native kernel library — shared device helpers for gfx950 (CDNA4).
//
// All kernels in csrc/*.hip are written for MI355X only: 64-lane wavefronts,
// MFMA bf16 matrix cores, 160 KiB LDS per CU. Nothing here is a CUDA shim.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;  // raw bf16 bits (activations / weights in HBM)

typedef short v8s __attribute__((ext_vector_type(8)));   // 8 x bf16 MFMA operand (4 VGPR)
typedef short v4s __attribute__((ext_vector_type(4)));   // 4 x bf16 (tr16 read result)
typedef float v4f __attribute__((ext_vector_type(4)));   // 16x16 MFMA accumulator / 4 x f32
typedef int v4i __attribute__((ext_vector_type(4)));     // 16x16 i8 MFMA accumulator / operand (16 x int8)
typedef float v16f __attribute__((ext_vector_type(16))); // 32x32 MFMA accumulator
typedef unsigned int v4u __attribute__((ext_vector_type(4)));  // 16-byte global access
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

#define WAVE 64
#define LDS_PTR(T) __attribute__((address_space(3))) T*

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  // Round-to-nearest-even; hipcc lowers the __bf16 cast to v_cvt_pk_bf16_f32 (keeps NaN a NaN).
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}
// pack two floats into one dword of 2 x bf16 (lo in bits 0..15)
__device__ __forceinline__ unsigned pack2bf(float lo, float hi) {
  return (unsigned)f2bf(lo) | ((unsigned)f2bf(hi) << 16);
}
__device__ __forceinline__ float lo_bf(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 "XCD swizzle
// must be bijective"): consecutive logical tiles land on the same XCD so neighbouring tiles that
// share operand panels hit that XCD's private L2. Speed only — correctness never depends on it.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg < 16) return bid;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// One byte of a post-ReLU sign mask (bit e = channel e of an 8-channel group is > 0) as the 16-byte bf16 granule the
// z-mask consumers compare against zero: 1.0 where the bit is set, 0 elsewhere (batchnorm.hip bn_apply writes it).
__device__ __forceinline__ v4u mask8_to_bf(unsigned b) {
  v4u r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = (((b >> (2 * e)) & 1u) ? 0x3f80u : 0u) | (((b >> (2 * e + 1)) & 1u) ? 0x3f800000u : 0u);
  return r;
}
// AND-mask of a 16-byte granule of 8 bf16 keeping element e where bit e of b is set (a masked residual addend)
__device__ __forceinline__ v4u mask8_to_and(unsigned b) {
  v4u r;
#pragma unroll
  for (int e = 0; e < 4; ++e) r[e] = (((b >> (2 * e)) & 1u) ? 0xffffu : 0u) | (((b >> (2 * e + 1)) & 1u) ? 0xffff0000u : 0u);
  return r;
}
// sign-mask byte of 8 bf16 values (bit e: value e > 0)
__device__ __forceinline__ unsigned bf_to_mask8(const v4u& o) {
  unsigned b = 0;
#pragma unroll
  for (int e = 0; e < 4; ++e) b |= ((lo_bf(o[e]) > 0.f) ? 1u : 0u) << (2 * e) | ((hi_bf(o[e]) > 0.f) ? 1u : 0u) << (2 * e + 1);
  return b;
}

#define HIP_LAUNCH_CHECK() (void)hipGetLastError()
