// Batched NT GEMM on the bf16 MFMA for gfx950: C[b][m][n] = sum_k A[b][m][k] * B[b][n][k] (fp32 out).
//
// The GPU engine's small matrix-product layers: MM / MV (reference S/nn/MM.scala:34 and S/nn/MV.scala:33, batched
// over a leading dimension), LocallyConnected1D/2D (S/nn/LocallyConnected2D.scala:233: one weight matrix per output
// location = a GEMM batched over locations) and the tree-LSTM gate products. Every transpose they need is an NT
// product of K-contiguous operands, so one kernel (and its three uses in the autograd wrapper, ops/bmm.py) covers
// forward and backward.
//
// Workgroup = 64 x 64 output tile, 4 waves as 2 x 2, each wave 32 x 32 = 2 x 2 tiles of v_mfma_f32_16x16x32_bf16.
// The operands are small and re-read by few tiles, so fragments are loaded straight from global memory (16-byte
// granules: row (lane & 15), 8 k-values (lane >> 4)) two k-steps ahead of their MFMAs — no LDS round trip. K is a
// multiple of 32 (the host zero-pads it); rows past M / N load a zero granule and are not stored.
#include "common.h"
#include "kernels.h"

namespace {

__device__ __forceinline__ v8s ldg8(const bf16_t* p, bool ok) {
  v8s z = {0, 0, 0, 0, 0, 0, 0, 0};
  return ok ? *reinterpret_cast<const v8s*>(p) : z;
}

__global__ __launch_bounds__(256) void bmm_nt_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                     float* __restrict__ C, int M, int N, int K, long sa, long sb,
                                                     long sc, int lda, int ldb, int ldc, float alpha, int accum) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int bt = blockIdx.z;
  const int m0 = blockIdx.y * 64 + wm * 32, n0 = blockIdx.x * 64 + wn * 32;
  const bf16_t* Ab = A + bt * sa;
  const bf16_t* Bb = B + bt * sb;
  const int r = lane & 15, kg = (lane >> 4) * 8;
  const bool am0 = m0 + r < M, am1 = m0 + 16 + r < M, bn0 = n0 + r < N, bn1 = n0 + 16 + r < N;
  const bf16_t* pa0 = Ab + (long)(am0 ? m0 + r : 0) * lda + kg;
  const bf16_t* pa1 = Ab + (long)(am1 ? m0 + 16 + r : 0) * lda + kg;
  const bf16_t* pb0 = Bb + (long)(bn0 ? n0 + r : 0) * ldb + kg;
  const bf16_t* pb1 = Bb + (long)(bn1 ? n0 + 16 + r : 0) * ldb + kg;
  v4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < K; k += 64) {
    // two k-steps of fragments in flight before their MFMAs
    v8s a[2][2], b[2][2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bool kin = k + 32 * s < K;
      a[s][0] = ldg8(pa0 + k + 32 * s, am0 && kin);
      a[s][1] = ldg8(pa1 + k + 32 * s, am1 && kin);
      b[s][0] = ldg8(pb0 + k + 32 * s, bn0 && kin);
      b[s][1] = ldg8(pb1 + k + 32 * s, bn1 && kin);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s][i], b[s][j], acc[i][j], 0, 0, 0);
  }
  // D[m][n]: lane holds column n = lane & 15 of rows 4 * (lane >> 4) + e
  float* Cb = C + bt * sc;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 16 * j + (lane & 15);
      if (n >= N) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + 16 * i + 4 * (lane >> 4) + e;
        if (m < M) {
          float* o = Cb + (long)m * ldc + n;
          *o = accum ? *o + alpha * acc[i][j][e] : alpha * acc[i][j][e];
        }
      }
    }
}

}  // namespace

extern "C" int bigdl_bmm_nt(const uint16_t* A, const uint16_t* B, float* C, int batch, int M, int N, int K, long sa,
                            long sb, long sc, int lda, int ldb, int ldc, float alpha, int accum, hipStream_t st) {
  if (K % 32 != 0 || lda % 8 != 0 || ldb % 8 != 0 || batch <= 0 || M <= 0 || N <= 0) return -1;
  if (batch > 65535 || (M + 63) / 64 > 65535) return -2;
  dim3 grid((N + 63) / 64, (M + 63) / 64, batch);
  bmm_nt_kernel<<<grid, 256, 0, st>>>(A, B, C, M, N, K, sa, sb, sc, lda, ldb, ldc, alpha, accum);
  HIP_LAUNCH_CHECK();
  return 0;
}
