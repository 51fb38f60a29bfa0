// Microbenchmark: streaming-bound 1x1 convolution GEMM out[M][N] = A[M][K] * W[N][K]^T (bf16 in/out, fp32 acc) with
// the fused BN-statistics epilogue, on the ResNet-50 layer shapes where the per-tile kernel runs at 2-3 TB/s
// (layer 3: M = 802816, K = 64, N = 256). Standalone (hipcc, no torch) so a structure can be iterated on quickly:
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/nt_stream tools/ubench/nt_stream.hip && /tmp/nt_stream [M K N]
//
// Kernels:
//   ceiling  : same bytes, no math (read A once, write out once) - what the memory system gives this access pattern
//   stream   : persistent workgroups; W for the wave's 64 channels held in VGPRs as MFMA A fragments for the whole
//              launch; A fragments loaded straight from HBM into VGPRs (16 B per lane), prefetched two tiles ahead;
//              epilogue through a wave-private LDS slice (bf16, XOR-swizzled 16-byte granules) into 16-byte stores
//              of whole 128-byte lines; per-channel sum / sum of squares kept in registers across all of the
//              workgroup's tiles and added once at the end (no per-tile reduction or atomics).
//   ref      : plain per-element fp32 reference (validation only).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <math.h>
#include <string.h>

typedef uint16_t bf16_t;
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((unsigned)v) << 16); }
__device__ __forceinline__ unsigned pack2bf(float lo, float hi) {
  __bf16 a = (__bf16)lo, b = (__bf16)hi;
  return (unsigned)__builtin_bit_cast(bf16_t, a) | ((unsigned)__builtin_bit_cast(bf16_t, b) << 16);
}
__device__ __forceinline__ float lo_bf(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(unsigned u) { return __uint_as_float(u & 0xffff0000u); }

// ------------------------------------------------------------------------------------------------ reference
__global__ void ref_kernel(const bf16_t* A, const bf16_t* W, float* out, int M, int K, int N) {
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  if (i >= (long)M * N) return;
  int m = i / N, n = i % N;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(A[(long)m * K + k]) * bf2f(W[(long)n * K + k]);
  out[i] = s;
}

// ------------------------------------------------------------------------------------------------ ceiling
__global__ __launch_bounds__(256) void ceiling_kernel(const v4u* A, v4u* out, long na, long no) {
  long i = blockIdx.x * 256L + threadIdx.x, st = (long)gridDim.x * 256;
  v4u acc = {0, 0, 0, 0};
  for (long j = i; j < na; j += st) acc ^= A[j];
  for (long j = i; j < no; j += st) out[j] = acc + v4u{(unsigned)j, 0, 0, 0};
}

// ------------------------------------------------------------------------------------------------ stream
// 256 threads = 4 waves; wave w: channel group cg = w % CG (64 channels), pixel group pg = w / CG. The workgroup's
// channel block chb = blockIdx.x % NCHB covers CG * 64 channels; its tiles are BMW * (4 / CG) pixels.
typedef float v2f __attribute__((ext_vector_type(2)));
constexpr int SLOTS = 128;
// STATS: 0 none, 1 scalar sums of the rounded bf16 output, 2 the same with packed (2 x f32) VALU
template <int K, int CG, int BMW, int STATS>
__global__ __launch_bounds__(256, 2) void stream_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ W,
                                                        bf16_t* __restrict__ out, float* __restrict__ stats, int M,
                                                        int N) {
  constexpr int KF = K / 32;          // MFMA K-steps
  constexpr int MI = BMW / 16;        // 16-pixel blocks per wave tile
  constexpr int PGN = 4 / CG;
  constexpr int BM = BMW * PGN;       // pixels per workgroup tile
  __shared__ __attribute__((aligned(16))) bf16_t lds[4 * BMW * 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cg = wave % CG, pg = wave / CG;
  const int nchb = N / (64 * CG);
  const int chb = blockIdx.x % nchb, wgi = blockIdx.x / nchb, ngr = gridDim.x / nchb;
  const int c0 = (chb * CG + cg) * 64;
  const int ntiles = M / BM;          // (M % BM == 0 in this benchmark)
  bf16_t* wl = lds + wave * BMW * 64;

  v8s wf[4][KF];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int kk = 0; kk < KF; ++kk)
      wf[j][kk] = *reinterpret_cast<const v8s*>(W + (size_t)(c0 + 16 * j + (lane & 15)) * K + 32 * kk + 8 * (lane >> 4));

  auto load = [&](v8s (&af)[MI][KF], int t) {
    const int p0 = t * BM + pg * BMW;
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int kk = 0; kk < KF; ++kk)
        af[i][kk] = *reinterpret_cast<const v8s*>(A + (size_t)(p0 + 16 * i + (lane & 15)) * K + 32 * kk + 8 * (lane >> 4));
  };
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  v2f p1[4], p2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) p1[e] = p2[e] = v2f{0.f, 0.f};

  auto compute_store = [&](v8s (&af)[MI][KF], int t) {
    v4f acc[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < KF; ++kk)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][kk], af[i][kk], acc[i][j], 0, 0, 0);
    // D[n][m]: lane holds channels 16 j + 4 (lane >> 4) + e of pixel 16 i + (lane & 15). To LDS as [pixel][64 ch]
    // bf16 rows of 128 B = 8 granules of 16 B; granule g of pixel p at slot g ^ (p & 7).
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = 16 * i + (lane & 15);
        const int q = lane >> 4;                      // 4-channel quarter within the 16-channel block j
        const int g = 2 * j + (q >> 1);
        const int off = p * 64 + ((g ^ (p & 7)) << 3) + (q & 1) * 4;
        *reinterpret_cast<v2u*>(wl + off) = v2u{pack2bf(acc[i][j][0], acc[i][j][1]), pack2bf(acc[i][j][2], acc[i][j][3])};
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): wave-private slice
    const int p0 = t * BM + pg * BMW;
#pragma unroll
    for (int rr = 0; rr < BMW / 8; ++rr) {
      const int p = rr * 8 + (lane >> 3), g = lane & 7;
      const v4u v = *reinterpret_cast<const v4u*>(wl + p * 64 + ((g ^ (p & 7)) << 3));
      if constexpr (STATS == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float y0 = lo_bf(v[e]), y1 = hi_bf(v[e]);
          s1[2 * e] += y0; s2[2 * e] = fmaf(y0, y0, s2[2 * e]);
          s1[2 * e + 1] += y1; s2[2 * e + 1] = fmaf(y1, y1, s2[2 * e + 1]);
        }
      } else if constexpr (STATS == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const v2f y = {lo_bf(v[e]), hi_bf(v[e])};
          p1[e] += y;
          p2[e] = __builtin_elementwise_fma(y, y, p2[e]);
        }
      }
      *reinterpret_cast<v4u*>(out + (size_t)(p0 + p) * N + c0 + 8 * g) = v;
    }
  };

  v8s a0[MI][KF], a1[MI][KF], a2[MI][KF];
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
  if constexpr (STATS == 2) {
#pragma unroll
    for (int e = 0; e < 4; ++e) { s1[2 * e] = p1[e][0]; s1[2 * e + 1] = p1[e][1]; s2[2 * e] = p2[e][0]; s2[2 * e + 1] = p2[e][1]; }
  }
  if constexpr (STATS != 0) {
    // lanes l, l + 8, ... share channels c0 + 8 (l & 7) + e: reduce over lane >> 3, one atomic per channel per wave
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    if (lane < 8) {
      float* sp = stats + (size_t)(blockIdx.x & (SLOTS - 1)) * 2 * N;   // slotted: same-address atomics serialise
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        atomicAdd(sp + c0 + 8 * lane + e, s1[e]);
        atomicAdd(sp + N + c0 + 8 * lane + e, s2[e]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------ host
static float bfr(float f) {   // round to bf16 (RNE) and back
  unsigned u; memcpy(&u, &f, 4);
  u = (u + 0x7fff + ((u >> 16) & 1)) & 0xffff0000u;
  float r; memcpy(&r, &u, 4); return r;
}
static bf16_t tobf(float f) { unsigned u; memcpy(&u, &f, 4); return (bf16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16); }

template <typename F>
static float timeit(F f, int iters = 20) {
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a));
    for (int i = 0; i < iters; ++i) f();
    CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms * 1e3f / iters);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 802816, K = argc > 2 ? atoi(argv[2]) : 64, N = argc > 3 ? atoi(argv[3]) : 256;
  int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  printf("M %d K %d N %d (CUs %d)\n", M, K, N, cus);
  std::vector<bf16_t> hA((size_t)M * K), hW((size_t)N * K);
  srand(1);
  for (auto& v : hA) v = tobf((rand() / (float)RAND_MAX) * 2.f - 1.f);
  for (auto& v : hW) v = tobf(((rand() / (float)RAND_MAX) * 2.f - 1.f) * 0.1f);
  bf16_t *A, *W, *out; float *stats, *ref;
  CK(hipMalloc(&A, hA.size() * 2)); CK(hipMalloc(&W, hW.size() * 2));
  CK(hipMalloc(&out, (size_t)M * N * 2)); CK(hipMalloc(&stats, (size_t)SLOTS * 2 * N * 4));
  CK(hipMemcpy(A, hA.data(), hA.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(W, hW.data(), hW.size() * 2, hipMemcpyHostToDevice));
  const double bytes = (double)M * K * 2 + (double)M * N * 2;
  // validation on the first 4096 rows
  const int MV = 4096;
  CK(hipMalloc(&ref, (size_t)MV * N * 4));
  ref_kernel<<<(MV * N + 255) / 256, 256>>>(A, W, ref, MV, K, N);
  std::vector<float> href((size_t)MV * N);
  CK(hipMemcpy(href.data(), ref, href.size() * 4, hipMemcpyDeviceToHost));

  float tc = timeit([&] { ceiling_kernel<<<cus * 8, 256>>>((const v4u*)A, (v4u*)out, (long)M * K / 8, (long)M * N / 8); });
  printf("ceiling  %8.1f us  %5.2f TB/s\n", tc, bytes / tc / 1e6);

  auto check = [&](const char* name, float us) {
    std::vector<bf16_t> ho((size_t)MV * N);
    CK(hipMemcpy(ho.data(), out, ho.size() * 2, hipMemcpyDeviceToHost));
    double maxd = 0;
    for (size_t i = 0; i < ho.size(); ++i) {
      unsigned u = ((unsigned)ho[i]) << 16; float f; memcpy(&f, &u, 4);
      maxd = std::max(maxd, (double)fabsf(f - bfr(href[i])));
    }
    std::vector<float> hs((size_t)SLOTS * 2 * N);
    CK(hipMemcpy(hs.data(), stats, hs.size() * 4, hipMemcpyDeviceToHost));
    for (int sl = 1; sl < SLOTS; ++sl) hs[0] += hs[(size_t)sl * 2 * N];
    printf("%-28s %8.1f us  %5.2f TB/s  %6.1f TF/s  max|d| %.3g  mean[0] %.4f\n", name, us, bytes / us / 1e6,
           2.0 * M * N * K / us / 1e6, maxd, hs[0] / M);
  };
#define RUN(KK, CG, BMW, ST, WPC)                                                                         \
  if (K == KK && N % (64 * CG) == 0 && (M % (BMW * (4 / CG))) == 0) {                                    \
    const int nchb = N / (64 * CG);                                                                       \
    const int grid = (cus * WPC / nchb) * nchb;                                                           \
    auto f = [&] { stream_kernel<KK, CG, BMW, ST><<<grid, 256>>>(A, W, out, stats, M, N); };             \
    CK(hipMemset(stats, 0, (size_t)SLOTS * 2 * N * 4)); f(); CK(hipDeviceSynchronize());                                 \
    char nm[96]; snprintf(nm, sizeof nm, "stream<K%d,CG%d,BMW%d,%s> x%d", KK, CG, BMW, ST == 2 ? "pk" : ST ? "st" : "--", WPC); \
    float us = timeit(f);                                                                                 \
    CK(hipMemset(stats, 0, (size_t)SLOTS * 2 * N * 4)); f(); CK(hipDeviceSynchronize());                                 \
    check(nm, us);                                                                                        \
  }
  RUN(64, 4, 32, 0, 2) RUN(64, 4, 32, 1, 2) RUN(64, 4, 32, 2, 2) RUN(64, 4, 64, 1, 2) RUN(64, 4, 64, 2, 2)
  RUN(64, 4, 32, 2, 3) RUN(64, 1, 32, 0, 2) RUN(64, 1, 32, 2, 2) RUN(64, 1, 64, 2, 2) RUN(64, 2, 32, 2, 2)
  RUN(128, 4, 32, 0, 2) RUN(128, 4, 32, 2, 2) RUN(128, 4, 16, 2, 2) RUN(128, 4, 16, 2, 3) RUN(128, 2, 32, 2, 2)
  RUN(128, 1, 32, 2, 2)
  return 0;
}
