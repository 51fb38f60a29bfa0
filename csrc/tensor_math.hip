// Native TensorMath backend for fp32 GPU tensors of the 1-based Tensor API (bigdl_amd/tensor/tensor.py).
//
// Reference: S/tensor/DenseTensorApply.scala:19 (apply1 / apply2 / apply3: an element function walked over up to
// three strided tensors), S/tensor/DenseTensorMath.scala + TensorMath.scala:38-829 (the ~150 element-wise ops,
// reductions along a dimension, and the BLAS entry points addmm / addmv / addr / baddbmm / dot routed to MKL).
//
// MI355X design:
//  * one strided apply kernel for unary / binary / ternary element ops: the host collapses the operands' shared
//    contiguous dimensions (at most 6 remain), each lane walks elements with a grid stride and turns its linear index
//    into per-operand offsets; zero strides give broadcasting (addr's outer product is ternary apply with the two
//    vectors strided along different dimensions); fully contiguous operands take a 4-wide vector path;
//  * reductions over [outer, R, inner] (sum / prod / max / min with 1-based arg index / sum of squares / p-norm
//    partials) in two passes when R is long: chunk partials from a grid over (rows, chunks), then the chunk
//    reduction, so one long row still spreads over the chip;
//  * fp32 GEMM on the f32-input MFMA (v_mfma_f32_16x16x4_f32: exact fp32, one fmaf chain per output — the MKL
//    sgemm numerics): 64 x 64 tiles through LDS from arbitrary strides (transposed operands are just strides),
//    batched over blockIdx.z, C = beta * M + alpha * A.B; gemv as one wave per output row.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int TD = 6;

struct ApplyDesc {
  long size[TD];
  long so[TD], sa[TD], sb[TD], sc[TD];
  int nd;
  long n;
};

enum Op : int {
  OP_COPY = 0, OP_FILL, OP_ADDS, OP_MULS, OP_NEG, OP_ABS, OP_EXP, OP_LOG, OP_LOG1P, OP_SQRT, OP_SQUARE, OP_TANH,
  OP_FLOOR, OP_CEIL, OP_SIGN, OP_RECIP, OP_POWS, OP_CLAMP, OP_SIGMOID, OP_DIVS,
  // binary: out = f(a, b)
  OP_ADD = 32, OP_SUB, OP_MUL, OP_DIV, OP_MAX, OP_MIN, OP_POW,
  // ternary: out = f(a, b, c)
  OP_ADDCMUL = 64, OP_ADDCDIV, OP_AXPBYZ
};

__device__ __forceinline__ float apply_op(int op, float a, float b, float c, float s0, float s1) {
  switch (op) {
    case OP_COPY: return a;
    case OP_FILL: return s0;
    case OP_ADDS: return a + s0;
    case OP_MULS: return a * s0;
    case OP_NEG: return -a;
    case OP_ABS: return fabsf(a);
    case OP_EXP: return expf(a);
    case OP_LOG: return logf(a);
    case OP_LOG1P: return log1pf(a);
    case OP_SQRT: return sqrtf(a);
    case OP_SQUARE: return a * a;
    case OP_TANH: return tanhf(a);
    case OP_FLOOR: return floorf(a);
    case OP_CEIL: return ceilf(a);
    case OP_SIGN: return a > 0.f ? 1.f : (a < 0.f ? -1.f : 0.f);
    case OP_RECIP: return 1.f / a;
    case OP_POWS: return powf(a, s0);
    case OP_CLAMP: return fminf(fmaxf(a, s0), s1);
    case OP_SIGMOID: return 1.f / (1.f + expf(-a));
    case OP_DIVS: return a / s0;
    case OP_ADD: return a + s0 * b;            // add(value, y): a + value * b
    case OP_SUB: return a - s0 * b;
    case OP_MUL: return a * b;
    case OP_DIV: return a / b;
    case OP_MAX: return fmaxf(a, b);
    case OP_MIN: return fminf(a, b);
    case OP_POW: return powf(a, b);
    case OP_ADDCMUL: return a + s0 * b * c;
    case OP_ADDCDIV: return a + s0 * b / c;
    case OP_AXPBYZ: return s1 * a + s0 * b * c; // addr: beta * M + alpha * x (outer) y
    default: return a;
  }
}

__global__ __launch_bounds__(256) void apply_kernel(float* __restrict__ out, const float* __restrict__ a,
                                                    const float* __restrict__ b, const float* __restrict__ c,
                                                    ApplyDesc d, int op, float s0, float s1) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < d.n; i += (long)gridDim.x * blockDim.x) {
    long rem = i, oo = 0, oa = 0, ob = 0, oc = 0;
    for (int k = d.nd - 1; k >= 0; --k) {
      const long sz = d.size[k];
      const long idx = rem % sz;
      rem /= sz;
      oo += idx * d.so[k];
      oa += idx * d.sa[k];
      ob += idx * d.sb[k];
      oc += idx * d.sc[k];
    }
    const float va = a ? a[oa] : 0.f, vb = b ? b[ob] : 0.f, vc = c ? c[oc] : 0.f;
    out[oo] = apply_op(op, va, vb, vc, s0, s1);
  }
}

// every operand contiguous (or absent) with the same element order: 16-byte vectors
__global__ __launch_bounds__(256) void apply_contig_kernel(float* __restrict__ out, const float* __restrict__ a,
                                                           const float* __restrict__ b, const float* __restrict__ c,
                                                           long n, int op, float s0, float s1) {
  const long n4 = n >> 2;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const v4f va = a ? reinterpret_cast<const v4f*>(a)[i] : v4f{0.f, 0.f, 0.f, 0.f};
    const v4f vb = b ? reinterpret_cast<const v4f*>(b)[i] : v4f{0.f, 0.f, 0.f, 0.f};
    const v4f vc = c ? reinterpret_cast<const v4f*>(c)[i] : v4f{0.f, 0.f, 0.f, 0.f};
    v4f r;
#pragma unroll
    for (int e = 0; e < 4; ++e) r[e] = apply_op(op, va[e], vb[e], vc[e], s0, s1);
    reinterpret_cast<v4f*>(out)[i] = r;
  }
  for (long i = (n4 << 2) + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = apply_op(op, a ? a[i] : 0.f, b ? b[i] : 0.f, c ? c[i] : 0.f, s0, s1);
}

// ------------------------------------------------------------------------------------------------ reductions
enum RedOp : int { R_SUM = 0, R_PROD, R_MAX, R_MIN, R_SUMSQ, R_ABSPOW };

struct Acc {
  float v;
  long i;
};

__device__ __forceinline__ Acc red_init(int op) {
  switch (op) {
    case R_PROD: return {1.f, 0};
    case R_MAX: return {-INFINITY, -1};
    case R_MIN: return {INFINITY, -1};
    default: return {0.f, 0};
  }
}

__device__ __forceinline__ float red_elem(int op, float x, float p) {
  if (op == R_SUMSQ) return x * x;
  if (op == R_ABSPOW) return powf(fabsf(x), p);
  return x;
}

// combine; for max / min the lower index wins ties, and NaN propagates (as torch.max)
__device__ __forceinline__ Acc red_comb(int op, Acc a, Acc b) {
  switch (op) {
    case R_PROD: return {a.v * b.v, 0};
    case R_MAX:
      if (b.i < 0) return a;
      if (a.i < 0) return b;
      if (isnan(a.v)) return a;
      if (isnan(b.v)) return b;
      return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
    case R_MIN:
      if (b.i < 0) return a;
      if (a.i < 0) return b;
      if (isnan(a.v)) return a;
      if (isnan(b.v)) return b;
      return (b.v < a.v || (b.v == a.v && b.i < a.i)) ? b : a;
    default: return {a.v + b.v, 0};
  }
}

// x viewed as [outer][R][inner] (contiguous); grid = (ceil(outer * inner / 4) blocks of 4 rows, chunks); each block of
// 256 threads reduces a chunk of R for 4 (outer, inner) rows: 64 lanes per row, wave shuffles. Writes partials
// [chunk][row] (value, index) or, with one chunk, the final value (and 1-based index).
__global__ __launch_bounds__(256) void reduce_kernel(const float* __restrict__ x, long outer, long R, long inner,
                                                     long chunk, int op, float p, float* __restrict__ pv,
                                                     long* __restrict__ pi, int final_out, float* __restrict__ out,
                                                     float* __restrict__ outi, int mean) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long rows = outer * inner;
  const long row = blockIdx.x * 4L + w;
  if (row >= rows) return;
  const long o = row / inner, in = row - o * inner;
  const long r0 = blockIdx.y * chunk, r1 = min(R, r0 + chunk);
  Acc acc = red_init(op);
  for (long r = r0 + lane; r < r1; r += 64) acc = red_comb(op, acc, Acc{red_elem(op, x[(o * R + r) * inner + in], p), r});
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    Acc other;
    other.v = __shfl_xor(acc.v, s, 64);
    other.i = __shfl_xor(acc.i, s, 64);
    acc = red_comb(op, acc, other);
  }
  if (lane != 0) return;
  if (pv != nullptr && !final_out) {
    pv[blockIdx.y * rows + row] = acc.v;
    pi[blockIdx.y * rows + row] = acc.i;
  } else {
    float v = acc.v;
    if (mean) v /= (float)R;
    out[row] = v;
    if (outi) outi[row] = (float)(acc.i + 1);
  }
}

// second pass: partials [chunks][rows] -> out[row] (+ 1-based index)
__global__ __launch_bounds__(256) void reduce_partials_kernel(const float* __restrict__ pv, const long* __restrict__ pi,
                                                              long rows, long chunks, long R, int op, float* __restrict__ out,
                                                              float* __restrict__ outi, int mean) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long row = blockIdx.x * 4L + w;
  if (row >= rows) return;
  Acc acc = red_init(op);
  for (long c = lane; c < chunks; c += 64) acc = red_comb(op, acc, Acc{pv[c * rows + row], pi[c * rows + row]});
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    Acc other;
    other.v = __shfl_xor(acc.v, s, 64);
    other.i = __shfl_xor(acc.i, s, 64);
    acc = red_comb(op, acc, other);
  }
  if (lane == 0) {
    float v = acc.v;
    if (mean) v /= (float)R;
    out[row] = v;
    if (outi) outi[row] = (float)(acc.i + 1);
  }
}

// ------------------------------------------------------------------------------------------------ fp32 GEMM
// C[b][m][n] = beta * M[b][m][n] + alpha * sum_k A[b][m][k] * B[b][k][n]; every operand by (row, col) strides.
// 64 x 64 tile, 4 waves as 2 x 2 (32 x 32 each = 2 x 2 tiles of v_mfma_f32_16x16x4_f32), K in chunks of 16 through
// LDS (A chunk [64][16 + 1], B chunk [16][64 + 1]: padded rows, conflict-free column reads).
struct GemmDesc {
  int M, N, K;
  long sam, sak, sbk, sbn, scm, scn, smm, smn;
  long bsa, bsb, bsc, bsm;
  float alpha, beta;
};

__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                       const float* __restrict__ Min, float* __restrict__ C, GemmDesc g) {
  __shared__ float As[64][17];
  __shared__ float Bs[16][65];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int bt = blockIdx.z;
  const int m0 = blockIdx.y * 64, n0 = blockIdx.x * 64;
  const float* Ab = A + bt * g.bsa;
  const float* Bb = B + bt * g.bsb;
  v4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < g.K; k0 += 16) {
    // A chunk: 64 x 16 = 1024 values, 4 per thread; B chunk: 16 x 64
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = tid + e * 256;
      const int r = idx >> 4, kk = idx & 15;
      const int m = m0 + r, k = k0 + kk;
      As[r][kk] = (m < g.M && k < g.K) ? Ab[m * g.sam + k * g.sak] : 0.f;
      const int kb = idx >> 6, cn = idx & 63;
      const int n = n0 + cn, k2 = k0 + kb;
      Bs[kb][cn] = (n < g.N && k2 < g.K) ? Bb[k2 * g.sbk + n * g.sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int k = ks * 4 + (lane >> 4);
      float fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) fa[i] = As[wm * 32 + i * 16 + (lane & 15)][k];
#pragma unroll
      for (int j = 0; j < 2; ++j) fb[j] = Bs[k][wn * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  float* Cb = C + bt * g.bsc;
  const float* Mb = Min ? Min + bt * g.bsm : nullptr;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 32 + j * 16 + (lane & 15);
      if (n >= g.N) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int m = m0 + wm * 32 + i * 16 + 4 * (lane >> 4) + e;
        if (m >= g.M) continue;
        float v = g.alpha * acc[i][j][e];
        if (Mb && g.beta != 0.f) v += g.beta * Mb[m * g.smm + n * g.smn];
        Cb[m * g.scm + n * g.scn] = v;
      }
    }
}

// y[m] = beta * Min[m] + alpha * sum_k A[m][k] x[k]: one wave per row, 4 rows per block
__global__ __launch_bounds__(256) void gemv_f32_kernel(const float* __restrict__ A, const float* __restrict__ x,
                                                       const float* __restrict__ Min, float* __restrict__ y, int M, int K,
                                                       long sam, long sak, long sx, long smi, long sy, float alpha,
                                                       float beta) {
  const int lane = threadIdx.x & 63;
  const long m = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (m >= M) return;
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s = fmaf(A[m * sam + k * sak], x[k * sx], s);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) {
    float v = alpha * s;
    if (Min && beta != 0.f) v += beta * Min[m * smi];
    y[m * sy] = v;
  }
}

int grid_for(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 8192 ? 8192 : (b < 1 ? 1 : b));
}

}  // namespace

extern "C" {

int bigdl_tensor_apply(float* out, const float* a, const float* b, const float* c, int nd, const long* size,
                       const long* so, const long* sa, const long* sb, const long* sc, int op, float s0, float s1,
                       int contiguous, hipStream_t st) {
  if (nd < 0 || nd > TD) return -1;
  long n = 1;
  for (int k = 0; k < nd; ++k) n *= size[k];
  if (n == 0) return 0;
  const bool aligned = ((reinterpret_cast<uintptr_t>(out) | reinterpret_cast<uintptr_t>(a) |
                         reinterpret_cast<uintptr_t>(b) | reinterpret_cast<uintptr_t>(c)) & 15) == 0;
  if (contiguous && aligned) {
    apply_contig_kernel<<<grid_for((n + 3) / 4), 256, 0, st>>>(out, a, b, c, n, op, s0, s1);
  } else {
    ApplyDesc d{};
    d.nd = nd;
    d.n = n;
    for (int k = 0; k < nd; ++k) {
      d.size[k] = size[k];
      d.so[k] = so[k];
      d.sa[k] = sa ? sa[k] : 0;
      d.sb[k] = sb ? sb[k] : 0;
      d.sc[k] = sc ? sc[k] : 0;
    }
    apply_kernel<<<grid_for(n), 256, 0, st>>>(out, a, b, c, d, op, s0, s1);
  }
  HIP_LAUNCH_CHECK();
  return 0;
}

// x contiguous [outer][R][inner]; out [outer * inner] (+ outi 1-based indices for max / min); ws: workspace of
// chunks * outer * inner * (4 + 8) bytes when chunks > 1
int bigdl_tensor_reduce(const float* x, long outer, long R, long inner, int op, float p, float* out, float* outi,
                        int mean, float* ws, long chunks, hipStream_t st) {
  const long rows = outer * inner;
  if (rows <= 0) return 0;
  const long rb = (rows + 3) / 4;
  if (rb > 2147483647L || chunks > 65535) return -1;
  if (chunks <= 1 || ws == nullptr) {
    reduce_kernel<<<dim3((unsigned)rb, 1), 256, 0, st>>>(x, outer, R, inner, R, op, p, nullptr, nullptr, 1, out, outi,
                                                         mean);
  } else {
    const long chunk = (R + chunks - 1) / chunks;
    float* pv = ws;
    long* pi = reinterpret_cast<long*>(ws + chunks * rows + ((chunks * rows) & 1));
    reduce_kernel<<<dim3((unsigned)rb, (unsigned)chunks), 256, 0, st>>>(x, outer, R, inner, chunk, op, p, pv, pi, 0,
                                                                        out, outi, mean);
    reduce_partials_kernel<<<(unsigned)rb, 256, 0, st>>>(pv, pi, rows, chunks, R, op, out, outi, mean);
  }
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_gemm_f32(const float* A, const float* B, const float* Min, float* C, int batch, int M, int N, int K,
                   const long* s, float alpha, float beta, hipStream_t st) {
  if (batch <= 0 || M <= 0 || N <= 0) return 0;
  if (batch > 65535 || (M + 63) / 64 > 65535) return -2;
  GemmDesc g{M, N, K, s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7], s[8], s[9], s[10], s[11], alpha, beta};
  if (K <= 0) {   // C = beta * M
    g.K = 0;
  }
  dim3 grid((N + 63) / 64, (M + 63) / 64, batch);
  gemm_f32_kernel<<<grid, 256, 0, st>>>(A, B, Min, C, g);
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_gemv_f32(const float* A, const float* x, const float* Min, float* y, int M, int K, long sam, long sak,
                   long sx, long smi, long sy, float alpha, float beta, hipStream_t st) {
  if (M <= 0) return 0;
  gemv_f32_kernel<<<(M + 3) / 4, 256, 0, st>>>(A, x, Min, y, M, K, sam, sak, sx, smi, sy, alpha, beta);
  HIP_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
