// Native index / sort / mask ops for fp32 GPU tensors of the 1-based Tensor API (bigdl_amd/tensor/tensor.py).
//
// Reference: S/tensor/TensorMath.scala gather (:199), scatter (:209), topk (:622), maskedFill / maskedCopy /
// maskedSelect (:700-719), index (:739), indexAdd (:751) — DenseTensor's per-element Scala loops over 1-based
// T-typed index tensors.
//
// MI355X design: every op sees the tensor as [outer, R, inner] around its dimension (the host makes operands
// contiguous). Index tensors stay T-typed (fp32, 1-based, the reference's representation) or int64; the kernels
// convert per element, so no index-cast pass runs on the device.
//  * index / gather: one lane per output element, a grid-stride loop, coalesced along inner;
//  * indexAdd: fp32 atomics (duplicate indices accumulate, as in the reference);
//  * scatter: one lane per source element (duplicates: last writer, unordered as in torch);
//  * topk: one workgroup per row, (key, index) pairs bitonic-sorted in LDS (rows up to 8192), k written sorted;
//  * masked select / copy: stream compaction in three launches — per-block mask counts, one-workgroup exclusive
//    scan of the block counts (wave prefix sums), then each block re-counts with a workgroup prefix sum and writes
//    in element order. The selected count is read back once by the host (it sizes the result, as in the reference).
#include "common.h"
#include "kernels.h"

namespace {

template <typename I>
__device__ __forceinline__ long idx0(const I* p, long i) { return (long)p[i] - 1; }

template <typename I>
__global__ __launch_bounds__(256) void index_select_kernel(const float* __restrict__ src, const I* __restrict__ idx,
                                                           float* __restrict__ out, long outer, long Rs, long n,
                                                           long inner, int* err) {
  const long total = outer * n * inner;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long i = e % inner, t = e / inner, j = t % n, o = t / n;
    const long r = idx0(idx, j);
    if (r < 0 || r >= Rs) { err[0] = 1; out[e] = 0.f; continue; }
    out[e] = src[(o * Rs + r) * inner + i];
  }
}

template <typename I>
__global__ __launch_bounds__(256) void index_add_kernel(float* __restrict__ dst, const I* __restrict__ idx,
                                                        const float* __restrict__ src, long outer, long Rd, long n,
                                                        long inner, int* err) {
  const long total = outer * n * inner;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long i = e % inner, t = e / inner, j = t % n, o = t / n;
    const long r = idx0(idx, j);
    if (r < 0 || r >= Rd) { err[0] = 1; continue; }
    atomicAdd(dst + (o * Rd + r) * inner + i, src[e]);
  }
}

// gather: out[o, j, i] = src[o, idx[o, j, i] - 1, i]    (idx and out are [outer, n, inner], src [outer, Rs, inner])
template <typename I>
__global__ __launch_bounds__(256) void gather_kernel(const float* __restrict__ src, const I* __restrict__ idx,
                                                     float* __restrict__ out, long outer, long Rs, long n, long inner,
                                                     int* err) {
  const long total = outer * n * inner;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long i = e % inner, o = e / (inner * n);
    const long r = idx0(idx, e);
    if (r < 0 || r >= Rs) { err[0] = 1; out[e] = 0.f; continue; }
    out[e] = src[(o * Rs + r) * inner + i];
  }
}

// scatter: dst[o, idx[o, j, i] - 1, i] = src[o, j, i]    (idx [outer, n, inner]; src indexed with its own row size)
template <typename I>
__global__ __launch_bounds__(256) void scatter_kernel(float* __restrict__ dst, const I* __restrict__ idx,
                                                      const float* __restrict__ src, long outer, long Rd, long n,
                                                      long inner, long Rsrc, int* err) {
  const long total = outer * n * inner;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const long i = e % inner, t = e / inner, j = t % n, o = t / n;
    const long r = idx0(idx, e);
    if (r < 0 || r >= Rd) { err[0] = 1; continue; }
    dst[(o * Rd + r) * inner + i] = src[(o * Rsrc + j) * inner + i];
  }
}

__global__ __launch_bounds__(256) void masked_fill_kernel(float* __restrict__ x, const float* __restrict__ mask,
                                                          float v, long n) {
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256)
    if (mask[e] != 0.f) x[e] = v;
}

// ---------------------------------------------------------------------------------------------- stream compaction
constexpr int CB = 1024;   // elements per compaction block (4 per lane)

__device__ __forceinline__ int block_exclusive_scan(int v, int* sh, int* total) {
  // 256 lanes: wave inclusive scan with shuffles, then the 4 wave totals through LDS
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int s = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(s, o, 64);
    if (lane >= o) s += t;
  }
  if (lane == 63) sh[w] = s;
  __syncthreads();
  int base = 0;
  for (int k = 0; k < w; ++k) base += sh[k];
  if (total) *total = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  return base + s - v;
}

__global__ __launch_bounds__(256) void mask_count_kernel(const float* __restrict__ mask, long n, int* __restrict__ cnt) {
  __shared__ int sh[4];
  const long b0 = (long)blockIdx.x * CB;
  int c = 0;
#pragma unroll
  for (int k = 0; k < CB / 256; ++k) {
    const long e = b0 + k * 256 + threadIdx.x;
    c += (e < n && mask[e] != 0.f) ? 1 : 0;
  }
  int tot;
  block_exclusive_scan(c, sh, &tot);
  if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}

// exclusive scan of nb block counts in place (one workgroup, 256-wide chunks); the total goes to cnt[nb]
__global__ __launch_bounds__(256) void scan_counts_kernel(int* __restrict__ cnt, int nb) {
  __shared__ int sh[4];
  int carry = 0;
  for (int c0 = 0; c0 < nb; c0 += 256) {
    const int i = c0 + threadIdx.x;
    const int v = i < nb ? cnt[i] : 0;
    int tot;
    const int ex = block_exclusive_scan(v, sh, &tot);
    if (i < nb) cnt[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) cnt[nb] = carry;
}

// select: out[rank] = x[e] for mask[e] != 0; copy (COPY = true): x[e] = src[rank] for mask[e] != 0
template <bool COPY>
__global__ __launch_bounds__(256) void mask_write_kernel(float* __restrict__ x, const float* __restrict__ mask,
                                                         const float* __restrict__ src, float* __restrict__ out,
                                                         long n, const int* __restrict__ base, long nsrc) {
  __shared__ int sh[4];
  const long b0 = (long)blockIdx.x * CB;
  int run = base[blockIdx.x];
#pragma unroll
  for (int k = 0; k < CB / 256; ++k) {
    const long e = b0 + k * 256 + threadIdx.x;
    const int m = (e < n && mask[e] != 0.f) ? 1 : 0;
    int tot;
    const int ex = block_exclusive_scan(m, sh, &tot);
    if (m) {
      const long r = run + ex;
      if (COPY) {
        if (r < nsrc) x[e] = src[r];
      } else {
        out[r] = x[e];
      }
    }
    run += tot;
  }
}

// ---------------------------------------------------------------------------------------------- topk
// One workgroup per row of R <= P elements (P = pow2 >= R, <= 8192): (key, index) pairs bitonic-sorted in LDS on a
// total-order 32-bit key, the first k written (values, 1-based fp32 indices). Key: the float's bits made monotone
// (negative: all bits flipped, else the sign bit set), every NaN canonicalised to +NaN, which then orders above +inf:
// last for smallest-k, first for largest-k (key complemented), as torch.topk orders NaN in both directions. Padding
// takes the maximal key, so it sorts behind every element, NaN included.
__device__ __forceinline__ unsigned topk_key(float v, int largest) {
  unsigned u = __float_as_uint(v != v ? __builtin_nanf("") : v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return largest ? ~u : u;
}

template <int P>
__global__ __launch_bounds__(256) void topk_kernel(const float* __restrict__ x, long R, long inner, int k, int largest,
                                                   float* __restrict__ vals, float* __restrict__ inds) {
  __shared__ unsigned key[P];
  __shared__ int id[P];
  const long row = blockIdx.x;
  const long o = row / inner, in = row % inner;
  const float* src = x + o * R * inner + in;
  for (int t = threadIdx.x; t < P; t += 256) {
    key[t] = t < R ? topk_key(src[(long)t * inner], largest) : 0xffffffffu;
    id[t] = t;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < P / 2; t += 256) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const unsigned a = key[lo], b = key[hi];
        const int ia = id[lo], ib = id[hi];
        const bool gt = a > b || (a == b && ia > ib);   // stable on ties: lower index first
        if (gt == up) {
          key[lo] = b; key[hi] = a;
          id[lo] = ib; id[hi] = ia;
        }
      }
      __syncthreads();
    }
  }
  for (int t = threadIdx.x; t < k; t += 256) {
    const long dst = (o * k + t) * inner + in;
    const int i = id[t];
    vals[dst] = src[(long)i * inner];
    inds[dst] = (float)(i + 1);
  }
}

int grid_for(long n) {
  long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" {

int bigdl_index_op(int op, float* a, const void* idx, int idx_i64, const float* b, float* out, long outer, long R,
                   long n, long inner, long Rsrc, int* err, hipStream_t st) {
  const long total = outer * n * inner;
  if (total <= 0) return 0;
  const int g = grid_for(total);
#define BIGDL_IDX_DISPATCH(I)                                                                                    \
  switch (op) {                                                                                                  \
    case 0: index_select_kernel<I><<<g, 256, 0, st>>>(b, (const I*)idx, out, outer, R, n, inner, err); break;   \
    case 1: index_add_kernel<I><<<g, 256, 0, st>>>(a, (const I*)idx, b, outer, R, n, inner, err); break;       \
    case 2: gather_kernel<I><<<g, 256, 0, st>>>(b, (const I*)idx, out, outer, R, n, inner, err); break;        \
    case 3: scatter_kernel<I><<<g, 256, 0, st>>>(a, (const I*)idx, b, outer, R, n, inner, Rsrc, err); break;   \
    default: return -1;                                                                                          \
  }
  if (idx_i64) {
    BIGDL_IDX_DISPATCH(long)
  } else {
    BIGDL_IDX_DISPATCH(float)
  }
#undef BIGDL_IDX_DISPATCH
  HIP_LAUNCH_CHECK();
  return 0;
}

void bigdl_masked_fill(float* x, const float* mask, float v, long n, hipStream_t st) {
  if (n <= 0) return;
  masked_fill_kernel<<<grid_for(n), 256, 0, st>>>(x, mask, v, n);
  HIP_LAUNCH_CHECK();
}

long bigdl_mask_blocks(long n) { return (n + CB - 1) / CB; }

// counts: int[nb + 1] workspace; after the call counts[nb] (device) holds the selected total
void bigdl_mask_scan(const float* mask, long n, int* counts, hipStream_t st) {
  const long nb = bigdl_mask_blocks(n);
  if (nb <= 0) return;
  mask_count_kernel<<<(unsigned)nb, 256, 0, st>>>(mask, n, counts);
  scan_counts_kernel<<<1, 256, 0, st>>>(counts, (int)nb);
  HIP_LAUNCH_CHECK();
}

void bigdl_mask_write(int copy, float* x, const float* mask, const float* src, float* out, long n, const int* counts,
                      long nsrc, hipStream_t st) {
  const long nb = bigdl_mask_blocks(n);
  if (nb <= 0) return;
  if (copy) mask_write_kernel<true><<<(unsigned)nb, 256, 0, st>>>(x, mask, src, out, n, counts, nsrc);
  else mask_write_kernel<false><<<(unsigned)nb, 256, 0, st>>>(x, mask, src, out, n, counts, nsrc);
  HIP_LAUNCH_CHECK();
}

int bigdl_topk(const float* x, long outer, long R, long inner, int k, int largest, float* vals, float* inds,
               hipStream_t st) {
  if (R > 8192 || k > R || k <= 0) return -1;
  const long rows = outer * inner;
  if (rows <= 0) return 0;
  if (R <= 256) topk_kernel<256><<<(unsigned)rows, 256, 0, st>>>(x, R, inner, k, largest, vals, inds);
  else if (R <= 1024) topk_kernel<1024><<<(unsigned)rows, 256, 0, st>>>(x, R, inner, k, largest, vals, inds);
  else if (R <= 4096) topk_kernel<4096><<<(unsigned)rows, 256, 0, st>>>(x, R, inner, k, largest, vals, inds);
  else topk_kernel<8192><<<(unsigned)rows, 256, 0, st>>>(x, R, inner, k, largest, vals, inds);
  HIP_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
