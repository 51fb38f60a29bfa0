// Forward of the 7x7 / stride-2 image stem over the pixel-pair view (stem.hip), as a halo-tile MFMA kernel (gfx950).
//
// Over the pair view [N][Hp][Wq][8] (two width taps x 4 channels per 16-byte granule) the stem is a stride-(2, 1)
// convolution with R = 7 row taps x 4 pair taps of 8 channels: output (oh, ow) reduces over granules (2 oh + r,
// ow + j). For a fixed row tap r the 4 pair taps of one output column are 4 CONSECUTIVE granules = one 32-element
// MFMA K-step read straight out of the input row, so the conv is 7 K-steps of v_mfma_f32_16x16x32_bf16 per output
// fragment. The implicit-GEMM tile (conv_nt_g4 over 28 per-lane-gathered taps, 384 us, 5x its HBM bound at batch 256)
// is replaced by: a workgroup stages the 2 * RB + 5 input rows its RB output rows need (one contiguous 24 KB block of
// the pair tensor: a 1.6x halo, read once) plus the 64 x 224 weight (rows padded to 30 granules: conflict-free
// fragment reads), then each wave computes one output row (112 columns = 7 fragments x 64 channels) from LDS; the
// epilogue is halo_epi_lean (bias, ReLU, BN statistics with one workgroup-level atomic commit; conv_epilogue.h).
// Reference: the ImageNet ResNet stem, S/models/resnet/ResNet.scala:249-260 (SpatialConvolution(3, 64, 7, 7, 2, 2,
// 3, 3) + BN + ReLU + pooling).
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "common.h"
#include "kernels.h"
#include "conv_epilogue.h"

namespace {

constexpr int SR = 7, SRB = 4, SOW = 112, SFM = SOW / 16, SXROWS = 2 * SRB + SR - 2;   // 13 input rows per tile
constexpr int SWST = 30 * 16;                                                             // weight row stride (B)

template <int WQ>
struct StemL {
  static constexpr int XB = SXROWS * WQ * 16;                 // input tile bytes
  static constexpr int XG = (XB / 16 + 255) / 256;            // DMA granules per thread
  static constexpr int WOFF = (XG * 256 * 16 + 1023) / 1024 * 1024;
  static constexpr int LDS0 = WOFF + 64 * SWST;
  static constexpr int EPI = 4 * SFM * 16 * 128 + 4 * 128 * 4;   // bf16 slices + per-wave sums
  static constexpr int LDS = LDS0 > EPI ? LDS0 : EPI;
};

struct StemRowMap {
  long base;
  __device__ __forceinline__ long operator()(const ConvArgs&, int v) const { return base + v; }
};

template <int WQ>
__global__ __launch_bounds__(256, 2) void stem_fwd_kernel(ConvArgs a) {
  using L = StemL<WQ>;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[L::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_img = a.OH / SRB;
  const int bid = xcd_remap(blockIdx.x, a.Nb * tiles_img);
  const int n = bid / tiles_img, oh0 = (bid - n * tiles_img) * SRB;

  // input rows 2 oh0 .. 2 oh0 + 12 of image n: one contiguous block (granules past the tensor read as zeros)
  const bf16_t* src = reinterpret_cast<const bf16_t*>(a.src);
  const size_t xoff = ((size_t)n * a.Hs + 2 * oh0) * WQ * 8;            // elements
  const size_t xend = (size_t)a.Nb * a.Hs * WQ * 8;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(src + xoff), (short)0,
                                                                      (int)((xend - xoff) * 2), 0x00020000);
#pragma unroll
  for (int d = 0; d < L::XG; ++d)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (LDS_PTR(void))(lds + (d * 4 + wave) * 1024), 16,
                                             ((d * 4 + wave) * 64 + lane) * 16, 0, 0, 0);
  // weights [64][224] -> rows of 30 granules (28 used)
  const bf16_t* wt = reinterpret_cast<const bf16_t*>(a.wt);
  for (int q = tid; q < 64 * 28; q += 256) {
    const int k = q / 28, g = q - k * 28;
    *reinterpret_cast<v4u*>(lds + L::WOFF + k * SWST + g * 16) =
        *reinterpret_cast<const v4u*>(wt + (size_t)k * a.ldw + g * 8);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // wave = output row oh0 + wave; fragment i = columns 16 i .. 16 i + 15; lane: column 16 i + (lane & 15), granule
  // lane >> 4 of the K-step (pair tap j)
  v4f acc[SFM][4];
#pragma unroll
  for (int i = 0; i < SFM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const unsigned char* W = lds + L::WOFF + (lane & 15) * SWST + (lane >> 4) * 16;
#pragma unroll
  for (int r = 0; r < SR; ++r) {
    v8s fw[4], fx[SFM];
#pragma unroll
    for (int j = 0; j < 4; ++j) fw[j] = *reinterpret_cast<const v8s*>(W + j * 16 * SWST + r * 64);
    const unsigned char* X = lds + ((2 * wave + r) * WQ + (lane & 15) + (lane >> 4)) * 16;
#pragma unroll
    for (int i = 0; i < SFM; ++i) fx[i] = *reinterpret_cast<const v8s*>(X + i * 16 * 16);
#pragma unroll
    for (int i = 0; i < SFM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[j], fx[i], acc[i][j], 0, 0, 0);
  }
  __syncthreads();     // every wave's fragment reads retired: the LDS becomes the epilogue's slices
  const StemRowMap rm{((long)n * a.OH + oh0) * SOW};
  halo_epi_lean<SFM, 4, 1, 64>(a, acc, wave * SOW, 0, lane, bid, lds + wave * SFM * 16 * 128, rm,
                               reinterpret_cast<float*>(lds + 4 * SFM * 16 * 128), 0);
}

}  // namespace

extern "C" {

// The pair-view stem conv (conv_igemm ConvArgs of ops/conv.py conv2d_pairs_fwd) when it has the ImageNet shape this
// kernel is built for: 7 row x 4 pair taps in (r, j) order, row stride 2, 64 output channels, 112 output columns,
// output rows a multiple of 4, no addend / consumer-BN epilogue. BIGDL_STEM_FWD=0 turns it off.
static int g_stem_fwd = -1;
void bigdl_set_stem_fwd(int v) { g_stem_fwd = v; }

int bigdl_stem_fwd_applies(const ConvArgs* a) {
  if (g_stem_fwd < 0) {
    const char* e = getenv("BIGDL_STEM_FWD");
    g_stem_fwd = e ? atoi(e) : 1;
  }
  if (!g_stem_fwd || a->Cs != 8 || a->ntaps != SR * 4 || a->mul_h != 2 || a->mul_w != 1 || a->OW != SOW || a->Ws != 115 ||
      a->OH % SRB || a->Ncol != 64 || a->ldw != SR * 32 || a->Kdim != SR * 32 || !a->ident_out || a->ldo != 64 ||
      a->out32 || a->addend || a->bnred || a->pstride || a->ws)
    return 0;
  if (a->Hs < 2 * a->OH + SR - 2) return 0;
  for (int t = 0; t < SR * 4; ++t)
    if (a->tap_h[t] != t / 4 || a->tap_w[t] != t % 4 || a->tap_k[t] != t) return 0;
  if ((size_t)a->Nb * a->Hs * a->Ws * 16 >= (1ull << 31) || (size_t)a->Nb * a->OH * a->OW * 128 >= (1ull << 31)) return 0;
  return 1;
}

int bigdl_stem_fwd(const ConvArgs* a, hipStream_t st) {
  stem_fwd_kernel<115><<<dim3(a->Nb * (a->OH / SRB)), dim3(256), 0, st>>>(*a);
  return 0;
}

}  // extern "C"

// ------------------------------------------------------------------------------------------------
// Weight gradient of the same pair-view stem: dW'[k][r * 32 + kk] = sum over output pixels p of dy[p][k] * X_r[p][kk],
// X_r[(oh, ow)][kk] = element kk % 8 of pair granule (2 oh + r, ow + kk / 8). The split-K im2col kernel gathered 28
// granules per pixel (394 us at batch 256, the last exposed weight gradient of the step). Here a persistent workgroup
// of 7 waves (wave = row tap r, one workgroup per CU) strides over tiles of 2 output rows: it stages the 9 input rows
// and the 224 x 64 dy rows of the next tile (two contiguous blocks, LDS-DMA, double-buffered), and every wave reduces the tile's 224 pixels in 32-pixel MFMA
// K-steps. Both operands are read down the pixel rows with ds_read_b64_tr_b16 (T10): dy rows are the A operand
// (channels k), and the overlapping windows of the input row are the B operand: the window row of pixel p starts
// 16 bytes after p - 1's, so consecutive "rows" overlap and no im2col copy exists anywhere. A wave keeps its 64 x 32
// partial dW'_r in 8 accumulators across all its tiles; the workgroup writes one fp32 partial [64][224] and a fixed-
// order reduce adds the partials into dW' (deterministic).
namespace {

constexpr int SWRB = 2, SWPX = SWRB * SOW, SWXROWS = 2 * SWRB + SR - 2;   // 224 pixels, 9 input rows per tile

template <int WQ>
struct StemW {
  static constexpr int XB = SWXROWS * WQ * 16;
  static constexpr int XI = (XB + 7 * 1024 - 1) / (7 * 1024);      // DMA rounds of 7 waves x 1 KiB
  static constexpr int XR = XI * 7 * 1024;
  static constexpr int DB = SWPX * 128;                            // dy tile: 224 pixels x 64 channels
  static constexpr int DI = DB / (7 * 1024);
  static constexpr int LDS1 = XR + DB;                            // one tile buffer
  static constexpr int LDS = 2 * LDS1;
  static_assert(DB % (7 * 1024) == 0, "dy tile must split into DMA rounds");
  static_assert(LDS <= 160 * 1024, "two tile buffers per workgroup");
};

__device__ __forceinline__ int dyswz(int row) { return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2); }

template <int OFF>
__device__ __forceinline__ v8s trd2s(unsigned a0, unsigned a1) {
  v4s lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(a0), "n"(OFF));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "n"(OFF));
  return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

template <int WQ>
__global__ __launch_bounds__(448, 1) void stem_wgrad_kernel(WgradArgs a) {
  using L = StemW<WQ>;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[L::LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int r = __builtin_amdgcn_readfirstlane(tid >> 6);          // row tap of this wave (7 waves)
  const int tiles_img = a.OH / SWRB, ntiles = a.Nb * tiles_img;
  const bf16_t* xs = reinterpret_cast<const bf16_t*>(a.src);
  const bf16_t* dys = reinterpret_cast<const bf16_t*>(a.dy);
  const size_t xend = (size_t)a.Nb * a.Hs * WQ * 8, dend = (size_t)a.M * 64;
  const unsigned lb = (unsigned)(uintptr_t)(LDS_PTR(unsigned char))lds;
  // dy DMA: LDS chunk (row, slot) holds source chunk (row, slot ^ dyswz(row)) (conflict-free transposed reads)
  unsigned dsrc[L::DI];
#pragma unroll
  for (int d = 0; d < L::DI; ++d) {
    const int Q = (d * 7 + r) * 64 + lane, row = Q >> 3, sl = Q & 7;
    dsrc[d] = (unsigned)((row * 8 + (sl ^ dyswz(row))) * 16);
  }
  // transposed-read lane geometry: g = lane >> 4 (8 pixels of the 32-pixel K-step), q = row of a 4-row block,
  // p = 4-column group
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  v4f acc[4][2], accb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = accb[i] = v4f{0.f, 0.f, 0.f, 0.f};
  // bias gradient: wave 0 also multiplies its dy fragments by a ones operand (column sums of dy, every column alike)
  const bool bias = a.dbias != nullptr && r == 0;
  const v8s ones = {(short)0x3f80, (short)0x3f80, (short)0x3f80, (short)0x3f80,
                    (short)0x3f80, (short)0x3f80, (short)0x3f80, (short)0x3f80};

  // double-buffered tiles: tile i + 1's DMA is issued right after the barrier that makes tile i visible (and retires
  // every wave's reads of tile i - 1, the buffer it overwrites)
  auto issue = [&](int t, int buf) {
    const int n = t / tiles_img, oh0 = (t - n * tiles_img) * SWRB;
    const size_t xo = ((size_t)n * a.Hs + 2 * oh0) * WQ * 8, dofs = ((size_t)n * a.OH + oh0) * SOW * 64;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(xs + xo), (short)0,
                                                                        (int)((xend - xo) * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(dys + dofs), (short)0,
                                                                        (int)((dend - dofs) * 2), 0x00020000);
    unsigned char* B = lds + buf * L::LDS1;
#pragma unroll
    for (int d = 0; d < L::XI; ++d)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (LDS_PTR(void))(B + (d * 7 + r) * 1024), 16,
                                               ((d * 7 + r) * 64 + lane) * 16, 0, 0, 0);
#pragma unroll
    for (int d = 0; d < L::DI; ++d)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (LDS_PTR(void))(B + L::XR + (d * 7 + r) * 1024), 16,
                                               (int)dsrc[d], 0, 0, 0);
  };
  int buf = 0;
  if ((int)blockIdx.x < ntiles) issue(blockIdx.x, 0);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x, buf ^= 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t + (int)gridDim.x < ntiles) issue(t + gridDim.x, buf ^ 1);
    const unsigned bb = lb + (unsigned)(buf * L::LDS1);
#pragma unroll
    for (int c = 0; c < SWPX / 32; ++c) {
      // A (dy): rows c * 32 + 8 g + q (+ 4), channels kf * 16 + 4 p .. + 3 -> chunk 2 kf + (p >> 1) ^ dyswz(row)
      const int ra = c * 32 + 8 * g + q;
      unsigned da[2][4];
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int kf = 0; kf < 4; ++kf)
          da[h][kf] = bb + L::XR + (unsigned)((ra + 4 * h) * 128 + (((2 * kf + (p >> 1)) ^ dyswz(ra + 4 * h)) << 4) +
                                              (p & 1) * 8);
      // B (windows): pixel c * 32 + 8 g + q (+ 4) -> input row 2 ohl + r, granule ow + 2 nf + (p >> 1)
      unsigned xa[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int px = ra + 4 * h;
        const int ohl = px >= SOW ? 1 : 0, ow = px - ohl * SOW;
        xa[h] = bb + (unsigned)((((2 * ohl + r) * WQ + ow + (p >> 1)) * 16) + (p & 1) * 8);
      }
      v8s fa[4], fb[2];
#pragma unroll
      for (int kf = 0; kf < 4; ++kf) fa[kf] = trd2s<0>(da[0][kf], da[1][kf]);
      fb[0] = trd2s<0>(xa[0], xa[1]);
      fb[1] = trd2s<32>(xa[0], xa[1]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kf = 0; kf < 4; ++kf)
#pragma unroll
        for (int nf = 0; nf < 2; ++nf)
          acc[kf][nf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kf], fb[nf], acc[kf][nf], 0, 0, 0);
      if (bias) {
#pragma unroll
        for (int kf = 0; kf < 4; ++kf) accb[kf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kf], ones, accb[kf], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // partial dW'[k][r * 32 + kk] of this workgroup: lane holds k = kf * 16 + 4 (lane >> 4) + e, kk = nf * 16 + (lane & 15)
  float* o = a.ws + (size_t)blockIdx.x * 64 * 224;
#pragma unroll
  for (int kf = 0; kf < 4; ++kf)
#pragma unroll
    for (int nf = 0; nf < 2; ++nf)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[(size_t)(kf * 16 + 4 * (lane >> 4) + e) * 224 + r * 32 + nf * 16 + (lane & 15)] = acc[kf][nf][e];
  if (bias && (lane & 15) == 0) {        // bias partials after the weight partials: [grid][64]
    float* ob = a.ws + (size_t)gridDim.x * 64 * 224 + (size_t)blockIdx.x * 64;
#pragma unroll
    for (int kf = 0; kf < 4; ++kf)
#pragma unroll
      for (int e = 0; e < 4; ++e) ob[kf * 16 + 4 * (lane >> 4) + e] = accb[kf][e];
  }
}

}  // namespace

extern "C" {

static int g_stem_wgrad = -1;
void bigdl_set_stem_wgrad(int v) { g_stem_wgrad = v; }

static int stem_wgrad_grid() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}

// Workspace floats (> 0) when the pair-view stem kernel takes this weight gradient (ops/conv.py conv2d_pairs_wgrad
// geometry: 8-element pairs, 7 row x 4 pair taps, row stride 2, 112 output columns, 64 channels), else 0.
long bigdl_stem_wgrad_plan(const WgradArgs* a) {
  if (g_stem_wgrad < 0) {
    const char* e = getenv("BIGDL_STEM_WGRAD");
    g_stem_wgrad = e ? atoi(e) : 1;
  }
  if (!g_stem_wgrad || a->Cs != 8 || a->R != SR || a->S != 4 || a->sh != 2 || a->sw != 1 || a->ph || a->pw ||
      a->dh != 1 || a->dwl != 1 || a->OW != SOW || a->Ws != 115 || (a->OH % SWRB) || a->Ncol != 64 ||
      a->Kdim != SR * 32 || a->ldy != 64 || a->M != a->Nb * a->OH * a->OW || a->Hs < 2 * a->OH + SR - 2)
    return 0;
  if ((size_t)a->Nb * a->Hs * a->Ws * 16 >= (1ull << 31) || (size_t)a->M * 128 >= (1ull << 31)) return 0;
  const long tiles = (long)a->Nb * (a->OH / SWRB);
  return (long)std::min<long>(tiles, stem_wgrad_grid()) * (64 * 224 + 64);
}

// dW' (fp32 [64][224], a->dw) += the stem weight gradient, a->dbias += the column sums of dy (wave 0's extra MFMAs
// against a ones operand); a->ws = the plan's workspace.
int bigdl_stem_wgrad(const WgradArgs* a, hipStream_t st) {
  const long tiles = (long)a->Nb * (a->OH / SWRB);
  const int grid = (int)std::min<long>(tiles, stem_wgrad_grid());
  stem_wgrad_kernel<115><<<dim3(grid), dim3(448), 0, st>>>(*a);
  bigdl_split_reduce_f32(a->ws, a->dw, 64 * 224, grid, st);
  if (a->dbias) bigdl_split_reduce_f32(a->ws + (size_t)grid * 64 * 224, a->dbias, 64, grid, st);
  return 0;
}

}  // extern "C"
