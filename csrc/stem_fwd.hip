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
