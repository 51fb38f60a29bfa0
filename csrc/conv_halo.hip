// Forward / data-gradient 3x3, stride-1, pad-1 convolutions from halo tiles (gfx950).
//
// out[p][k] = sum over taps (dh, dw) in [-1, 1]^2 and channels c of x[p + (dh, dw)][c] * w[k][tap][c]
// (reference: S/nn/SpatialConvolution.scala updateOutput / updateGradInput, the MKL-DNN forward and backward-data
// primitives of S/nn/mkldnn/SpatialConvolution.scala:331-589). The data gradient of a 3x3 / stride-1 / pad-1
// convolution is the same computation over dy with the (C, R, S, K) transposed weight and the taps flipped, which
// conv2d_dgrad already describes through ConvArgs' tap table, so one kernel serves both passes.
//
// The im2col implicit-GEMM tiles (conv_igemm.hip conv_nt_g4 / p8) DMA one input granule per (pixel, tap): every
// activation crosses the DMA engine 9 times, and a 128 x 128 tile brings in 64 FLOP per staged byte. ResNet-50's 3x3
// layers ran at 4-6x their MFMA bound there (profiles/r4_resnet50_layer_roofline.txt). Here a workgroup stages a
// halo tile of the input ONCE per 32-channel chunk and reads the 9 shifted windows out of LDS:
//   * tile = NIMG segments of RB output rows (RB < H: one segment of an image; RB == H: NIMG whole images stacked
//     with one shared zero row between them). Its rows are stored padded by one zero column on each side (WP = W + 2
//     "virtual pixel" columns), behind one guard row, so output virtual pixel v = (vr, j) reads tap (dh, dw) at tile
//     row v + 1 + (1 + dh) * WP + dw: a constant shift per tap, no masks (the wgrad_halo.hip layout). Virtual pixels
//     on the pad columns / separator rows compute garbage that the epilogue never stores.
//   * x chunks (32 channels = one 64-byte row per tile row) are double-buffered and issued 9 K-steps ahead; the
//     weights of one (chunk, tap) K-step (KT rows of 64 B) stream through an NSW-slot ring D = NSW - 1 steps ahead.
//     Everything moves by LDS-DMA (buffer_load ... lds) with precomputed per-lane offsets; halo rows and columns
//     outside the image are offsets past num_records, which the buffer unit returns as zeros.
//   * 64-byte rows hold granule g of row r in slot g ^ (2 * ((r >> 2) & 1)): every ds_read_b128 fragment read (16
//     consecutive rows, 4 granules) is conflict-free for ANY row offset, so one swizzle serves all 9 tap shifts, and
//     fragment fm of a wave (16 rows further) has the same swizzle: one address per K-step + immediate offsets.
//   * staged FLOP per byte: 256 virtual pixels x 64 channels (W = 56) or 224 x 128 (W <= 28) per K-step against one
//     4 / 8 KB weight slice plus 1/9 of a chunk: 130-200, 2-3x the im2col tile.
// 4 waves (WPX pixel groups x WCH channel groups), 2 workgroups per CU; the fused epilogue is nt_epilogue_lds
// (conv_epilogue.h) with a virtual-pixel row map: BN statistics, the consumer-BN backward reduction, addend, ReLU.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "common.h"
#include "kernels.h"
#include "conv_epilogue.h"

namespace {

__device__ __forceinline__ int hswz(int r) { return ((r >> 2) & 1) << 1; }

template <int W, int RB, int NIMG, int KT, int WPX>
struct HaloF {
  static constexpr int WP = W + 2;
  static constexpr int VR = NIMG * (RB + 1) - 1;                 // virtual output rows
  static constexpr int VM = 16 * WPX;                            // virtual pixels rounded to whole wave groups
  static constexpr int V = (VR * WP + VM - 1) / VM * VM;         // virtual pixels per tile
  static constexpr int HR = NIMG * (RB + 1) + 1;                 // halo rows (incl. top / bottom / separators)
  static constexpr int XROWS = V + 2 * WP + 2;                   // tile rows any tap of any virtual pixel reads
  static constexpr int XI = (XROWS + 63) / 64;                   // x DMA instructions per thread per chunk
  static constexpr int XR = XI * 64;
  static constexpr int XBYTES = XR * 64;
  static constexpr int WI = KT / 64;                             // weight DMA instructions per thread per step
  static constexpr int WBYTES = KT * 64;
  static constexpr int NSW = 4, D = NSW - 1;
  static constexpr int LDS = 2 * XBYTES + NSW * WBYTES;
  static constexpr int WCH = 4 / WPX;
  static constexpr int TM = V / WPX, TN = KT / WCH;
  static constexpr int FM = TM / 16, FN = TN / 16;
  static_assert(V % (16 * WPX) == 0 && KT % (16 * WCH) == 0 && KT % 64 == 0, "tile");
  static_assert(2 * LDS <= 160 * 1024, "two workgroups per CU");
};

template <int N>
__device__ __forceinline__ void vmw() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int OFF>
__device__ __forceinline__ v8s ldsr(unsigned addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  v8s r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "n"(OFF));
  return r;
}

template <class F, int... I>
__device__ __forceinline__ void hfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void hfor(F&& f) {
  hfor_impl(f, std::make_integer_sequence<int, N>{});
}

// Virtual pixel -> output row (-1: pad column, separator row, tail, or an image past the batch)
template <int W, int RB, int NIMG>
struct HaloRowMap {
  int n0, oh0, vend;
  __device__ __forceinline__ long operator()(const ConvArgs& a, int v) const {
    constexpr int WP = W + 2;
    if (v >= vend) return -1;
    const int vr = v / WP, j = v - vr * WP;
    if (j < 1 || j > W) return -1;
    const int b = vr / (RB + 1), i = vr - b * (RB + 1);
    if (i == RB) return -1;                                   // separator row between stacked images
    const int n = n0 + b;
    if (n >= a.Nb) return -1;
    return ((long)n * a.OH + oh0 + i) * a.OW + (j - 1);
  }
};

// Full form, straight from the accumulators (a lane owns 4 consecutive channels of one pixel per fragment): bias,
// residual addend (fp32 add before rounding), ReLU, 8-byte stores, BN statistics or the consumer-BN backward reduction
// of the rounded gradient under the z / sign-mask / affine ReLU mask (nt_epilogue_lds semantics). Every optional
// operand is loaded unconditionally from its own buffer (a null operand gets num_records 0: loads return 0).
template <int FM, int FN, int WCH, int KT, class RM>
__device__ __forceinline__ void halo_epi_full(const ConvArgs& a, v4f (&acc)[FM][FN], int vbase, int nbase, int lane,
                                              int bid, const RM& rm, float* rl0, int k0) {
  float* rl = rl0 + (threadIdx.x >> 6) * 128;
  const size_t rows = (size_t)a.Nb * a.OH * a.OW;
  const size_t nb2 = ((rows - 1) * a.ldo + a.Ncol) * 2;
  const __amdgpu_buffer_rsrc_t ro = rsrc_of(a.out, nb2);
  const __amdgpu_buffer_rsrc_t rad = rsrc_of(a.addend, a.addend ? nb2 : 0);
  const bool bnw = a.bnred != nullptr && a.stats == nullptr;
  const __amdgpu_buffer_rsrc_t rbx = rsrc_of(a.bnx, bnw ? nb2 : 0);
  const __amdgpu_buffer_rsrc_t rbz = rsrc_of(a.bnz, (bnw && a.bnz) ? nb2 : 0);
  const __amdgpu_buffer_rsrc_t rzm = rsrc_of(a.bnzm, (bnw && a.bnzm) ? nb2 / 16 : 0);
  const __amdgpu_buffer_rsrc_t rzad = rsrc_of(a.addzm, a.addzm ? nb2 / 16 : 0);
  const int c4 = 4 * (lane >> 4);
  float bs[FN][4], mu[FN][4], sc[FN][4], sh[FN][4], s1[FN][4], s2[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = nbase + j * 16 + c4 + e;
      bs[j][e] = a.bias ? a.bias[c] : 0.f;
      mu[j][e] = bnw ? a.bnmean[c] : 0.f;
      sc[j][e] = (bnw && a.bnaff) ? a.bnaff[c] : 0.f;
      sh[j][e] = (bnw && a.bnaff) ? a.bnaff[a.Ncol + c] : 0.f;
      s1[j][e] = s2[j][e] = 0.f;
    }
  const bool relu = a.relu != 0, st = a.stats != nullptr;
  const int zmode = !bnw ? 0 : a.bnzm ? 1 : a.bnz ? 2 : a.bnaff ? 3 : 0;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const long orow = rm(a, vbase + i * 16 + (lane & 15));
    const float vm = orow >= 0 ? 1.f : 0.f;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const size_t el = (size_t)(orow >= 0 ? orow : 0) * a.ldo + nbase + j * 16 + c4;
      const unsigned off = orow >= 0 ? (unsigned)(el * 2) : EOOB;
      v2u ad = __builtin_amdgcn_raw_buffer_load_b64(rad, off, 0, 0);
      if (a.addzm) {
        const unsigned zb2 = __builtin_amdgcn_raw_buffer_load_b8(rzad, orow >= 0 ? (unsigned)(el >> 3) : EOOB, 0, 0);
        const unsigned bits = (zb2 >> (el & 7)) & 0xfu;
        ad[0] &= ((bits & 1u) ? 0xffffu : 0u) | ((bits & 2u) ? 0xffff0000u : 0u);
        ad[1] &= ((bits & 4u) ? 0xffffu : 0u) | ((bits & 8u) ? 0xffff0000u : 0u);
      }
      const v2u bx = __builtin_amdgcn_raw_buffer_load_b64(rbx, off, 0, 0);
      const v2u bz = __builtin_amdgcn_raw_buffer_load_b64(rbz, off, 0, 0);
      const unsigned zb = __builtin_amdgcn_raw_buffer_load_b8(rzm, orow >= 0 ? (unsigned)(el >> 3) : EOOB, 0, 0);
      const float adf[4] = {lo_bf(ad[0]), hi_bf(ad[0]), lo_bf(ad[1]), hi_bf(ad[1])};
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = acc[i][j][e] + bs[j][e] + adf[e];
        if (relu) t = fmaxf(t, 0.f);
        v[e] = t;
      }
      const v2u o = {pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
      __builtin_amdgcn_raw_buffer_store_b64(o, ro, off, 0, 0);
      const float y[4] = {lo_bf(o[0]) * vm, hi_bf(o[0]) * vm, lo_bf(o[1]) * vm, hi_bf(o[1]) * vm};
      if (st) {
#pragma unroll
        for (int e = 0; e < 4; ++e) { s1[j][e] += y[e]; s2[j][e] += y[e] * y[e]; }
      } else if (bnw) {
        const float xf[4] = {lo_bf(bx[0]), hi_bf(bx[0]), lo_bf(bx[1]), hi_bf(bx[1])};
        const float zf[4] = {lo_bf(bz[0]), hi_bf(bz[0]), lo_bf(bz[1]), hi_bf(bz[1])};
        const unsigned zbits = (zb >> ((nbase + j * 16 + c4) & 7)) & 0xfu;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bool keep = true;
          if (zmode == 1) keep = (zbits >> e) & 1u;
          else if (zmode == 2) keep = zf[e] > 0.f;
          else if (zmode == 3) keep = xf[e] * sc[j][e] + sh[j][e] > 0.f;
          const float d = keep ? y[e] : 0.f;
          s1[j][e] += d;
          s2[j][e] += d * (xf[e] - mu[j][e]);
        }
      }
    }
  }
  float* const red = st ? a.stats : (bnw ? a.bnred : nullptr);
  if (red) {
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s1[j][e] += __shfl_xor(s1[j][e], o, 64);
          s2[j][e] += __shfl_xor(s2[j][e], o, 64);
        }
    if ((lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) { rl[j * 16 + c4 + e] = s1[j][e]; rl[64 + j * 16 + c4 + e] = s2[j][e]; }
    }
    halo_commit<WCH, KT>(red, rl0, k0, a.Ncol, bid);
  }
}


// int8 epilogue, straight from the i32 accumulators (lane: 4 consecutive channels of one pixel per fragment):
// dequantize (per-sample input scale x per-channel weight scale), + bias, ReLU, then requantized int8 (4-byte
// groups), fp32 or bf16 stores (quant.hip i8_tile_epilogue_direct semantics; no residual addend here).
template <int FM, int FN, class RM>
__device__ __forceinline__ void halo_epi_i8(const ConvArgs& a, const I8Epi& ep, v4i (&acc)[FM][FN], int vbase,
                                            int nbase, int lane, const RM& rm) {
  const int ohw = a.OH * a.OW;
  const int nl = 4 * (lane >> 4), ml = lane & 15;
  const bool q8 = ep.out_mode == 2;
  const float oi = q8 ? ep.out_inv : 1.f;
  // per-channel scales / bias as 16-byte loads, the bias through a buffer resource (0 bytes without one): the
  // per-element `a.bias ? a.bias[n] : 0` loads were waited for one by one at the branch joins
  float ws[FN][4], bs[FN][4];
  {
    const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.bias), (short)0,
                                                                        a.bias ? a.Ncol * 4 : 0, 0x00020000);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = nbase + j * 16 + nl;
      const v4f w = *reinterpret_cast<const v4f*>(ep.wscale + n);
      const v4f b = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(rb, (unsigned)(n * 4), 0, 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        ws[j][e] = w[e] * oi;
        bs[j][e] = b[e] * oi;
      }
    }
  }
  // branch-free rows: the per-sample scale through a buffer resource (0 bytes without one), rows without an output
  // stored at an out-of-range offset (a skipped row / `xscale ? xscale[..] : c` was a wait at each join)
  const int esz = q8 ? 1 : ep.out_mode == 1 ? 4 : 2;
  const size_t orows_n = a.ident_out ? (size_t)a.M : (size_t)a.Nb * a.OHo * a.OWo;
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
      a.out, (short)0, (int)min(((orows_n - 1) * a.ldo + a.Ncol) * esz, (size_t)0x7fffffff), 0x00020000);
  const __amdgpu_buffer_rsrc_t rxs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ep.xscale), (short)0,
                                                                       ep.xscale ? a.Nb * 4 : 0, 0x00020000);
  const float xs0 = ep.xscale ? 0.f : ep.xs_const;
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const long orow = rm(a, vbase + i * 16 + ml);
    const float xl = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                   rxs, orow >= 0 ? (unsigned)(orow / ohw * 4) : EOOB, 0, 0));
    const float xs = xl + xs0;         // xl reads 0 without per-sample scales
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = nbase + j * 16 + nl;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[e] = (float)acc[i][j][e] * (xs * ws[j][e]) + bs[j][e];
        if (a.relu) v[e] = fmaxf(v[e], 0.f);
      }
      const unsigned off = orow >= 0 ? (unsigned)(((size_t)orow * a.ldo + n) * esz) : EOOB;
      if (q8) {
        unsigned pk = 0u;
#pragma unroll
        for (int e = 0; e < 4; ++e) pk |= (unsigned)(max(-127, min(127, __float2int_rn(v[e]))) & 0xff) << (8 * e);
        __builtin_amdgcn_raw_buffer_store_b32(pk, ro, off, 0, 0);
      } else if (ep.out_mode == 1) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, v4f{v[0], v[1], v[2], v[3]}), ro, off, 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b64(v2u{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])}, ro, off, 0, 0);
      }
    }
  }
}

// ABL (timing ablations, BIGDL_CONV_HALO_ABL, wrong outputs): bit 0 no epilogue, bit 1 no MFMAs, bit 2 no DMA after
// the prologue (stale LDS), bit 3 no fragment reads
// EPI: 0 lean epilogue (no addend / consumer-BN reduction), 2 lean + consumer-BN reduction, 1 full epilogue,
// 3 int8 (EB = 1: int8 activations and weights, 64-channel chunks on v_mfma_i32_16x16x64_i8, I8Epi epilogue)
// PRE: the source is the input of a training BatchNorm + ReLU (ConvArgs::pre = [scale | shift], C <= PRE_MAXC): each
// lane rewrites the granules it staged, relu(x * scale + shift) rounded to bf16 (bn_apply_kernel's expression), once
// its own DMA has landed and before the barrier that publishes the chunk; granules of halo / pad rows (out-of-range
// offsets, read as zeros) are left zero. The per-channel table sits in LDS behind the pipeline buffers.
constexpr int PRE_MAXC = 512;
template <int W, int RB, int NIMG, int KT, int WPX, int EPI, int ABL = 0, int EB = 2, bool PRE = false>
__global__ __launch_bounds__(256, 2) void conv_halo_kernel(ConvArgs a, I8Epi ep) {
  static_assert((EB == 1) == (EPI == 3), "int8 operands go with the int8 epilogue");
  static_assert(!PRE || (EB == 2 && EPI == 0), "BN-on-load: bf16 forwards with the lean epilogue");
  constexpr int CH = 64 / EB;                                 // channels per 64-byte chunk row
  using H = HaloF<W, RB, NIMG, KT, WPX>;
  constexpr int PREB = PRE ? PRE_MAXC * 8 : 0;
  static_assert(2 * (H::LDS + PREB) <= 160 * 1024, "two workgroups per CU");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[H::LDS + PREB];
  constexpr int WCH = H::WCH, FM = H::FM, FN = H::FN, WP = H::WP;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wpx = wave / WCH, wch = wave % WCH;
  const int C = a.Cs, IH = a.Hs;
  const int tiles_n = a.Ncol / KT;
  const int segs = IH / RB;                                   // RB < H: segments per image; RB == H: 1
  const int tiles_m = NIMG == 1 ? a.Nb * segs : (a.Nb + NIMG - 1) / NIMG;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int n0 = NIMG == 1 ? tm / segs : tm * NIMG;
  const int oh0 = NIMG == 1 ? (tm - n0 * segs) * RB : 0;
  const int k0 = tn * KT;
  const int nch = C / CH, nk = nch * 9;

  // ---- x DMA: instruction d of wave w fills tile rows (d * 4 + w) * 16 + lane / 4, slot lane & 3 (granule
  // (lane & 3) ^ hswz(row)). Offsets (bytes) from the segment base pixel (n0, oh0 - 1, 0); variant bit 0 / 1 = the
  // top / bottom halo row lies outside the image (RB < H only; RB == H separators are always zero).
  constexpr unsigned OOB = 0x7ffffff0u;
  // per instruction: its offset, and whether its row is the top / bottom halo row (for RB < H those are zeroed
  // per tile by a uniform select when they fall outside the image; no per-variant copies)
  unsigned xo[H::XI];
  unsigned xtop = 0, xbot = 0;                                  // bit d: instruction d's row is the top / bottom halo
#pragma unroll
  for (int d = 0; d < H::XI; ++d) {
    const int row = (d * 4 + wave) * 16 + (lane >> 2);
    const int g = (lane & 3) ^ hswz(row);
    const int t = row - 1;
    const int hr = t >= 0 ? t / WP : -1, pc = t - hr * WP;
    const int b = hr >= 0 ? hr / (RB + 1) : 0, i = hr - b * (RB + 1);   // i == 0: separator / top halo
    const bool real = t >= 0 && hr < H::HR && pc >= 1 && pc <= W;
    // source image row relative to the segment's first row - 1
    const int srow = NIMG == 1 ? hr : (b * IH + i);
    const bool sep = NIMG == 1 ? false : (i == 0);
    xo[d] = (real && !sep) ? (unsigned)((((srow * W) + (pc - 1)) * C) * EB + g * 16) : OOB;
    if (NIMG == 1 && hr == 0) xtop |= 1u << d;
    if (NIMG == 1 && hr == RB + 1) xbot |= 1u << d;
  }
  // ---- weight DMA: instruction j of wave w fills rows (j * 4 + w) * 16 + lane / 4 of the KT x 64 B slice
  unsigned wo[H::WI];
#pragma unroll
  for (int j = 0; j < H::WI; ++j) {
    const int row = (j * 4 + wave) * 16 + (lane >> 2);
    const int g = (lane & 3) ^ hswz(row);
    wo[j] = (unsigned)((k0 + row) * a.ldw * EB + g * 16);
  }
  const bf16_t* xsrc = reinterpret_cast<const bf16_t*>(a.src);
  const size_t xend = (size_t)a.Nb * IH * W * C;
  // segment base: pixel (n0, oh0 - 1, 0) for RB < H (one image row above; wraps below 0 only when n0 = oh0 = 0, and
  // every top-halo offset is OOB then), pixel (n0, -1, 0) for stacked whole images (row -1 is a separator: OOB)
  const size_t xbase = ((size_t)n0 * IH + oh0) * W * C - (size_t)W * C;
  const bool top_out = NIMG == 1 && oh0 == 0, bot_out = NIMG == 1 && oh0 + RB == IH;
  if (top_out || bot_out) {
#pragma unroll
    for (int d = 0; d < H::XI; ++d)
      if ((top_out && ((xtop >> d) & 1)) || (bot_out && ((xbot >> d) & 1))) xo[d] = OOB;
  }
  const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(reinterpret_cast<const bf16_t*>(a.wt)), (short)0,
      (int)(((size_t)(a.Ncol - 1) * a.ldw + a.Kdim) * EB), 0x00020000);
  // PRE: rows this lane staged from the image (bit d: instruction d's offset is in range), its granule's channels
  unsigned xreal = 0;
  float* const ptab = reinterpret_cast<float*>(lds + H::LDS);
  if constexpr (PRE) {
#pragma unroll
    for (int d = 0; d < H::XI; ++d)
      if (xo[d] != OOB) xreal |= 1u << d;
    for (int i = tid; i < C / 2; i += 256)            // [scale C | shift C] as float4s
      reinterpret_cast<v4f*>(ptab)[i] = reinterpret_cast<const v4f*>(a.pre)[i];
    __syncthreads();
  }
  // granule slot lane & 3 of every row this lane fills holds source granule (lane & 3) ^ hswz(row), and
  // hswz(row) = 2 * ((lane >> 4) & 1) for all of them
  const int pre_c = 8 * ((lane & 3) ^ (((lane >> 4) & 1) << 1));
  auto pre_apply = [&](int ch) {
    if constexpr (PRE) {
      unsigned char* X = lds + (ch & 1) * H::XBYTES;
      const int c = ch * CH + pre_c;
      const v4f s0 = *reinterpret_cast<const v4f*>(ptab + c), s1 = *reinterpret_cast<const v4f*>(ptab + c + 4);
      const v4f b0 = *reinterpret_cast<const v4f*>(ptab + C + c), b1 = *reinterpret_cast<const v4f*>(ptab + C + c + 4);
      const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
      const float sh[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      // every granule's read in flight at once, one wait, then branch-free rewrites (halo / pad granules keep zero)
      const unsigned xa = (unsigned)(uintptr_t)(LDS_PTR(unsigned char))X + (unsigned)(wave * 1024 + lane * 16);
      v4u u[H::XI];
#pragma unroll
      for (int d = 0; d < H::XI; ++d)
        asm volatile("ds_read_b128 %0, %1" : "=v"(u[d]) : "v"(xa + (unsigned)(d * 4096)) : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // tie every loaded value to a volatile asm behind the wait: the arithmetic on it cannot be hoisted above it
#pragma unroll
      for (int d = 0; d < H::XI; ++d) asm volatile("" : "+v"(u[d]));
#pragma unroll
      for (int d = 0; d < H::XI; ++d) {
        const bool real = (xreal >> d) & 1u;
        v4u t;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          t[e] = pack2bf(fmaxf(lo_bf(u[d][e]) * sc[2 * e] + sh[2 * e], 0.f),
                         fmaxf(hi_bf(u[d][e]) * sc[2 * e + 1] + sh[2 * e + 1], 0.f));
        const v4u o = real ? t : u[d];
        asm volatile("ds_write_b128 %0, %1" ::"v"(xa + (unsigned)(d * 4096)), "v"(o) : "memory");
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // the rewritten chunk is complete before the barrier
    }
  };

  auto issue_x = [&](int ch) {
    const size_t xb = xbase + (size_t)ch * CH;                 // elements
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(reinterpret_cast<const char*>(xsrc) + xb * EB), (short)0, (int)((xend - xb) * EB),
        0x00020000);
    unsigned char* X = lds + (ch & 1) * H::XBYTES;
#pragma unroll
    for (int d = 0; d < H::XI; ++d)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (LDS_PTR(void))(X + (d * 4 + wave) * 1024), 16, (int)xo[d], 0, 0, 0);
  };
  // tap tables in SGPRs (the K-loop runs the 9 taps as static iterations): LDS row shift and weight K offset
  int tshift[9], twk[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    tshift[t] = __builtin_amdgcn_readfirstlane(1 + (1 + a.tap_h[t]) * WP + a.tap_w[t]);
    twk[t] = __builtin_amdgcn_readfirstlane(a.tap_k[t] * C * EB);
  }
  auto issue_w = [&](int ch, int t, int slot) {
    const int soff = twk[t] + ch * 64;
    unsigned char* Wt = lds + 2 * H::XBYTES + slot * H::WBYTES;
#pragma unroll
    for (int j = 0; j < H::WI; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, (LDS_PTR(void))(Wt + (j * 4 + wave) * 1024), 16, (int)wo[j],
                                               soff, 0, 0);
  };
  auto issue_ws = [&](int s) {            // weight step s = 9 * chunk + tap (prologue: s < D, static)
    const int ch = s / 9;
    issue_w(ch, s - 9 * ch, s % H::NSW);
  };

  // ---- fragment read addresses: weight rows wch * TN + fn * 16 + (lane & 15), x rows v0 + shift + fm * 16
  const unsigned lds_base = (unsigned)(uintptr_t)(LDS_PTR(unsigned char))lds;
  const int gi = lane >> 4;
  const int wrow = wch * H::TN + (lane & 15);
  const unsigned wrd = (unsigned)(2 * H::XBYTES + wrow * 64 + ((gi ^ hswz(wrow)) << 4));
  const int v0 = wpx * H::TM + (lane & 15);

  using AccT = std::conditional_t<EB == 1, v4i, v4f>;
  AccT acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = AccT{0, 0, 0, 0};

  // prologue: chunk 0 and weight steps 0 .. D-1; retire step 0 (younger: steps 1 .. D-1)
  issue_x(0);
#pragma unroll
  for (int s = 0; s < H::D; ++s)
    if (s < nk) issue_ws(s);
  if (nk > H::D - 1) vmw<(H::D - 1) * H::WI>();
  else vmw<0>();
  pre_apply(0);
  __builtin_amdgcn_s_barrier();

  for (int ch = 0; ch < nch; ++ch) {
    const unsigned xb = lds_base + (unsigned)((ch & 1) * H::XBYTES);
    hfor<9>([&](auto tc) {
      constexpr int t = decltype(tc)::value;
      const int s = ch * 9 + t;
      // slot (s + D) % NSW was read in step s - 1 (retired by the barrier that ended it); x buffer (ch + 1) & 1 was
      // last read by chunk ch - 1
      if (!(ABL & 4) && s + H::D < nk) {
        constexpr int t2 = (t + H::D) % 9, dc = (t + H::D) / 9;
        issue_w(ch + dc, t2, (s + H::D) % H::NSW);
      }
      if (!(ABL & 4) && t == 0 && ch + 1 < nch) issue_x(ch + 1);
      const int r0 = v0 + tshift[t];
      const unsigned xrd = xb + (unsigned)(r0 * 64 + ((gi ^ hswz(r0)) << 4));
      const unsigned wrs = lds_base + wrd + (unsigned)((s % H::NSW) * H::WBYTES);
      v8s fw[FN], fx[FM];
      if constexpr (ABL & 8) {
        hfor<FN>([&](auto jc) { fw[decltype(jc)::value] = v8s{(short)(xrd & 7), 1, 2, 3, 4, 5, 6, 7}; });
        hfor<FM>([&](auto ic) { fx[decltype(ic)::value] = v8s{(short)(wrs & 7), 1, 2, 3, 4, 5, 6, 7}; });
      } else {
        hfor<FN>([&](auto jc) {
          constexpr int j = decltype(jc)::value;
          fw[j] = ldsr<j * 16 * 64>(wrs);
        });
        hfor<FM>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          fx[i] = ldsr<i * 16 * 64>(xrd);
        });
      }
      // pixel fragment i's MFMAs start once it landed (the weight fragments were read first); the tie keeps every
      // use of fx[i] behind its wait
      hfor<FM>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(fx[i]) : "n"(FM - 1 - i));
        if constexpr (!(ABL & 2)) {
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            if constexpr (EB == 1)
              acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(__builtin_bit_cast(v4i, fw[j]), __builtin_bit_cast(v4i, fx[i]),
                                                               acc[i][j], 0, 0, 0);
            else
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[j], fx[i], acc[i][j], 0, 0, 0);
          }
        } else {
          acc[i][0][0] += fw[0][0] * fx[i][0];
        }
      });
      __builtin_amdgcn_sched_barrier(0);
      // retire step s + 1 for every wave: younger than W(s + 1) are W(s + 2 .. s + D) and the x chunk issued at this
      // chunk's start when that start lies in [s + 1 - D, s] (it was issued after W(D) = W(s + 1) or later)
      if (s + H::D < nk) {
        if (t + 1 - H::D <= 0 && ch + 1 < nch) vmw<(H::D - 1) * H::WI + H::XI>();
        else vmw<(H::D - 1) * H::WI>();
      } else {
        vmw<0>();
      }
      // chunk ch + 1 (issued at t = 0) is older than weight step s + 1 from t = D on: this lane's part has landed
      if constexpr (PRE && t == H::D) {
        if (ch + 1 < nch) pre_apply(ch + 1);
      }
      __builtin_amdgcn_s_barrier();
    });
  }

  if constexpr (ABL & 1) {
    float t = 0.f;                                 // keep every accumulator (and so every MFMA) alive
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
    if (t == 123.f) a.out[0] = 1;
    return;
  }
  const HaloRowMap<W, RB, NIMG> rm{n0, oh0, H::VR * WP};
  // per-wave channel sums go behind the bf16 slices (lean) or at the start of the idle LDS (full)
  if constexpr (EPI == 3) {
    halo_epi_i8<FM, FN>(a, ep, acc, wpx * H::TM, k0 + wch * H::TN, lane, rm);
  } else if constexpr (EPI == 0 || EPI == 2) {
    static_assert(4 * H::TM * 128 + 4 * 128 * 4 <= H::LDS, "bf16 epilogue slices must fit the LDS");
    halo_epi_lean<FM, FN, WCH, KT, EPI == 2>(a, acc, wpx * H::TM, k0 + wch * H::TN, lane, bid,
                                             lds + wave * H::TM * 128, rm,
                                             reinterpret_cast<float*>(lds + 4 * H::TM * 128), k0);
  } else {
    halo_epi_full<FM, FN, WCH, KT>(a, acc, wpx * H::TM, k0 + wch * H::TN, lane, bid, rm, reinterpret_cast<float*>(lds),
                                   k0);
  }
}

int g_conv_halo_bn = 1;     // BIGDL_CONV_HALO_BN=0: data gradients with a BN reduction take the full epilogue

template <int W, int RB, int NIMG, int KT, int WPX>
void launch_halo_f(const ConvArgs& a, hipStream_t st) {
  const int segs = a.Hs / RB;
  const int tiles_m = NIMG == 1 ? a.Nb * segs : (a.Nb + NIMG - 1) / NIMG;
  const int nwg = tiles_m * (a.Ncol / KT);
  static const int abl = [] { const char* e = getenv("BIGDL_CONV_HALO_ABL"); return e ? atoi(e) : 0; }();
  const bool lean = a.addend == nullptr && (a.bnred == nullptr || a.stats != nullptr);
  const bool leanbn = a.addend == nullptr && a.bnred != nullptr && a.stats == nullptr && a.bias == nullptr &&
                      (a.bnz == nullptr || a.bnzm != nullptr);
  const dim3 g(nwg), b(256);
  if (abl == 1) conv_halo_kernel<W, RB, NIMG, KT, WPX, 0, 1><<<g, b, 0, st>>>(a, I8Epi{});
  else if (abl == 3) conv_halo_kernel<W, RB, NIMG, KT, WPX, 0, 3><<<g, b, 0, st>>>(a, I8Epi{});
  else if (abl == 5) conv_halo_kernel<W, RB, NIMG, KT, WPX, 0, 5><<<g, b, 0, st>>>(a, I8Epi{});
  else if (abl == 9) conv_halo_kernel<W, RB, NIMG, KT, WPX, 0, 9><<<g, b, 0, st>>>(a, I8Epi{});
  else if (abl == 13) conv_halo_kernel<W, RB, NIMG, KT, WPX, 0, 13><<<g, b, 0, st>>>(a, I8Epi{});
  else if (abl == 15) conv_halo_kernel<W, RB, NIMG, KT, WPX, 0, 15><<<g, b, 0, st>>>(a, I8Epi{});
  else if (lean && a.pre) conv_halo_kernel<W, RB, NIMG, KT, WPX, 0, 0, 2, true><<<g, b, 0, st>>>(a, I8Epi{});
  else if (lean) conv_halo_kernel<W, RB, NIMG, KT, WPX, 0><<<g, b, 0, st>>>(a, I8Epi{});
  else if (leanbn && g_conv_halo_bn) conv_halo_kernel<W, RB, NIMG, KT, WPX, 2><<<g, b, 0, st>>>(a, I8Epi{});
  else conv_halo_kernel<W, RB, NIMG, KT, WPX, 1><<<g, b, 0, st>>>(a, I8Epi{});
}

// ------------------------------------------------------------------------------------------------
// int8 image stem (7x7 / stride 2 / pad 3, 64 output channels, 224 -> 112) over the width im2col the input quantizer
// writes (quant.hip quantize_wim2col_f32: row (n, h, ow) = 32 bytes, byte e * 4 + c = q(x[c][h][2 ow + e - 3])): an
// R x 1 convolution with a reduction of 7 x 32 bytes. A workgroup stages the 13 input rows its 4 output rows need
// (one contiguous block of the im2col, LDS-DMA; rows above / below the image come back as zeros through out-of-range
// buffer offsets) plus the 64 x 224 weight (rows padded to 256 bytes, taps 7 zero); each wave computes one output row
// (7 fragments of 16 columns x 64 channels) in 4 K-steps of v_mfma_i32_16x16x64_i8, a K-step = two row taps (lane
// group g: row tap 2 s + (g >> 1), bytes (g & 1) * 16 of the 32-byte column). Integer accumulation: bit-equal to the
// generic int8 implicit GEMM (conv_i8_g3). Epilogue: halo_epi_i8 (dequantize, bias, ReLU, requantize / bf16 / fp32).
constexpr int SI_RB = 4, SI_OW = 112, SI_ROW = SI_OW * 32, SI_XROWS = 2 * SI_RB + 5;   // 13 staged input rows
constexpr int SI_XCH = (SI_XROWS * SI_ROW + 1023) / 1024;                           // 1 KiB DMA chunks (46)
constexpr int SI_XG = (SI_XCH + 3) / 4;                                               // chunks per wave
constexpr int SI_XB = (SI_XROWS + 1) * SI_ROW;    // + the row wave 3's zero-weight tap 7 reads
constexpr int SI_WST = 272;                       // weight row stride (256 bytes + 16: conflict-free reads)
constexpr int SI_WOFF = ((SI_XG * 4 * 1024 > SI_XB ? SI_XG * 4 * 1024 : SI_XB) + 1023) / 1024 * 1024;
constexpr int SI_LDS = SI_WOFF + 64 * SI_WST;

struct LinRowMap {
  long base;
  __device__ __forceinline__ long operator()(const ConvArgs&, int v) const { return base + v; }
};

__global__ __launch_bounds__(256, 2) void stem_i8_kernel(ConvArgs a, I8Epi ep) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[SI_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_img = a.OH / SI_RB;
  const int bid = xcd_remap(blockIdx.x, a.Nb * tiles_img);
  const int n = bid / tiles_img, oh0 = (bid - n * tiles_img) * SI_RB;
  // im2col rows 2 oh0 - 3 .. 2 oh0 + 9 of image n; offsets before the image wrap to huge unsigned values, past it
  // they exceed the record count: both read as zeros
  const int8_t* src = reinterpret_cast<const int8_t*>(a.src) + (size_t)n * a.Hs * SI_ROW;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<int8_t*>(src), (short)0,
                                                                      a.Hs * SI_ROW, 0x00020000);
  const int row0 = (2 * oh0 - 3) * SI_ROW;
#pragma unroll
  for (int d = 0; d < SI_XG; ++d) {
    const int ch = d * 4 + wave;
    if (ch < SI_XCH)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (LDS_PTR(void))(lds + ch * 1024), 16,
                                               (int)(unsigned)(row0 + (ch * 64 + lane) * 16), 0, 0, 0);
  }
  // weights [64][224] -> rows of 256 (+16) bytes, bytes 224..255 (row tap 7) zero
  const int8_t* wt = reinterpret_cast<const int8_t*>(a.wt);
#pragma unroll
  for (int q = tid; q < 64 * 16; q += 256) {
    const int k = q >> 4, gr = q & 15;
    const v4u v = gr < 14 ? *reinterpret_cast<const v4u*>(wt + (size_t)k * a.ldw + gr * 16) : v4u{0u, 0u, 0u, 0u};
    *reinterpret_cast<v4u*>(lds + SI_WOFF + k * SI_WST + gr * 16) = v;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  constexpr int FM = SI_OW / 16;
  v4i acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  const int g = lane >> 4, col = lane & 15;
  const unsigned char* Wl = lds + SI_WOFF + col * SI_WST + g * 16;
  const unsigned char* Xl = lds + (2 * wave + (g >> 1)) * SI_ROW + col * 32 + (g & 1) * 16;
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    v4i fw[4], fx[FM];
#pragma unroll
    for (int j = 0; j < 4; ++j) fw[j] = *reinterpret_cast<const v4i*>(Wl + j * 16 * SI_WST + st * 64);
#pragma unroll
    for (int i = 0; i < FM; ++i) fx[i] = *reinterpret_cast<const v4i*>(Xl + 2 * st * SI_ROW + i * 16 * 32);
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fw[j], fx[i], acc[i][j], 0, 0, 0);
  }
  const LinRowMap rm{((long)n * a.OH + oh0) * SI_OW};
  halo_epi_i8<FM, 4>(a, ep, acc, wave * SI_OW, 0, lane, rm);
}

// The same stem straight from the fp32 NCHW image (C <= 3 channels, 224 x 224): the workgroup stages its 13 input
// rows x 3 channel planes as fp32 (lane-gathered LDS-DMA: 39 row segments of 896 bytes, rows outside the image read
// as zeros), quantizes every staged pixel once into an int8 plane [13 rows][3 + 224 + 5 pixels][4 channel bytes]
// (the quantizer's exact expression, rint(x * inv) clamped to +-127), and reads each MFMA operand — 4 width taps x 4
// channel bytes of one output column, the 16 bytes the width im2col would hold — as 16 contiguous plane bytes
// (pixels 2 ow + 4 (g & 1) .. + 3; the 4th tap of the upper group is tap 7, whose weights are zero). No im2col
// tensor is written or read: the quantize pass (~0.13 ms at batch 256) and the im2col read disappear.
constexpr int SF_W = 224, SF_SEG = SF_W * 4, SF_NSEG = SI_XROWS * 3;                  // 896-byte row segments
constexpr int SF_GR = SF_NSEG * (SF_SEG / 16);                                          // 2184 granules
constexpr int SF_CH = (SF_GR + 63) / 64, SF_XG = (SF_CH + 3) / 4;                       // 35 chunks, 9 per wave
constexpr int SF_PW = 232;                                   // int8 plane row: 3 pad + 224 + 5 pad pixels x 4 bytes
constexpr int SF_POFF = SF_XG * 4 * 1024;
constexpr int SF_WOFF = (SF_POFF + SI_XROWS * SF_PW * 4 + 1023) / 1024 * 1024;
constexpr int SF_LDS = SF_WOFF + 64 * SI_WST;

__global__ __launch_bounds__(256, 2) void stem_i8f_kernel(ConvArgs a, I8Epi ep, const float* __restrict__ img, int C,
                                                          float inv) {
  __shared__ __attribute__((aligned(1024))) unsigned char lds[SF_LDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_img = a.OH / SI_RB;
  const int bid = xcd_remap(blockIdx.x, a.Nb * tiles_img);
  const int n = bid / tiles_img, oh0 = (bid - n * tiles_img) * SI_RB;
  const int H = a.Hs;
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), (short)0,
                                                                      (int)((size_t)a.Nb * C * H * SF_SEG), 0x00020000);
  // LDS segment sg = t * 3 + c holds image row 2 oh0 - 3 + t of channel c (zeros for c >= C or rows off the image)
#pragma unroll
  for (int d = 0; d < SF_XG; ++d) {
    const int ch = d * 4 + wave;
    const int q = ch * 64 + lane, sg = q / 56, gi = q - sg * 56;
    const int t = sg / 3, c = sg - t * 3, h = 2 * oh0 - 3 + t;
    const bool ok = q < SF_GR && c < C && h >= 0 && h < H;
    const unsigned off = ok ? (unsigned)((((size_t)n * C + c) * H + h) * SF_SEG + gi * 16) : EOOB;
    if (ch < SF_CH)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (LDS_PTR(void))(lds + ch * 1024), 16, (int)off, 0, 0, 0);
  }
  const int8_t* wt = reinterpret_cast<const int8_t*>(a.wt);
#pragma unroll
  for (int q = tid; q < 64 * 16; q += 256) {
    const int k = q >> 4, gr = q & 15;
    const v4u v = gr < 14 ? *reinterpret_cast<const v4u*>(wt + (size_t)k * a.ldw + gr * 16) : v4u{0u, 0u, 0u, 0u};
    *reinterpret_cast<v4u*>(lds + SF_WOFF + k * SI_WST + gr * 16) = v;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  {
    const float* F = reinterpret_cast<const float*>(lds);
    unsigned* P = reinterpret_cast<unsigned*>(lds + SF_POFF);
    for (int q = tid; q < SI_XROWS * SF_PW; q += 256) {
      const int t = q / SF_PW, w = q - t * SF_PW - 3;
      unsigned u = 0u;
      if ((unsigned)w < (unsigned)SF_W) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int v = max(-127, min(127, __float2int_rn(F[(t * 3 + c) * SF_W + w] * inv)));
          u |= (unsigned)(v & 0xff) << (8 * c);
        }
      }
      P[q] = u;
    }
  }
  __syncthreads();

  constexpr int FM = SI_OW / 16;
  v4i acc[FM][4];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4i{0, 0, 0, 0};
  const int g = lane >> 4, col = lane & 15;
  const unsigned char* Wl = lds + SF_WOFF + col * SI_WST + g * 16;
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const int r = 2 * st + (g >> 1);                 // row tap of this lane group (7: zero weights, any data)
    const int t = 2 * wave + (r < 7 ? r : 6);
    const unsigned char* Pl = lds + SF_POFF + (t * SF_PW + 2 * col + 4 * (g & 1)) * 4;
    v4i fw[4], fx[FM];
#pragma unroll
    for (int j = 0; j < 4; ++j) fw[j] = *reinterpret_cast<const v4i*>(Wl + j * 16 * SI_WST + st * 64);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const v2u lo = *reinterpret_cast<const v2u*>(Pl + i * 32 * 4), hi = *reinterpret_cast<const v2u*>(Pl + i * 32 * 4 + 8);
      fx[i] = v4i{(int)lo[0], (int)lo[1], (int)hi[0], (int)hi[1]};
    }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fw[j], fx[i], acc[i][j], 0, 0, 0);
  }
  const LinRowMap rm{((long)n * a.OH + oh0) * SI_OW};
  halo_epi_i8<FM, 4>(a, ep, acc, wave * SI_OW, 0, lane, rm);
}

int g_conv_halo = -1;

template <int W, int RB, int NIMG, int KT, int WPX>
void launch_halo_i8(const ConvArgs& a, const I8Epi& ep, hipStream_t st) {
  const int segs = a.Hs / RB;
  const int tiles_m = NIMG == 1 ? a.Nb * segs : (a.Nb + NIMG - 1) / NIMG;
  const int nwg = tiles_m * (a.Ncol / KT);
  conv_halo_kernel<W, RB, NIMG, KT, WPX, 3, 0, 1><<<dim3(nwg), dim3(256), 0, st>>>(a, ep);
}

}  // namespace

extern "C" {

void bigdl_set_conv_halo(int v) { g_conv_halo = v; }

// 1 when bigdl_conv_halo takes this forward / data-gradient GEMM (BIGDL_CONV_HALO=0 turns it off; 2 / 3: see below)
int bigdl_conv_halo_applies(const ConvArgs* a) {
  if (g_conv_halo < 0) {
    const char* e = getenv("BIGDL_CONV_HALO");
    // default 1: forwards and data gradients (those with a consumer-BN reduction and no addend take the lean
    // epilogue with preloaded BN operands: 23.81 ms/step vs 24.20 with the data gradients on the im2col kernels;
    // 2 = forwards only, 3 = all but the 56 x 56 data gradients)
    g_conv_halo = e ? atoi(e) : 1;
  }
  if (!g_conv_halo || a->ntaps != 9 || a->mul_h != 1 || a->mul_w != 1 || !a->ident_out || a->out32 || a->pstride ||
      a->Hs != a->OH || a->Ws != a->OW || a->Hs != a->Ws || a->Kdim != 9 * a->Cs || (a->Cs % 32) ||
      (a->ldo % 8) || (a->Ncol % 8) || a->ldw < a->Kdim || (a->ldw % 8))
    return 0;
  const int W = a->Ws;
  const int kt = W == 56 ? 64 : 128;
  if (W != 56 && W != 28 && W != 14 && W != 7) return 0;
  // 2: only GEMMs with the lean epilogue (forwards); 3: also the full epilogue (data gradients) except at 56 x 56
  const bool lean = a->addend == nullptr && (a->bnred == nullptr || a->stats != nullptr);
  if ((g_conv_halo == 2 && !lean) || (g_conv_halo == 3 && !lean && W == 56)) return 0;
  if (a->Ncol % kt) return 0;
  unsigned seen = 0;
  for (int t = 0; t < 9; ++t) {
    if (a->tap_h[t] < -1 || a->tap_h[t] > 1 || a->tap_w[t] < -1 || a->tap_w[t] > 1 || a->tap_k[t] < 0 ||
        a->tap_k[t] > 8)
      return 0;
    seen |= 1u << ((a->tap_h[t] + 1) * 3 + a->tap_w[t] + 1);
  }
  if (seen != 0x1ffu) return 0;
  if ((size_t)a->Nb * a->Hs * a->Ws * a->Cs * 2 >= (1ull << 31) - (1ull << 20)) return 0;   // 32-bit buffer offsets
  if ((size_t)a->Ncol * a->ldw * 2 >= (1ull << 31)) return 0;
  // the epilogue reads / writes out, addend, bnx and the masks through the same 32-bit buffer offsets: the whole
  // output extent (bf16 rows of ldo) must fit too (int8 callers go through here with the same bound)
  const size_t M = (size_t)a->Nb * a->OH * a->OW;
  if (((M - 1) * (size_t)a->ldo + a->Ncol) * 2 >= 0x7ff00000ull) return 0;
  // a BN applied on load: the lean epilogue only (no addend / consumer-BN reduction), channel table in LDS
  if (a->pre && (a->addend || (a->bnred && !a->stats) || a->Cs > PRE_MAXC || (g_conv_halo != 1 && g_conv_halo != 2)))
    return 0;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return al(a->src) && al(a->wt) && al(a->out) && al(a->addend) && al(a->bnx) && al(a->bnz);
}

int bigdl_conv_halo(const ConvArgs* a, hipStream_t st) {
  switch (a->Ws) {
    case 56: launch_halo_f<56, 4, 1, 64, 4>(*a, st); break;
    case 28: launch_halo_f<28, 7, 1, 128, 2>(*a, st); break;
    case 14: launch_halo_f<14, 14, 1, 128, 2>(*a, st); break;
    case 7: launch_halo_f<7, 7, 3, 128, 2>(*a, st); break;
    default: return -1;
  }
  return 0;
}

// int8 form (quant.hip bigdl_conv_i8): the same geometry with 64-channel chunks; no residual addend; 4-byte aligned
// output groups. BIGDL_CONV_HALO=0 turns it off too.
int bigdl_conv_halo_i8_applies(const ConvArgs* a, const I8Epi* ep) {
  if (ep->add8 != nullptr || (a->Cs % 64) || (a->Ncol % 4) || (a->ldo % 4) || (a->ldw % 16)) return 0;
  if (g_conv_halo < 0) (void)bigdl_conv_halo_applies(a);     // reads BIGDL_CONV_HALO once
  if (!g_conv_halo) return 0;
  // bigdl_conv_halo_applies's geometry checks, on int8 operands (16-byte aligned rows)
  ConvArgs b = *a;
  b.addend = nullptr; b.bnred = nullptr; b.stats = nullptr;
  const int keep = g_conv_halo;
  g_conv_halo = 1;
  const int ok = bigdl_conv_halo_applies(&b);
  g_conv_halo = keep;
  return ok;
}

// The int8 stem over the width im2col (see stem_i8_kernel): 7 row taps (r - 3) x 1, 32-byte rows, stride (2, 1),
// 112 output columns, 64 channels, no residual. BIGDL_STEM_I8=0 turns it off.
static int g_stem_i8 = -1;
void bigdl_set_stem_i8(int v) { g_stem_i8 = v; }

int bigdl_stem_i8_applies(const ConvArgs* a, const I8Epi* ep) {
  if (g_stem_i8 < 0) {
    const char* e = getenv("BIGDL_STEM_I8");
    g_stem_i8 = e ? atoi(e) : 1;
  }
  if (!g_stem_i8 || ep->add8 != nullptr || a->Cs != 32 || a->ntaps != 7 || a->mul_h != 2 || a->mul_w != 1 ||
      a->Ws != SI_OW || a->OW != SI_OW || a->OH % SI_RB || a->Hs != 2 * a->OH || a->Ncol != 64 || a->ldw != 224 ||
      a->Kdim != 224 || !a->ident_out || a->ldo % 4 || a->ldo < 64)
    return 0;
  for (int t = 0; t < 7; ++t)
    if (a->tap_h[t] != t - 3 || a->tap_w[t] != 0 || a->tap_k[t] != t) return 0;
  if ((size_t)a->Hs * SI_ROW >= (1ull << 31)) return 0;
  return 1;
}

int bigdl_stem_i8(const ConvArgs* a, const I8Epi* ep, hipStream_t st) {
  stem_i8_kernel<<<dim3(a->Nb * (a->OH / SI_RB)), dim3(256), 0, st>>>(*a, *ep);
  return 0;
}

// The stem from the fp32 image (stem_i8f_kernel): `a` carries the width-im2col geometry (what bigdl_stem_i8_applies
// checks, Hs = image rows), img the [N][C][Hs][224] fp32 image, inv the quantizer's 1 / scale. -1: not applicable.
int bigdl_stem_i8_f32(const ConvArgs* a, const I8Epi* ep, const float* img, int C, int W, float inv, hipStream_t st) {
  if (!bigdl_stem_i8_applies(a, ep) || W != SF_W || C < 1 || C > 3 || a->src != nullptr) return -1;
  if ((size_t)a->Nb * C * a->Hs * SF_SEG >= (1ull << 31)) return -1;
  stem_i8f_kernel<<<dim3(a->Nb * (a->OH / SI_RB)), dim3(256), 0, st>>>(*a, *ep, img, C, inv);
  return 0;
}

int bigdl_conv_halo_i8(const ConvArgs* a, const I8Epi* ep, hipStream_t st) {
  switch (a->Ws) {
    case 56: launch_halo_i8<56, 4, 1, 64, 4>(*a, *ep, st); break;
    case 28: launch_halo_i8<28, 7, 1, 128, 2>(*a, *ep, st); break;
    case 14: launch_halo_i8<14, 14, 1, 128, 2>(*a, *ep, st); break;
    case 7: launch_halo_i8<7, 7, 3, 128, 2>(*a, *ep, st); break;
    default: return -1;
  }
  return 0;
}

}  // extern "C"
