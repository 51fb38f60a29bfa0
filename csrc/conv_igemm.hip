// Implicit-GEMM convolution for gfx950 (MI355X), NHWC bf16 activations, fp32 accumulation.
//
// Replaces the reference's per-sample im2col + MKL sgemm path
// (S/nn/SpatialConvolution.scala:253-362 updateOutput, :364-426 updateGradInput, :435-520
// accGradParameters; NNPrimitive.im2colFloat S/nn/NNPrimitive.scala:108) and the MKL-DNN
// conv primitives (S/nn/mkldnn/SpatialConvolution.scala:331-589). Design is MI355X-first:
//
//  * one kernel family for fwd and dgrad ("NT" GEMM: C[m][n] = sum_k A[m][k] * B[n][k]) where the
//    A rows are gathered on the fly from the NHWC source tensor (no im2col buffer in HBM): a 16-byte
//    granule of 8 channels of one input pixel is one lane's global load;
//  * MFMA v_mfma_f32_16x16x32_bf16, 64-lane waves, 4 waves per workgroup, BK = 64;
//  * register-staged, double-buffered LDS tiles with an XOR swizzle of the 16-byte slot by row so the
//    ds_read_b128 fragment reads are spread across banks (cdna_hip_programming.md T2);
//  * operands swapped in the MFMA (weights as the "A" operand) so each lane ends up owning four
//    consecutive output channels of one pixel: 8-byte bf16 stores along the NHWC channel dim;
//  * fused epilogue: + bias, ReLU, and per-channel BatchNorm statistics (sum, sum of squares) reduced
//    across the 16 lanes that share a channel and added with one atomic per channel per wave;
//  * weight-gradient kernel ("TN" GEMM over the pixel dimension) reads both operands from row-major
//    NHWC tiles with the gfx950 transposed LDS read ds_read_b64_tr_b16, split-K over pixels with
//    fp32 atomics into the flat fp32 gradient buffer (bias gradient folded into the same pass);
//  * XCD-aware bijective block remap so neighbouring tiles share an XCD L2.
#include "common.h"
#include "kernels.h"
#include <stdlib.h>

#include "conv_epilogue.h"


namespace {

constexpr int BK = 64;          // K elements per LDS stage (8 granules of 16 B per row)

// 16 zero bytes in global memory: out-of-range lanes (padding taps, tile tails) load from here instead of
// branching around the load, which keeps the staging code branch-free (no exec-mask save/restore).
__device__ __attribute__((aligned(64))) bf16_t g_zero_granule[32];
__device__ __forceinline__ v4u load16(const bf16_t* p, bool ok) {
  return *reinterpret_cast<const v4u*>(ok ? p : g_zero_granule);
}

// Fused epilogue shared by the NT kernels: D[n][m] (weights were the MFMA A operand), so lane owns
// channels n = 4*(lane>>4)+j (j=0..3) of pixel m = lane&15: + bias, + addend, ReLU, bf16 store along the
// NHWC channel dim, per-channel BatchNorm (sum, sumsq) partials with one atomic per channel per wave.
template <int MI, int NI, int TM, int TN>
__device__ __forceinline__ void nt_epilogue(const ConvArgs& a, v4f (&acc)[MI][NI], int mbase, int nbase, int lane,
                                            int bid) {
  const int ohw = a.OH * a.OW;
  const bool vec_ok = (a.Ncol & 3) == 0 && (a.ldo & 3) == 0;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int nb = nbase + j * 16 + (lane >> 4) * 4;
    float bs[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.bias) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bs[e] = (nb + e < a.Ncol) ? a.bias[nb + e] : 0.f;
    }
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = mbase + i * 16 + (lane & 15);
      long orow = m;
      if (!a.ident_out && m < a.M) {
        const int nb = m / ohw, rem = m - nb * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        orow = ((long)nb * a.OHo + oh * a.omul_h + a.ooff_h) * a.OWo + ow * a.omul_w + a.ooff_w;
      }
      float ad[4] = {0.f, 0.f, 0.f, 0.f};
      if (a.addend && m < a.M) {  // fused residual-gradient sum (ResNet block input gradient)
        const bf16_t* ap = a.addend + (size_t)orow * a.ldo + nb;
        if (vec_ok && nb + 3 < a.Ncol) {
          const v2u q = *reinterpret_cast<const v2u*>(ap);
          ad[0] = lo_bf(q[0]); ad[1] = hi_bf(q[0]); ad[2] = lo_bf(q[1]); ad[3] = hi_bf(q[1]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) ad[e] = (nb + e < a.Ncol) ? bf2f(ap[e]) : 0.f;
        }
        if (a.addzm) {
          const size_t el = (size_t)orow * a.ldo + nb;
          const unsigned bits = (a.addzm[el >> 3] >> (el & 7)) & 0xfu;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (!((bits >> e) & 1u)) ad[e] = 0.f;
        }
      }
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = acc[i][j][e] + bs[e] + ad[e];
        if (a.relu) t = fmaxf(t, 0.f);
        v[e] = t;
      }
      const unsigned p0 = pack2bf(v[0], v[1]), p1 = pack2bf(v[2], v[3]);
      if (m < a.M) {
        if (a.stats) {
          s1[0] += lo_bf(p0); s1[1] += hi_bf(p0); s1[2] += lo_bf(p1); s1[3] += hi_bf(p1);
          s2[0] += lo_bf(p0) * lo_bf(p0); s2[1] += hi_bf(p0) * hi_bf(p0);
          s2[2] += lo_bf(p1) * lo_bf(p1); s2[3] += hi_bf(p1) * hi_bf(p1);
        }
        bf16_t* o = a.out + (size_t)orow * a.ldo + nb;
        if (vec_ok && nb + 3 < a.Ncol) {
          *reinterpret_cast<v2u*>(o) = v2u{p0, p1};
        } else {
          const unsigned pp[2] = {p0, p1};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (nb + e < a.Ncol) o[e] = (bf16_t)((pp[e >> 1] >> ((e & 1) * 16)) & 0xffff);
        }
      }
    }
    if (a.stats) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s1[e] += __shfl_xor(s1[e], o, 64);
          s2[e] += __shfl_xor(s2[e], o, 64);
        }
      }
      if ((lane & 15) == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (nb + e < a.Ncol) {
            float* sp = a.stats + (size_t)(bid & (BIGDL_STAT_SLOTS - 1)) * 2 * a.Ncol;  // slot: see batchnorm.hip
            atomicAdd(sp + nb + e, s1[e]);
            atomicAdd(sp + a.Ncol + nb + e, s2[e]);
          }
      }
    }
  }
}

// nt_epilogue_lds (coalescing epilogue through LDS): conv_epilogue.h

template <int BM, int BN, int WM, bool FASTK>
__global__ __launch_bounds__(256, 2) void conv_nt_kernel(ConvArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM, TN = BN / WN;      // per-wave tile
  constexpr int MI = TM / 16, NI = TN / 16;      // MFMA tiles per wave
  constexpr int AROWS = BM / 32, BROWS = BN / 32; // rows loaded per thread per stage
  constexpr int STAGE = (BM + BN) * BK;           // bf16 elements per LDS stage
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (a.Ncol + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  // n fastest: the tiles_n blocks that share one A panel run back to back (same XCD after remap)
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // ---- per-thread A-row precompute (rows fixed through the K loop) ----
  const int lrow = tid >> 3, lg = tid & 7;
  int a_pix[AROWS], a_h[AROWS], a_w[AROWS];
  const int ohw = a.OH * a.OW;
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
  const bf16_t* wrow[BROWS];
  bool bvalid[BROWS];
#pragma unroll
  for (int i = 0; i < BROWS; ++i) {
    const int n = n0 + lrow + 32 * i;
    bvalid[i] = n < a.Ncol;
    wrow[i] = a.wt + (size_t)(bvalid[i] ? n : 0) * a.ldw;
  }

  v4u ra[AROWS], rb[BROWS];
  auto gload = [&](int kt) {
    int t, c, wk;
    bool kvalid;
    if constexpr (FASTK) {
      const int k0 = kt * BK;                 // the whole BK chunk lies in one tap (Cs % BK == 0)
      t = k0 / a.Cs;
      c = k0 - t * a.Cs + lg * 8;
      kvalid = true;
    } else {
      const int kk = kt * BK + lg * 8;
      kvalid = kk < a.Kdim;
      const int kc = kvalid ? kk : 0;
      t = kc / a.Cs;
      c = kc - t * a.Cs;
    }
    const int th = a.tap_h[t], tw = a.tap_w[t];
    wk = a.tap_k[t] * a.Cs + c;
#pragma unroll
    for (int i = 0; i < AROWS; ++i) {
      const int ch = a_h[i] + th, cw = a_w[i] + tw;
      const bool ok = kvalid && (unsigned)ch < (unsigned)a.Hs && (unsigned)cw < (unsigned)a.Ws;
      ra[i] = load16(a.src + (unsigned)((a_pix[i] + ch * a.Ws + cw) * a.Cs + c), ok);
    }
#pragma unroll
    for (int i = 0; i < BROWS; ++i) {
      rb[i] = load16(wrow[i] + wk, bvalid[i] && kvalid);
    }
  };
  auto swz = [](int row, int g) { return row * BK + ((g ^ (row & 7)) << 3); };
  auto swrite = [&](int buf) {
    bf16_t* A = lds + buf * STAGE;
    bf16_t* B = A + BM * BK;
#pragma unroll
    for (int i = 0; i < AROWS; ++i) *reinterpret_cast<v4u*>(A + swz(lrow + 32 * i, lg)) = ra[i];
#pragma unroll
    for (int i = 0; i < BROWS; ++i) *reinterpret_cast<v4u*>(B + swz(lrow + 32 * i, lg)) = rb[i];
  };

  v4f acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int nk = (a.Kdim + BK - 1) / BK;
  gload(0);
  swrite(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kt + 1);   // next stage in flight during the MFMAs
    const bf16_t* A = lds + cur * STAGE;
    const bf16_t* B = A + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      v8s fa[MI], fb[NI];
      const int g = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int row = wm * TM + i * 16 + (lane & 15);
        fa[i] = *reinterpret_cast<const v8s*>(A + swz(row, g));
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int row = wn * TN + j * 16 + (lane & 15);
        fb[j] = *reinterpret_cast<const v8s*>(B + swz(row, g));
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) swrite(cur ^ 1);
    __syncthreads();
  }

  if ((a.Ncol & 7) == 0 && (a.ldo & 7) == 0)
    nt_epilogue_lds<MI, NI, TM, TN>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid,
                                    reinterpret_cast<float*>(lds) + wave * TM * TN);
  else
    nt_epilogue<MI, NI, TM, TN>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid);
}

// ------------------------------------------------------------------------------------------------
// LDS-DMA variant of the NT kernel (Cs % 64 == 0): operands go global -> LDS with
// global_load_lds_dwordx4 (no VGPR staging, no ds_write pass, no address-swizzle VALU on the write
// side). The DMA writes wave-base + 16*lane, so each wave instruction fills 8 rows x 128 B of the
// lane-linear LDS image; the XOR swizzle that keeps the ds_read_b128 fragment reads conflict-free is
// applied on the *source* side: the lane that lands in slot s of row r fetches granule s ^ (r & 7)
// (cdna_hip_programming.md §5 "Async global->LDS copy", T2). Two LDS stages; the DMA for stage k+1 is
// in flight during the MFMAs of stage k and retired by the barrier that ends the step.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ void glds16(const void* g, LDS_PTR(void) l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g, l, 16, 0, 0);
}

// FASTK = false (Cs % 64 != 0, e.g. the 7x7 stem over 8 padded channels): a K stage spans several taps, so each
// lane resolves its own granule's tap (kk = k0 + 8 * gsrc) and zero-fills past Kdim.
// NST = 1: single-K-stage layers (Kdim == BK, the 1x1 convolutions over 64 channels): one LDS stage and a two-chunk
// epilogue (NH = 2) fit the workgroup in 32 KB, so 3 workgroups share a CU (launch bound 3: 168 registers, no spills) and one workgroup's
// operand DMA overlaps the others' epilogue stores on these store-bound layers.
template <int BM, int BN, int WM, bool FASTK = true, int NST = 2>
__global__ __launch_bounds__(256, NST == 1 ? 3 : 2) void conv_nt_glds_kernel(ConvArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int AI = BM / 32, BI = BN / 32;       // DMA instructions per thread per stage (8 rows each x 4 waves)
  constexpr int STAGE = (BM + BN) * BK;
  static_assert(NST == 2 || (NST == 1 && TM * TN * 4 * 2 <= STAGE * 2), "one-stage epilogue must fit the stage");
  __shared__ __attribute__((aligned(1024))) bf16_t lds[NST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (a.Ncol + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  // DMA lane geometry: instruction i of wave w covers rows (i*4 + w)*8 .. +8; lane -> row += lane>>3,
  // slot lane&7, which holds granule (lane&7) ^ (row&7) = (lane ^ (lane>>3)) & 7.
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
  const bf16_t* wrow[BI];
  bool bvalid[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int n = n0 + (i * 4 + wave) * 8 + rsub;
    bvalid[i] = n < a.Ncol;
    wrow[i] = a.wt + (size_t)(bvalid[i] ? n : 0) * a.ldw;
  }

  auto issue = [&](int kt, int buf) {
    const int k0 = kt * BK;
    int th, tw, c, wk;
    bool kv = true;
    if constexpr (FASTK) {                  // the whole stage lies in one tap
      const int t = k0 / a.Cs;
      c = k0 - t * a.Cs + gsrc * 8;
      th = a.tap_h[t]; tw = a.tap_w[t];
      wk = a.tap_k[t] * a.Cs + c;
    } else {                                // per-lane tap of granule kk
      const int kk = k0 + gsrc * 8;
      kv = kk < a.Kdim;
      const int kc = kv ? kk : 0;
      const int t = kc / a.Cs;
      c = kc - t * a.Cs;
      th = a.tap_h[t]; tw = a.tap_w[t];
      wk = a.tap_k[t] * a.Cs + c;
    }
    bf16_t* A = lds + buf * STAGE;
    bf16_t* B = A + BM * BK;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int ch = a_h[i] + th, cw = a_w[i] + tw;
      const bool ok = kv && (unsigned)ch < (unsigned)a.Hs && (unsigned)cw < (unsigned)a.Ws;
      const bf16_t* src = ok ? a.src + (unsigned)((a_pix[i] + ch * a.Ws + cw) * a.Cs + c) : g_zero_granule;
      glds16(src, (LDS_PTR(void))(A + (i * 4 + wave) * 8 * BK));
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const bf16_t* src = (bvalid[i] && kv) ? wrow[i] + wk : g_zero_granule;
      glds16(src, (LDS_PTR(void))(B + (i * 4 + wave) * 8 * BK));
    }
  };
  auto swz = [](int row, int g) { return row * BK + ((g ^ (row & 7)) << 3); };

  v4f acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int nk = NST == 1 ? 1 : (a.Kdim + BK - 1) / BK;
  issue(0, 0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = NST == 1 ? 0 : (kt & 1);
    if (NST == 2 && kt + 1 < nk) issue(kt + 1, cur ^ 1);
    const bf16_t* A = lds + cur * STAGE;
    const bf16_t* B = A + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      v8s fa[MI], fb[NI];
      const int g = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const v8s*>(A + swz(wm * TM + i * 16 + (lane & 15), g));
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[j] = *reinterpret_cast<const v8s*>(B + swz(wn * TN + j * 16 + (lane & 15), g));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    __syncthreads();   // retires the stage-(k+1) DMA (vmcnt(0)) and the stage-k fragment reads
  }
  if constexpr (NST == 1) {   // launched for aligned outputs only (bigdl_conv_nt)
    constexpr int NH = NI >= 4 ? 4 : 2;   // row chunks: fewer live epilogue registers on the wide tile
    constexpr int SL = (TM / NH) * TN;
    nt_epilogue_lds<MI, NI, TM, TN, NH, WM == 2 ? WN * SL : 0>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid,
                                                               reinterpret_cast<float*>(lds) + wave * SL, wm);
  } else if ((a.Ncol & 7) == 0 && (a.ldo & 7) == 0) {
    nt_epilogue_lds<MI, NI, TM, TN, 1, WM == 2 ? WN * TM * TN : 0>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid,
                                                                   reinterpret_cast<float*>(lds) + wave * TM * TN,
                                                                   wm);
  } else {
    nt_epilogue<MI, NI, TM, TN>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid);
  }
}

// ------------------------------------------------------------------------------------------------
// Persistent LDS-DMA NT kernel: a grid of 2 workgroups per CU walks the tiles (tile = blockIdx + k * grid,
// through the same XCD remap, so each XCD keeps its contiguous tile range). When a tile's K loop ends the
// first K-slice of the NEXT tile is DMA'd into stage 0 before the epilogue runs, and the epilogue stages
// its accumulators through stage 1 in two row chunks — so the next tile's load latency hides behind this
// tile's epilogue (stores, statistics atomics). Aimed at the many-tile, short-K layers (1x1 convs over 64-256
// channels: 1-4 K-slices per tile) where load -> MFMA -> epilogue run back to back. Measured on ResNet-50
// b256 it is slower than the one-tile-per-workgroup kernel (33.3 vs 32.4 ms/step): the barrier opening each
// tile waits on vmcnt(0), which now includes the previous epilogue's stores, while a retiring workgroup lets
// its stores drain under the next workgroup's loads. Opt-in (BIGDL_CONV_IMPL=3) until the wait is counted.
// ------------------------------------------------------------------------------------------------
template <int BM, int BN, int WM>
__global__ __launch_bounds__(256, 2) void conv_nt_pers_kernel(ConvArgs a) {
  constexpr int WN = 4 / WM;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int AI = BM / 32, BI = BN / 32;
  constexpr int STAGE = (BM + BN) * BK;
  static_assert(4 * (TM / 2) * TN * 4 <= STAGE * 2, "epilogue chunk must fit one stage");
  __shared__ __attribute__((aligned(1024))) bf16_t lds[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int tiles_n = (a.Ncol + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int rsub = lane >> 3;
  const int gsrc = (lane ^ rsub) & 7;
  const int ohw = a.OH * a.OW;
  const int nk = a.Kdim / BK;

  int a_pix[AI], a_h[AI], a_w[AI];
  const bf16_t* wrow[BI];
  bool bvalid[BI];
  auto setup = [&](int m0, int n0) {
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
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const int n = n0 + (i * 4 + wave) * 8 + rsub;
      bvalid[i] = n < a.Ncol;
      wrow[i] = a.wt + (size_t)(bvalid[i] ? n : 0) * a.ldw + gsrc * 8;
    }
  };
  auto issue = [&](int kt, int buf) {
    const int k0 = kt * BK;
    const int t = k0 / a.Cs;
    const int c = k0 - t * a.Cs + gsrc * 8;
    const int th = a.tap_h[t], tw = a.tap_w[t];
    const int wk = a.tap_k[t] * a.Cs + (k0 - t * a.Cs);
    bf16_t* A = lds + buf * STAGE;
    bf16_t* B = A + BM * BK;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int ch = a_h[i] + th, cw = a_w[i] + tw;
      const bool ok = (unsigned)ch < (unsigned)a.Hs && (unsigned)cw < (unsigned)a.Ws;
      const bf16_t* src = ok ? a.src + (unsigned)((a_pix[i] + ch * a.Ws + cw) * a.Cs + c) : g_zero_granule;
      glds16(src, (LDS_PTR(void))(A + (i * 4 + wave) * 8 * BK));
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const bf16_t* src = bvalid[i] ? wrow[i] + wk : g_zero_granule;
      glds16(src, (LDS_PTR(void))(B + (i * 4 + wave) * 8 * BK));
    }
  };
  auto swz = [](int row, int g) { return row * BK + ((g ^ (row & 7)) << 3); };

  int t = blockIdx.x;
  if (t >= nwg) return;
  int bid = xcd_remap(t, nwg);
  setup((bid / tiles_n) * BM, (bid % tiles_n) * BN);
  issue(0, 0);
  while (true) {
    const int m0 = (bid / tiles_n) * BM, n0 = (bid % tiles_n) * BN;
    v4f acc[MI][NI];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    __syncthreads();   // stage 0 of this tile landed; the previous epilogue is done with stage 1
    for (int kt = 0; kt < nk; ++kt) {
      // the tile's first slice is in stage 0; slice kt lives in stage kt & 1
      const int cur = kt & 1;
      if (kt + 1 < nk) issue(kt + 1, cur ^ 1);
      const bf16_t* A = lds + cur * STAGE;
      const bf16_t* B = A + BM * BK;
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        v8s fa[MI], fb[NI];
        const int g = ks * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const v8s*>(A + swz(wm * TM + i * 16 + (lane & 15), g));
#pragma unroll
        for (int j = 0; j < NI; ++j) fb[j] = *reinterpret_cast<const v8s*>(B + swz(wn * TN + j * 16 + (lane & 15), g));
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
      __syncthreads();
    }
    // next tile's first K-slice into stage 0 while this tile's epilogue runs out of stage 1
    const int tn_next = t + gridDim.x;
    const int bid_cur = bid;
    if (tn_next < nwg) {
      t = tn_next;
      bid = xcd_remap(t, nwg);
      setup((bid / tiles_n) * BM, (bid % tiles_n) * BN);
      issue(0, 0);
    }
    nt_epilogue_lds<MI, NI, TM, TN, 2>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid_cur,
                                       reinterpret_cast<float*>(lds + STAGE) + wave * (TM / 2) * TN);
    if (bid == bid_cur) break;
  }
}

// ------------------------------------------------------------------------------------------------
// Deep-pipelined LDS-DMA NT kernel for large grids: 256 pixels x BN channels per workgroup, 8 waves,
// BK = 64, THREE LDS stages with two K-tiles of DMA in flight across each barrier: the step ends with a
// counted `s_waitcnt vmcnt(L)` (L = DMA instructions of one tile, so only tile k+1 is retired while tile
// k+2 keeps streaming) and a raw s_barrier — never __syncthreads(), whose vmcnt(0) would drain the
// pipeline (cdna_hip_programming.md §5 "Pipelining across barriers"). All LDS — the three stages and the
// tap table — lives in one __shared__ array, and the loop issues no VGPR-destination global load, so the
// compiler has no reason to insert a vmcnt(0) of its own (§5 "Projection GEMM" item 4).
// ------------------------------------------------------------------------------------------------
template <int BN, int WGM, int WGN>
__global__ __launch_bounds__(512, 1) void conv_nt_p3_kernel(ConvArgs a) {
  constexpr int BM = 256;
  constexpr int TM = BM / WGM, TN = BN / WGN;     // per-wave tile (pixels x channels)
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int AI = BM / 64, BI = BN / 64;       // DMA instructions per thread per stage (8 waves x 8 rows)
  constexpr int L = AI + BI;
  constexpr int STAGE = (BM + BN) * BK;
  constexpr int NSTAGE = 3;
  __shared__ __attribute__((aligned(1024))) bf16_t lds[NSTAGE * STAGE + 3 * CONV_MAX_TAPS];
  short* taps = reinterpret_cast<short*>(lds + NSTAGE * STAGE);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int tiles_n = (a.Ncol + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;

  if (tid < a.ntaps) {
    taps[tid] = a.tap_h[tid];
    taps[CONV_MAX_TAPS + tid] = a.tap_w[tid];
    taps[2 * CONV_MAX_TAPS + tid] = a.tap_k[tid];
  }

  const int rsub = lane >> 3;
  const int gsrc = (lane ^ rsub) & 7;
  int a_pix[AI], a_h[AI], a_w[AI];
  const int ohw = a.OH * a.OW;
#pragma unroll
  for (int i = 0; i < AI; ++i) {
    const int m = m0 + (i * 8 + wave) * 8 + rsub;
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
  const bf16_t* wrow[BI];
  bool bvalid[BI];
#pragma unroll
  for (int i = 0; i < BI; ++i) {
    const int n = n0 + (i * 8 + wave) * 8 + rsub;
    bvalid[i] = n < a.Ncol;
    wrow[i] = a.wt + (size_t)(bvalid[i] ? n : 0) * a.ldw + gsrc * 8;
  }
  __syncthreads();   // tap table visible (no DMA outstanding yet)

  auto issue = [&](int kt, int buf) {
    const int k0 = kt * BK;
    const int t = k0 / a.Cs;
    const int cin = k0 - t * a.Cs;
    const int th = taps[t], tw = taps[CONV_MAX_TAPS + t];
    const int wk = taps[2 * CONV_MAX_TAPS + t] * a.Cs + cin;
    const int c = cin + gsrc * 8;
    bf16_t* A = lds + buf * STAGE;
    bf16_t* B = A + BM * BK;
#pragma unroll
    for (int i = 0; i < AI; ++i) {
      const int ch = a_h[i] + th, cw = a_w[i] + tw;
      const bool ok = (unsigned)ch < (unsigned)a.Hs && (unsigned)cw < (unsigned)a.Ws;
      const bf16_t* src = ok ? a.src + (unsigned)((a_pix[i] + ch * a.Ws + cw) * a.Cs + c) : g_zero_granule;
      glds16(src, (LDS_PTR(void))(A + (i * 8 + wave) * 8 * BK));
    }
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const bf16_t* src = bvalid[i] ? wrow[i] + wk : g_zero_granule;
      glds16(src, (LDS_PTR(void))(B + (i * 8 + wave) * 8 * BK));
    }
  };
  auto swz = [](int row, int g) { return row * BK + ((g ^ (row & 7)) << 3); };

  v4f acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  const int nk = a.Kdim / BK;
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
    const bool more2 = kt + 2 < nk;
    if (more2) issue(kt + 2, cur == 0 ? 2 : cur - 1);
    const bf16_t* A = lds + cur * STAGE;
    const bf16_t* B = A + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      v8s fa[MI], fb[NI];
      const int g = ks * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const v8s*>(A + swz(wm * TM + i * 16 + (lane & 15), g));
#pragma unroll
      for (int j = 0; j < NI; ++j) fb[j] = *reinterpret_cast<const v8s*>(B + swz(wn * TN + j * 16 + (lane & 15), g));
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    // retire tile k+1 (tile k+2 stays in flight), then make every wave's reads of this stage and every
    // wave's tile-(k+1) DMA ordered before anything after the barrier
    if (more2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(L) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }
  if ((a.Ncol & 7) == 0 && (a.ldo & 7) == 0)
    nt_epilogue_lds<MI, NI, TM, TN, 1, WGN * TM * TN, WGM>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid,
                                                          reinterpret_cast<float*>(lds) + wave * TM * TN, wm);
  else
    nt_epilogue<MI, NI, TM, TN>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid);
}

// ------------------------------------------------------------------------------------------------
// Weight gradient: dW[n][kk] += sum_m dY[m][n] * im2col(X)[m][kk]   (fp32 out, split-K over m)
// ------------------------------------------------------------------------------------------------

constexpr int WBM = 64;    // pixels (reduction) per LDS stage
constexpr int WT = 128;    // output tile: 128 n x 128 kk

// [WBM][128] bf16 image, 16 granules of 16 B per row, granule g of row r stored at g ^ f(r).
// f is chosen for the ds_read_b64_tr_b16 fragment reads: a 16-lane group reads rows {q} (q = 0..3) x a granule
// pair {g0, g0+1} (g0 even), and its 32-lane partner reads rows {8+q}: f(r) = 2(r&3) | 8((r>>3)&1) | ((r>>2)&1)
// sends those 32 lanes' 8-byte halves to 32 distinct bank pairs (conflict-free); within a row it is a
// permutation, so the 16-byte staging writes stay conflict-free too.
__device__ __forceinline__ int wswz(int row, int col) {
  const int f = ((row & 3) << 1) | (((row >> 3) & 1) << 3) | ((row >> 2) & 1);
  return row * WT + ((((col >> 3) ^ f)) << 3) + (col & 7);
}

__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(WgradArgs a) {
  constexpr int STAGE = 2 * WBM * WT;
  __shared__ __attribute__((aligned(16))) bf16_t lds[2 * STAGE];
  __shared__ float red[256 * 8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wk = wave >> 1, wn = wave & 1;     // wave tile: 64 kk x 64 n
  const int tiles_n = (a.Ncol + WT - 1) / WT, tiles_k = (a.Kdim + WT - 1) / WT;
  const int ntile = tiles_n * tiles_k;
  const int t = xcd_remap(blockIdx.x, ntile);
  const int tk = t / tiles_n, tn = t % tiles_n;
  const int n0 = tn * WT, k0 = tk * WT;
  const int mbeg = blockIdx.y * a.m_per_split;
  const int mend = min(a.M, mbeg + a.m_per_split);
  if (mbeg >= mend) return;

  // loader mapping: row = tid>>4 (+16*i), granule g = tid&15 (8 elements)
  const int lrow = tid >> 4, lg = tid & 15;
  const int nn = n0 + lg * 8;
  const bool nvalid = nn < a.Ncol;
  const int kk = k0 + lg * 8;
  const bool kvalid = kk < a.Kdim;
  const int SC = a.S * a.Cs;
  int r = 0, s = 0, c = 0;
  if (kvalid) { r = kk / SC; int rem = kk - r * SC; s = rem / a.Cs; c = rem - s * a.Cs; }
  const int roff = r * a.dh - a.ph, soff = s * a.dwl - a.pw;

  // Per-stage pixel table, built one stage ahead by wave 0 (one div/mod chain per pixel instead of per
  // loader row): entry = {P = (nb*Hs + oh*sh - ph)*Ws + ow*sw - pw, packed (oh*sh - ph, ow*sw - pw)}.
  __shared__ int2 tbl[2][WBM];
  const int ohw = a.OH * a.OW;
  const int rdh = r * a.dh, sdw = s * a.dwl;
  const int tapoff = rdh * a.Ws + sdw;
  auto build_table = [&](int mb, int slot) {
    if (tid < WBM) {
      const int m = mb + tid;
      int2 e;
      if (m < mend) {
        const int nb = m / ohw, rem = m - nb * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        const int hb = oh * a.sh - a.ph, wb = ow * a.sw - a.pw;
        e.x = (nb * a.Hs + hb) * a.Ws + wb;
        e.y = (hb << 16) | (wb & 0xffff);
      } else {
        e.x = 0;
        e.y = (int)0x80008000;  // hb = wb = -32768: never in range
      }
      tbl[slot][tid] = e;
    }
  };
  v4u rdy[4], rx[4];
  float bsum[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bsum[e] = 0.f;
  const bool do_bias = a.dbias != nullptr && tk == 0;

  auto gload = [&](int mb, int slot) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = lrow + 16 * i;
      const int m = mb + row;
      const int2 e = tbl[slot][row];
      const int ih = (e.y >> 16) + rdh, iw = ((int)(short)(e.y & 0xffff)) + sdw;
      rdy[i] = load16(a.dy + (unsigned)(m * a.ldy + nn), nvalid && m < mend);
      rx[i] = load16(a.src + (unsigned)((e.x + tapoff) * a.Cs + c),
                     kvalid && (unsigned)ih < (unsigned)a.Hs && (unsigned)iw < (unsigned)a.Ws);
    }
  };
  auto swrite = [&](int buf) {
    bf16_t* D = lds + buf * STAGE;
    bf16_t* X = D + WBM * WT;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = lrow + 16 * i;
      *reinterpret_cast<v4u*>(D + wswz(row, lg * 8)) = rdy[i];
      *reinterpret_cast<v4u*>(X + wswz(row, lg * 8)) = rx[i];
      if (do_bias) {
#pragma unroll
        for (int e = 0; e < 4; ++e) { bsum[2 * e] += lo_bf(rdy[i][e]); bsum[2 * e + 1] += hi_bf(rdy[i][e]); }
      }
    }
  };

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // transposed-read lane geometry (ds_read_b64_tr_b16): lane 4q+p of each 16-lane group addresses
  // row q, columns 4p..4p+3 of a 4x16 block; lane i receives column i of the 4 rows.
  const int G = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;

  build_table(mbeg, 0);
  build_table(mbeg + WBM, 1);
  __syncthreads();
  gload(mbeg, 0);
  swrite(0);
  __syncthreads();
  int cur = 0;
  for (int mb = mbeg; mb < mend; mb += WBM) {
    const bool more = mb + WBM < mend;
    if (more) gload(mb + WBM, cur ^ 1);          // table of stage t+1 (built last iteration)
    build_table(mb + 2 * WBM, cur);              // table of stage t+2 into the slot stage t used
    const bf16_t* D = lds + cur * STAGE;
    const bf16_t* X = D + WBM * WT;
#pragma unroll
    for (int ks = 0; ks < WBM / 32; ++ks) {
      v8s fx[4], fd[4];
      const int rbase = ks * 32 + 8 * G + q;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = wk * 64 + i * 16 + 4 * p;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(X + wswz(rbase, col)));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(X + wswz(rbase + 4, col)));
        fx[i] = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + 4 * p;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(D + wswz(rbase, col)));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(D + wswz(rbase + 4, col)));
        fd[j] = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[i], fd[j], acc[i][j], 0, 0, 0);
    }
    if (more) swrite(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // D[kk][n]: lane holds kk = 4*(lane>>4)+e (e=0..3) for n = lane&15
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kb = k0 + wk * 64 + i * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane & 15);
      if (n < a.Ncol) {
        float* o = a.dw + (size_t)n * a.Kdim + kb;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (kb + e < a.Kdim) atomicAdd(o + e, acc[i][j][e]);
      }
    }
  }
  if (do_bias) {
#pragma unroll
    for (int e = 0; e < 8; ++e) red[e * 256 + tid] = bsum[e];
    __syncthreads();
    if (tid < 128) {  // 16 granules x 8 channels; sum over the 16 row-groups
      const int g = tid >> 3, e = tid & 7;
      float tot = 0.f;
      for (int rg = 0; rg < 16; ++rg) tot += red[e * 256 + rg * 16 + g];
      const int n = n0 + g * 8 + e;
      if (n < a.Ncol) atomicAdd(a.dbias + n, tot);
    }
  }
}

// LDS-DMA weight-gradient kernel: same tile / fragment geometry as conv_wgrad_kernel, but the [pixel][channel]
// operand tiles are streamed with global_load_lds (no VGPR staging, no LDS write instructions). A wave's
// DMA instruction fills 4 consecutive rows x 16 granules; lane l writes slot l&15 of row 4j + (l>>4), so the
// wswz row permutation f(row) is fixed per (lane, wave) and applied on the source side: the lane fetches
// granule (l&15) ^ f. For the im2col operand that fixes each lane's (tap, channel) for the whole kernel.
__global__ __launch_bounds__(256, 2) void conv_wgrad_glds_kernel(WgradArgs a) {
  constexpr int STAGE = 2 * WBM * WT;
  __shared__ __attribute__((aligned(1024))) bf16_t lds[2 * STAGE];
  __shared__ int2 tbl[3][WBM];
  __shared__ float red[4][128];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wave >> 1, wn = wave & 1;
  const int tiles_n = (a.Ncol + WT - 1) / WT, tiles_k = (a.Kdim + WT - 1) / WT;
  const int ntile = tiles_n * tiles_k;
  // XCD-aware split-major order: workgroup L runs on XCD L & 7; all tiles of split s live on XCD s & 7 and are
  // dispatched back to back, so the split's dy / x pixel rows come from HBM once per XCD and the other tiles of
  // that split hit the XCD's L2 (tile-major order re-read them from HBM once per tile).
  const int L = blockIdx.x, kq = L >> 3;
  const int split = 8 * (kq / ntile) + (L & 7);
  const int t = kq % ntile;
  const int tk = t / tiles_n, tn = t % tiles_n;
  const int n0 = tn * WT, k0 = tk * WT;
  const int mbeg = split * a.m_per_split;
  const int mend = min(a.M, mbeg + a.m_per_split);
  if (split >= a.splits || mbeg >= mend) return;

  // source granule of this lane (see wswz): rows 16i + 4*wave + (lane>>4)
  const int Lg = lane >> 4;
  const int f = (Lg << 1) | (((wave >> 1) & 1) << 3) | (wave & 1);
  const int gsrc = (lane & 15) ^ f;
  const int nn = n0 + gsrc * 8;
  const bool nvalid = nn < a.Ncol;
  const int kk = k0 + gsrc * 8;
  const bool kvalid = kk < a.Kdim;
  const int SC = a.S * a.Cs;
  int r = 0, s = 0, c = 0;
  if (kvalid) { r = kk / SC; const int rem = kk - r * SC; s = rem / a.Cs; c = rem - s * a.Cs; }
  const int rdh = r * a.dh, sdw = s * a.dwl;
  const int tapoff = rdh * a.Ws + sdw;

  const int ohw = a.OH * a.OW;
  auto build_table = [&](int mb, int slot) {
    if (tid < WBM) {
      const int m = mb + tid;
      int2 e;
      if (m < mend) {
        const int nb = m / ohw, rem = m - nb * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        const int hb = oh * a.sh - a.ph, wb = ow * a.sw - a.pw;
        e.x = (nb * a.Hs + hb) * a.Ws + wb;
        e.y = (hb << 16) | (wb & 0xffff);
      } else {
        e.x = 0;
        e.y = (int)0x80008000;
      }
      tbl[slot][tid] = e;
    }
  };
  auto issue = [&](int mb, int tslot, int buf) {
    bf16_t* D = lds + buf * STAGE;
    bf16_t* X = D + WBM * WT;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rowblk = (i * 4 + wave) * 4;          // first of the 4 rows this instruction fills
      const int row = rowblk + Lg;
      const int m = mb + row;
      const int2 e = tbl[tslot][row];
      const int ih = (e.y >> 16) + rdh, iw = ((int)(short)(e.y & 0xffff)) + sdw;
      // columns past Ncol / Kdim only feed discarded outputs: no DMA at all for those lanes
      const bf16_t* pd = m < mend ? a.dy + (unsigned)(m * a.ldy + nn) : g_zero_granule;
      const bool okx = (unsigned)ih < (unsigned)a.Hs && (unsigned)iw < (unsigned)a.Ws;
      const bf16_t* px = okx ? a.src + (unsigned)((e.x + tapoff) * a.Cs + c) : g_zero_granule;
      if (nvalid) glds16(pd, (LDS_PTR(void))(D + rowblk * WT));
      if (kvalid) glds16(px, (LDS_PTR(void))(X + rowblk * WT));
    }
  };

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = a.dbias != nullptr && tk == 0 && wk == 0;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};

  const int G = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;

  build_table(mbeg, 0);
  build_table(mbeg + WBM, 1);
  __syncthreads();
  issue(mbeg, 0, 0);
  build_table(mbeg + 2 * WBM, 2);
  __syncthreads();
  int cur = 0, ts = 1;
  for (int mb = mbeg; mb < mend; mb += WBM) {
    const bool more = mb + WBM < mend;
    if (more) issue(mb + WBM, ts, cur ^ 1);
    const bf16_t* D = lds + cur * STAGE;
    const bf16_t* X = D + WBM * WT;
#pragma unroll
    for (int ks = 0; ks < WBM / 32; ++ks) {
      v8s fx[4], fd[4];
      const int rbase = ks * 32 + 8 * G + q;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = wk * 64 + i * 16 + 4 * p;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(X + wswz(rbase, col)));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(X + wswz(rbase + 4, col)));
        fx[i] = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + 4 * p;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(D + wswz(rbase, col)));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(D + wswz(rbase + 4, col)));
        fd[j] = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[i], fd[j], acc[i][j], 0, 0, 0);
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (n0 + wn * 64 + j * 16 + (lane & 15) < a.Ncol) {
#pragma unroll
            for (int e = 0; e < 8; ++e) bsum[j] += bf2f((bf16_t)fd[j][e]);
          }
      }
    }
    // table of stage t+3 into the slot stage t used; then retire stage t+1's DMA (vmcnt(0)) before reuse
    build_table(mb + 3 * WBM, (ts + 2) % 3);
    __syncthreads();
    cur ^= 1;
    ts = ts == 2 ? 0 : ts + 1;
  }

  float* part = a.ws ? a.ws + (size_t)split * a.Ncol * a.Kdim : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kb = k0 + wk * 64 + i * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane & 15);
      if (n < a.Ncol) {
        if (part) {   // this split owns its partial tile: plain 16-byte stores (Kdim % 8 == 0)
          if (kb < a.Kdim) *reinterpret_cast<v4f*>(part + (size_t)n * a.Kdim + kb) = acc[i][j];
        } else {
          float* o = a.dw + (size_t)n * a.Kdim + kb;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (kb + e < a.Kdim) atomicAdd(o + e, acc[i][j][e]);
        }
      }
    }
  }
  if (a.dbias != nullptr && tk == 0) {
    // waves wk==0 (wn = 0, 1) hold, per lane, partial sums of column wn*64 + j*16 + (lane&15) over the rows of
    // row-group G; reduce the 4 groups through LDS
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < 4; ++j) red[G][wn * 64 + j * 16 + (lane & 15)] = bsum[j];
    }
    __syncthreads();
    if (tid < 128) {
      const float tot = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
      const int n = n0 + tid;
      if (n < a.Ncol) atomicAdd(a.dbias + n, tot);
    }
  }
}

// Deep-pipelined variant of conv_wgrad_glds_kernel: 32-pixel LDS stages (16 KB: dy and x tiles of 32 x 128), THREE
// stages with two in flight across every barrier (counted `s_waitcnt vmcnt`, raw s_barrier — the 2-stage kernel's
// __syncthreads drains the DMA queue every 64 pixels), 3 workgroups per CU. Every lane issues every DMA (zero granule
// for columns past Ncol / Kdim) so each wave's vmcnt counts L = 4 instructions per stage exactly. The pixel tables
// and the bias reduction live behind the stages in the one __shared__ array.
__global__ __launch_bounds__(256, 3) void conv_wgrad_g3_kernel(WgradArgs a) {
  constexpr int PB = 32;                     // pixels per stage
  constexpr int STAGE = 2 * PB * WT;
  constexpr int NS = 3;
  constexpr int L = 2 * (PB / 16);           // DMA instructions per thread per stage (dy + x)
  __shared__ __attribute__((aligned(1024))) bf16_t lds[NS * STAGE + (3 * PB * 8 + 4 * 128 * 4) / 2];
  int2* tblv = reinterpret_cast<int2*>(lds + NS * STAGE);              // [3][PB]
  float* red = reinterpret_cast<float*>(lds + NS * STAGE + 3 * PB * 4); // [4][128]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wave >> 1, wn = wave & 1;
  const int tiles_n = (a.Ncol + WT - 1) / WT, tiles_k = (a.Kdim + WT - 1) / WT;
  const int ntile = tiles_n * tiles_k;
  const int Lb = blockIdx.x, kq = Lb >> 3;
  const int split = 8 * (kq / ntile) + (Lb & 7);
  const int t = kq % ntile;
  const int tk = t / tiles_n, tn = t % tiles_n;
  const int n0 = tn * WT, k0 = tk * WT;
  const int mbeg = split * a.m_per_split;
  const int mend = min(a.M, mbeg + a.m_per_split);
  if (split >= a.splits || mbeg >= mend) return;

  const int Lg = lane >> 4;
  const int f = (Lg << 1) | (((wave >> 1) & 1) << 3) | (wave & 1);
  const int gsrc = (lane & 15) ^ f;
  const int nn = n0 + gsrc * 8;
  const bool nvalid = nn < a.Ncol;
  const int kk = k0 + gsrc * 8;
  const bool kvalid = kk < a.Kdim;
  const int SC = a.S * a.Cs;
  int r = 0, s = 0, c = 0;
  if (kvalid) { r = kk / SC; const int rem = kk - r * SC; s = rem / a.Cs; c = rem - s * a.Cs; }
  const int rdh = r * a.dh, sdw = s * a.dwl;
  const int tapoff = rdh * a.Ws + sdw;

  const int ohw = a.OH * a.OW;
  auto build_table = [&](int mb, int slot) {
    if (tid < PB) {
      const int m = mb + tid;
      int2 e;
      if (m < mend) {
        const int nb = m / ohw, rem = m - nb * ohw;
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        const int hb = oh * a.sh - a.ph, wb = ow * a.sw - a.pw;
        e.x = (nb * a.Hs + hb) * a.Ws + wb;
        e.y = (hb << 16) | (wb & 0xffff);
      } else {
        e.x = 0;
        e.y = (int)0x80008000;
      }
      tblv[slot * PB + tid] = e;
    }
  };
  auto issue = [&](int mb, int slot, int buf) {
    bf16_t* D = lds + buf * STAGE;
    bf16_t* X = D + PB * WT;
#pragma unroll
    for (int i = 0; i < PB / 16; ++i) {
      const int rowblk = (i * 4 + wave) * 4;
      const int row = rowblk + Lg;
      const int m = mb + row;
      const int2 e = tblv[slot * PB + row];
      const int ih = (e.y >> 16) + rdh, iw = ((int)(short)(e.y & 0xffff)) + sdw;
      const bf16_t* pd = (nvalid && m < mend) ? a.dy + (unsigned)(m * a.ldy + nn) : g_zero_granule;
      const bool okx = kvalid && (unsigned)ih < (unsigned)a.Hs && (unsigned)iw < (unsigned)a.Ws;
      const bf16_t* px = okx ? a.src + (unsigned)((e.x + tapoff) * a.Cs + c) : g_zero_granule;
      glds16(pd, (LDS_PTR(void))(D + rowblk * WT));
      glds16(px, (LDS_PTR(void))(X + rowblk * WT));
    }
  };

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = a.dbias != nullptr && tk == 0 && wk == 0;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};
  const int G = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int nst = (mend - mbeg + PB - 1) / PB;

  build_table(mbeg, 0);
  build_table(mbeg + PB, 1);
  build_table(mbeg + 2 * PB, 2);
  __syncthreads();                        // tables visible, no DMA outstanding yet
  issue(mbeg, 0, 0);
  if (nst > 1) {
    issue(mbeg + PB, 1, 1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  int cur = 0;
  for (int st = 0; st < nst; ++st) {
    const int mb = mbeg + st * PB;
    const bool more2 = st + 2 < nst;
    // stage st + 2 goes into the buffer and table slot that stage st - 1 used (retired before the last barrier)
    if (more2) issue(mb + 2 * PB, cur == 0 ? 2 : cur - 1, cur == 0 ? 2 : cur - 1);
    const bf16_t* D = lds + cur * STAGE;
    const bf16_t* X = D + PB * WT;
    {
      v8s fx[4], fd[4];
      const int rbase = 8 * G + q;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int col = wk * 64 + i * 16 + 4 * p;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(X + wswz(rbase, col)));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(X + wswz(rbase + 4, col)));
        fx[i] = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int col = wn * 64 + j * 16 + 4 * p;
        v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(D + wswz(rbase, col)));
        v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(D + wswz(rbase + 4, col)));
        fd[j] = v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[i], fd[j], acc[i][j], 0, 0, 0);
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (n0 + wn * 64 + j * 16 + (lane & 15) < a.Ncol) {
#pragma unroll
            for (int e = 0; e < 8; ++e) bsum[j] += bf2f((bf16_t)fd[j][e]);
          }
      }
    }
    // the table of stage st + 3 replaces stage st's (issued two steps ago); retire stage st + 1's DMA
    build_table(mb + 3 * PB, cur);
    if (more2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(L) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == 2 ? 0 : cur + 1;
  }

  float* part = a.ws ? a.ws + (size_t)split * a.Ncol * a.Kdim : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kb = k0 + wk * 64 + i * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane & 15);
      if (n < a.Ncol) {
        if (part) {
          if (kb < a.Kdim) *reinterpret_cast<v4f*>(part + (size_t)n * a.Kdim + kb) = acc[i][j];
        } else {
          float* o = a.dw + (size_t)n * a.Kdim + kb;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (kb + e < a.Kdim) atomicAdd(o + e, acc[i][j][e]);
        }
      }
    }
  }
  if (a.dbias != nullptr && tk == 0) {
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < 4; ++j) red[G * 128 + wn * 64 + j * 16 + (lane & 15)] = bsum[j];
    }
    __syncthreads();
    if (tid < 128) {
      const float tot = red[tid] + red[128 + tid] + red[256 + tid] + red[384 + tid];
      const int n = n0 + tid;
      if (n < a.Ncol) atomicAdd(a.dbias + n, tot);
    }
  }
}

// dw += sum over splits of the workspace partials. Split group g (blockIdx.y) sums splits g, g+G, ... with two
// independent accumulators; with G > 1 the groups meet in dw through fp32 atomics (G-way contention at most), so
// tiny weights (64x64 with ~1000 splits) still spread the reduction over the whole chip.
template <bool ALIGNED>
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw,
                                                           long n4, int splits) {
  const int g = blockIdx.y, G = gridDim.y;
  const v4f* w4 = reinterpret_cast<const v4f*>(ws);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    v4f s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
    int sp = g;
    for (; sp + G < splits; sp += 2 * G) {
      s0 += w4[(long)sp * n4 + i];
      s1 += w4[(long)(sp + G) * n4 + i];
    }
    if (sp < splits) s0 += w4[(long)sp * n4 + i];
    s0 += s1;
    if (G > 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) unsafeAtomicAdd(dw + 4 * i + e, s0[e]);
    } else if (ALIGNED) {
      reinterpret_cast<v4f*>(dw)[i] += s0;
    } else {   // dw is a view into the flat gradient buffer at a 4-byte-aligned offset
#pragma unroll
      for (int e = 0; e < 4; ++e) dw[4 * i + e] += s0[e];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Weight gradient on the phase-interleaved 256 x 256 tile of conv_nt_p8_kernel: dW[n][kk] = sum_p dy[p][n] x[p][kk]
// (kk = (r, s, c) of KRSC, x gathered im2col-style), reduction over output pixels p in K-steps of 64, split over
// pixel ranges per blockIdx.y (fp32 partials [split][Ncol][Kdim] summed by wgrad_reduce_kernel; one split adds into
// dw directly; the bias gradient goes out as fp32 atomics, one per column and split). 8 waves = 2 kk-halves x 4
// n-quarters, 128 kk x 64 n per wave, MFMA A = x fragment (rows kk), B = dy fragment (columns n), so a lane ends up
// with 4 consecutive kk of one n: 16-byte stores along dw's rows.
// LDS: per K-step four 16 KB pieces of 64 pixel rows x 128 columns (256 B rows): P0 / P2 = x columns of
// kk-quadrant 0 / 1 of both kk-halves, P1 / P3 = dy columns of n-quadrant 0 / 1 of the four n-quarters. The
// fragments are read down the pixel rows with the transposing ds_read_b64_tr_b16 (T10); 16-byte chunk k of row r
// sits at slot k ^ f(r), f(r) = 2 * ((r & 3) | ((r >> 3) & 1) << 2), which keeps every 32-lane transposed read
// conflict-free; the DMA applies f on the source side (constant per lane and wave, so each lane's tap / channel /
// output channel is fixed for the whole kernel). Phases, pieces, waits and the wave-group stagger are exactly those
// of conv_nt_p8_kernel (see there for the hazard argument).
__device__ __forceinline__ int p8w_f(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }
typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

// DIRECT: 1 x 1, stride 1, no padding (GEMM-shaped): x row = output pixel, no per-row geometry in the DMA issue
// (the general path divides every DMA row's pixel index into (image, oh, ow): ~9 VALU instructions per MFMA)
template <bool DIRECT>
__global__ __launch_bounds__(512, 2) void conv_wgrad_p8_kernel(WgradArgs a) {
  constexpr int PIX = 64;                          // pixels per K-step
  constexpr int PC = 128;                          // columns per piece
  constexpr int PIECE = PIX * PC;                  // 16 KB
  constexpr int BUF = 4 * PIECE;
  __shared__ __attribute__((aligned(1024))) bf16_t lds[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;         // wave tile: kk rows wm * 128 .., n columns wn * 64 ..
  const int tiles_n = (a.Ncol + 255) / 256, tiles_k = (a.Kdim + 255) / 256;
  const int ntile = tiles_n * tiles_k;
  const int t = xcd_remap(blockIdx.x, ntile);
  const int tk = t / tiles_n, tn = t % tiles_n;
  const int n0 = tn * 256, k0 = tk * 256;
  const int mbeg = blockIdx.y * a.m_per_split;
  const int mend = min(a.M, mbeg + a.m_per_split);
  const int nk = mend > mbeg ? (mend - mbeg + PIX - 1) / PIX : 0;

  // DMA geometry: instruction j of wave w fills piece rows (j * 8 + w) * 4 .. +4 (4 rows x 256 B); lane -> row
  // + (lane >> 4), slot lane & 15, which holds chunk (lane & 15) ^ f(row), f constant per lane and wave
  const int fr = p8w_f((lane >> 4) | (((wave >> 1) & 1) << 3));
  const int chunk = (lane & 15) ^ fr;              // this lane's source chunk (8 columns) of every piece
  // A pieces (x): tile column kk of piece column pc = chunk * 8 is (pc >> 6) * 128 + q * 64 + (pc & 63)
  int xr[2], xs[2], xc[2];
  bool xv[2];
  const int SC = a.S * a.Cs;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int pc = chunk * 8;
    const int kk = k0 + (pc >> 6) * 128 + q * 64 + (pc & 63);
    xv[q] = kk < a.Kdim;
    const int k = xv[q] ? kk : 0;
    xr[q] = k / SC;
    const int rem = k - xr[q] * SC;
    xs[q] = rem / a.Cs;
    xc[q] = rem - xs[q] * a.Cs;
  }
  // B pieces (dy): tile column n of piece column pc is (pc >> 5) * 64 + q * 32 + (pc & 31)
  int dn[2];
  bool dv[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int pc = chunk * 8;
    dn[q] = n0 + (pc >> 5) * 64 + q * 32 + (pc & 31);
    dv[q] = dn[q] < a.Ncol;
  }
  const int ohw = a.OH * a.OW;

  // piece P (0 x q0, 1 dy q0, 2 x q1, 3 dy q1) of K-step kt into buffer buf: 2 DMA instructions per thread
  auto issue = [&](int kt, int buf, int P) {
    bf16_t* base = lds + buf * BUF + P * PIECE;
    const int q = P >> 1;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = (j * 8 + wave) * 4 + (lane >> 4);
      const int m = mbeg + kt * PIX + row;
      const bf16_t* src = g_zero_granule;
      if (m < mend) {
        if ((P & 1) == 0) {
          if (DIRECT) {
            if (xv[q]) src = a.src + (size_t)m * a.Cs + xc[q];
          } else if (xv[q]) {
            const int nb = m / ohw, rem = m - nb * ohw;
            const int oh = rem / a.OW, ow = rem - oh * a.OW;
            const int ih = oh * a.sh - a.ph + xr[q] * a.dh, iw = ow * a.sw - a.pw + xs[q] * a.dwl;
            if ((unsigned)ih < (unsigned)a.Hs && (unsigned)iw < (unsigned)a.Ws)
              src = a.src + (unsigned)(((nb * a.Hs + ih) * a.Ws + iw) * a.Cs + xc[q]);
          }
        } else if (dv[q]) {
          src = a.dy + (unsigned)(m * a.ldy + dn[q]);
        }
      }
      glds16(src, (LDS_PTR(void))(base + (j * 8 + wave) * 4 * PC));
    }
  };
  // transposed fragment reads: lane 4q'+p of 16-lane group g supplies row 32 kh + 8 g + q' (+4), columns c0 + 4p
  const int G = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
  auto tr = [&](const bf16_t* P, int row, int col) -> v4s {
    const int off = row * PC + (((col >> 3) ^ p8w_f(row)) << 3) + (col & 7);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_PTR(v4s))(P + off));
  };
  auto frag = [&](const bf16_t* P, int kh, int c0) -> v8s {
    const int r = 32 * kh + 8 * G + qq;
    const v4s lo = tr(P, r, c0 + 4 * pp), hi = tr(P, r + 4, c0 + 4 * pp);
    return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };

  v4f acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  v8s fa[4][2], fb[4][2];
  auto quad = [&](int ib, int jb) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ib + i][jb + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][kh], fb[jb + j][kh], acc[ib + i][jb + j], 0, 0, 0);
  };
  auto read_a = [&](const bf16_t* P) {            // x: this wave's kk quadrant = piece columns wm * 64 + 16 i
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i][0] = frag(P, 0, wm * 64 + i * 16);
      fa[i][1] = frag(P, 1, wm * 64 + i * 16);
    }
  };
  auto read_b = [&](const bf16_t* P, int jb) {    // dy: this wave's n quadrant = piece columns wn * 32 + 16 j
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fb[jb + j][0] = frag(P, 0, wn * 32 + j * 16);
      fb[jb + j][1] = frag(P, 1, wn * 32 + j * 16);
    }
  };
  // bias gradient: the kk-tile-0 workgroups also sum their dy fragments over the pixels, wave half wm taking the
  // n columns of fb[2 wm], fb[2 wm + 1] (v_dot2 against ones: 4 VALU per fragment beside 16 MFMA)
  const bool do_bias = a.dbias != nullptr && tk == 0;
  float bsum[2] = {0.f, 0.f};
  auto bias = [&](int jb) {
    const v2bf one = {(__bf16)1.0f, (__bf16)1.0f};
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const v8bf f = __builtin_bit_cast(v8bf, fb[jb + j][kh]);
#pragma unroll
        for (int e = 0; e < 4; ++e) bsum[j] = __builtin_amdgcn_fdot2_f32_bf16(v2bf{f[2 * e], f[2 * e + 1]}, one, bsum[j], false);
      }
  };
  auto compute = [&](int ib, int jb, bool sum_bias) {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    quad(ib, jb);
    if (sum_bias) bias(jb);
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
  if (wm == 1) __builtin_amdgcn_s_barrier();     // stagger

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bf16_t* L = lds + cur * BUF;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    if (n1) issue(kt + 1, cur ^ 1, 3);
    read_a(L); read_b(L + PIECE, 0);
    if (n1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    compute(0, 0, do_bias && wm == 0);
    if (n1) issue(kt + 1, cur ^ 1, 2);
    read_b(L + 3 * PIECE, 2);
    if (n1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    compute(0, 2, do_bias && wm == 1);
    if (n2) issue(kt + 2, cur, 0);
    read_a(L + 2 * PIECE);
    compute(4, 2, false);
    if (n2) issue(kt + 2, cur, 1);
    if (n2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    compute(4, 0, false);
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();     // balance the stagger
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // acc[i][j] = D[kk][n]: kk = k0 + wm * 128 + 16 i + 4 (lane >> 4) + e (quadrant rows: i < 4 -> q0, else q1),
  // n = n0 + wn * 64 + 16 j + (lane & 15)
  if (do_bias) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float v = bsum[j];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int n = n0 + wn * 64 + (2 * wm + j) * 16 + lane;
      if (lane < 16 && n < a.Ncol) unsafeAtomicAdd(a.dbias + n, v);
    }
  }
  float* part = a.splits > 1 ? a.ws + (size_t)blockIdx.y * a.Ncol * a.Kdim : nullptr;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int kb = k0 + wm * 128 + i * 16 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + (lane & 15);
      if (n < a.Ncol && kb < a.Kdim) {
        if (part) {
          *reinterpret_cast<v4f*>(part + (size_t)n * a.Kdim + kb) = acc[i][j];
        } else {
          float* o = a.dw + (size_t)n * a.Kdim + kb;   // a view into the flat gradient: maybe only 4-byte aligned
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] += acc[i][j][e];
        }
      }
    }
  }
}

// wt[c][rs][k] = w[k][rs][c]: per tap, a [K][C] -> [C][K] transpose through a 32 x 32 LDS tile (coalesced
// reads along c and writes along k, +1 column pad against bank conflicts). Small tiles keep >= 4 workgroups on
// the 64 x 64 layers: most of the 53 per-step launches are latency-, not bandwidth-bound.
__global__ __launch_bounds__(256) void transpose_krsc_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt,
                                                             int K, int RS, int C) {
  __shared__ bf16_t tile[32][33];
  const int c0 = blockIdx.x * 32, k0 = blockIdx.y * 32, rs = blockIdx.z;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  bf16_t v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + ty + 8 * i, c = c0 + tx;
    v[i] = (k < K && c < C) ? w[((size_t)k * RS + rs) * C + c] : (bf16_t)0;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) tile[ty + 8 * i][tx] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = c0 + ty + 8 * i, k = k0 + tx;
    if (c < C && k < K) wt[((size_t)c * RS + rs) * K + k] = tile[tx][ty + 8 * i];
  }
}

// 16-byte form for K % 8 == 0 and C % 8 == 0 (every activation transpose of the GEMM weight-gradient path): 64 x 64
// tile, each thread loads two 8-element granules along C and stores two packed granules along K, so global traffic is
// full 16-byte accesses both ways (the 2-byte 32 x 32 kernel above moved [32768 x 10000] at ~3.4 TB/s).
__global__ __launch_bounds__(256) void transpose_krsc_v8_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wt,
                                                                int K, int RS, int C) {
  __shared__ bf16_t tile[64][64 + 2];
  const int c0 = blockIdx.x * 64, k0 = blockIdx.y * 64, rs = blockIdx.z;
  const int t = threadIdx.x, g = t & 7, rr = t >> 3;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int kl = rr + 32 * h, k = k0 + kl, c = c0 + g * 8;
    v4u q = v4u{0u, 0u, 0u, 0u};
    if (k < K && c < C) q = *reinterpret_cast<const v4u*>(w + ((size_t)k * RS + rs) * C + c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      tile[kl][g * 8 + 2 * e] = (bf16_t)(q[e] & 0xffffu);
      tile[kl][g * 8 + 2 * e + 1] = (bf16_t)(q[e] >> 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int cl = rr + 32 * h, c = c0 + cl, k = k0 + g * 8;
    if (c < C && k < K) {
      v4u q;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        q[e] = (unsigned)tile[g * 8 + 2 * e][cl] | ((unsigned)tile[g * 8 + 2 * e + 1][cl] << 16);
      *reinterpret_cast<v4u*>(wt + ((size_t)c * RS + rs) * K + k) = q;
    }
  }
}

// All conv weights of a model transposed for the data-gradient GEMMs in ONE launch (once per training step, after
// the optimizer has rewritten the bf16 weights) instead of one small launch per layer. desc[i] = {w, wt, K, RS, C,
// first tile}: workgroup b handles 32 x 32 tile (b - first tile) of the last layer whose first tile is <= b.
__global__ __launch_bounds__(256) void transpose_krsc_batched_kernel(const long* __restrict__ desc, int n) {
  __shared__ bf16_t tile[32][33];
  __shared__ int li;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) {
    int i = 0;
    while (i + 1 < n && desc[(i + 1) * 6 + 5] <= b) ++i;
    li = i;
  }
  __syncthreads();
  const long* d = desc + li * 6;
  const bf16_t* w = reinterpret_cast<const bf16_t*>(d[0]);
  bf16_t* wt = reinterpret_cast<bf16_t*>(d[1]);
  const int K = (int)d[2], RS = (int)d[3], C = (int)d[4];
  int t = b - (int)d[5];
  const int tc = (C + 31) / 32, tk = (K + 31) / 32;
  const int c0 = (t % tc) * 32;
  t /= tc;
  const int k0 = (t % tk) * 32, rs = t / tk;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  bf16_t v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = k0 + ty + 8 * i, c = c0 + tx;
    v[i] = (k < K && c < C) ? w[((size_t)k * RS + rs) * C + c] : (bf16_t)0;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) tile[ty + 8 * i][tx] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = c0 + ty + 8 * i, k = k0 + tx;
    if (c < C && k < K) wt[((size_t)c * RS + rs) * K + k] = tile[tx][ty + 8 * i];
  }
}

// ------------------------------------------------------------------------------------------------
// 256 x 256 implicit-GEMM NT tile for the compute-heavy layers (N >= 256): 8 waves as 2 (pixels) x 4 (channels),
// wave tile 128 x 64 (32 accumulators), BK = 32 per K-step and FOUR LDS-DMA stages of 32 KB: three K-steps stay in
// flight across every barrier (counted `s_waitcnt vmcnt`, raw s_barrier: never the vmcnt(0) of __syncthreads,
// cdna_hip_programming.md §5 "Pipelining across barriers"). Twice the FLOP per staged byte of the 128 x 128 tile
// (128 vs 64), which is what the per-CU LDS-DMA rate bounds on these layers (≈36 GB/s per CU measured on the
// 256 x 128 kernel). 64-byte LDS rows; the 16-byte granule g of row r sits in slot g ^ ((r >> 1) & 3): the
// ds_read_b128 fragment reads (16 rows x 4 granules per 16-lane group) then hit 16 distinct bank quads. All LDS is
// one __shared__ array (a second object can make hipcc drain vmcnt before the first ds_read).
// SPLIT: blockIdx.y is a K split of ksteps_per_split K-steps; the accumulators go to fp32 partials
// ws[split][M][Ncol] and conv_splitk_epilogue_kernel applies the fused epilogue after summing them.
// ------------------------------------------------------------------------------------------------
template <int MI, int NI, int TM, int TN, int NH>
__device__ __forceinline__ void store_partials_lds(float* __restrict__ ws, int M, int Ncol, v4f (&acc)[MI][NI],
                                                   int mbase, int nbase, int lane, float* wl) {
  constexpr int GR = TN / 4, LPR = TN / 8, PPI = 64 / LPR, NR = TM / PPI, MIH = MI / NH, NRH = NR / NH;
  auto gpos = [](int p, int g) { return (p * GR + (g ^ (p & (GR - 1)))) * 4; };
  const int q = lane % LPR;
  const int n = nbase + q * 8;
#pragma unroll
  for (int h = 0; h < NH; ++h) {
#pragma unroll
    for (int i = 0; i < MIH; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        *reinterpret_cast<v4f*>(wl + gpos(i * 16 + (lane & 15), j * 4 + (lane >> 4))) = acc[h * MIH + i][j];
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): wave-private slice
#pragma unroll
    for (int rr = 0; rr < NRH; ++rr) {
      const int p = rr * PPI + lane / LPR;
      const int m = mbase + h * (TM / NH) + p;
      const v4f lo = *reinterpret_cast<const v4f*>(wl + gpos(p, 2 * q));
      const v4f hi = *reinterpret_cast<const v4f*>(wl + gpos(p, 2 * q + 1));
      if (m < M && n < Ncol) {
        float* o = ws + (size_t)m * Ncol + n;
        *reinterpret_cast<v4f*>(o) = lo;
        *reinterpret_cast<v4f*>(o + 4) = hi;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // the slice is rewritten by the next chunk
  }
}

template <bool SPLIT>
__global__ __launch_bounds__(512, 1) void conv_nt_w8_kernel(ConvArgs a) {
  constexpr int BM = 256, BN = 256, BKS = 32, NS = 4;
  constexpr int WGM = 2, WGN = 4;
  constexpr int TM = BM / WGM, TN = BN / WGN;      // 128 x 64 per wave
  constexpr int MI = TM / 16, NI = TN / 16;        // 8 x 4 MFMA tiles
  constexpr int STAGE = (BM + BN) * BKS;           // 16384 bf16 = 32 KB
  constexpr int L = 4;                             // DMA instructions per thread per stage (2 A + 2 B)
  constexpr int NH = SPLIT ? 2 : 4;                 // epilogue row chunks (4: fewer live prefetch registers)
  constexpr int SL = (TM / NH) * TN;
  static_assert(8 * SL * 4 <= NS * STAGE * 2, "epilogue chunk must fit the stages");
  // the tap table lives behind the stages: indexing the kernarg copy with a run-time tap makes hipcc emit VECTOR
  // loads of it and a vmcnt(0) before their use, which would drain the DMA pipeline every K-step
  __shared__ __attribute__((aligned(1024))) bf16_t lds[NS * STAGE + 3 * CONV_MAX_TAPS];
  short* taps = reinterpret_cast<short*>(lds + NS * STAGE);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int tiles_n = (a.Ncol + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk_all = a.Kdim / BKS;
  int kt0 = 0, nk = nk_all;
  if constexpr (SPLIT) {
    const int per = (nk_all + a.ksplit - 1) / a.ksplit;
    kt0 = blockIdx.y * per;
    nk = min(nk_all, kt0 + per) - kt0;
  }

  // DMA geometry: instruction j of wave w fills rows (j * 8 + w) * 16 .. +16 (64 B each, 4 granules); lane -> row
  // + (lane >> 2), slot lane & 3, which must hold granule (lane & 3) ^ ((row >> 1) & 3)
  const int rsub = lane >> 2;
  const int gsrc = (lane & 3) ^ ((rsub >> 1) & 3);
  int a_pix[2], a_h[2], a_w[2];
  const int ohw = a.OH * a.OW;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = m0 + (j * 8 + wave) * 16 + rsub;
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
  const bf16_t* wrow[2];
  bool bvalid[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + (j * 8 + wave) * 16 + rsub;
    bvalid[j] = n < a.Ncol;
    wrow[j] = a.wt + (size_t)(bvalid[j] ? n : 0) * a.ldw + gsrc * 8;
  }
  if (tid < a.ntaps) {
    taps[tid] = a.tap_h[tid];
    taps[CONV_MAX_TAPS + tid] = a.tap_w[tid];
    taps[2 * CONV_MAX_TAPS + tid] = a.tap_k[tid];
  }
  __syncthreads();   // tap table visible (no DMA outstanding yet)

  auto issue = [&](int kt, int buf) {
    const int k0 = kt * BKS;
    const int t = k0 / a.Cs;
    const int cin = k0 - t * a.Cs;
    const int th = taps[t], tw = taps[CONV_MAX_TAPS + t];
    const int wk = taps[2 * CONV_MAX_TAPS + t] * a.Cs + cin;
    const int c = cin + gsrc * 8;
    bf16_t* A = lds + buf * STAGE;
    bf16_t* B = A + BM * BKS;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ch = a_h[j] + th, cw = a_w[j] + tw;
      const bool ok = (unsigned)ch < (unsigned)a.Hs && (unsigned)cw < (unsigned)a.Ws;
      const bf16_t* src = ok ? a.src + (unsigned)((a_pix[j] + ch * a.Ws + cw) * a.Cs + c) : g_zero_granule;
      glds16(src, (LDS_PTR(void))(A + (j * 8 + wave) * 16 * BKS));
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bf16_t* src = bvalid[j] ? wrow[j] + wk : g_zero_granule;
      glds16(src, (LDS_PTR(void))(B + (j * 8 + wave) * 16 * BKS));
    }
  };
  // fragment of rows row0 .. row0 + 15: lane reads row row0 + (lane & 15), K granule lane >> 4
  const int foff = (lane & 15) * BKS + ((((lane >> 4) ^ ((lane >> 1) & 3))) << 3);

  v4f acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // prologue: K-steps 0, 1, 2 in flight; retire step 0
  if (nk > 0) issue(kt0, 0);
  if (nk > 1) issue(kt0 + 1, 1);
  if (nk > 2) issue(kt0 + 2, 2);
  if (nk > 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * L) : "memory");
  else if (nk > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 3;
    // stage (kt + 3) & 3 == (kt - 1) & 3 was last read in step kt - 1, before the barrier that ended it
    if (kt + 3 < nk) issue(kt0 + kt + 3, (kt + 3) & 3);
    const bf16_t* A = lds + cur * STAGE;
    const bf16_t* B = A + BM * BKS;
    v8s fa[MI], fb[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) fb[j] = *reinterpret_cast<const v8s*>(B + (wn * TN + j * 16) * BKS + foff);
#pragma unroll
    for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const v8s*>(A + (wm * TM + i * 16) * BKS + foff);
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    // retire step kt + 1 (steps kt + 2, kt + 3 stay in flight), make every wave's reads of this stage and every
    // wave's step-(kt + 1) DMA ordered before anything after the barrier
    const int ahead = min(nk - 1, kt + 3) - (kt + 1);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * L) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(L) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  float* wl = reinterpret_cast<float*>(lds) + wave * SL;
  if constexpr (SPLIT) {
    store_partials_lds<MI, NI, TM, TN, NH>(a.ws + (size_t)blockIdx.y * a.M * a.Ncol, a.M, a.Ncol, acc,
                                           m0 + wm * TM, n0 + wn * TN, lane, wl);
  } else {
    nt_epilogue_lds<MI, NI, TM, TN, NH, WGN * SL, WGM>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid, wl, wm);
  }
}

// ------------------------------------------------------------------------------------------------
// 128 x BN (BN = 128 / 64) implicit-GEMM NT tile, 4 waves as 2 x 2, BK = 32 per K-step and NS (3 or 4) LDS-DMA stages
// of (128 + BN) x 64 B: NS - 1 K-steps stay in flight across every barrier (counted `s_waitcnt vmcnt`, raw s_barrier,
// never the vmcnt(0) of __syncthreads — cdna_hip_programming.md §5 "Pipelining across barriers"). The pipeline of
// conv_nt_w8_kernel at the 128 x 128 tile of conv_nt_glds_kernel: 16 KB stages, so NS = 4 leaves room for two
// workgroups per CU (NS = 3: three) and one workgroup's epilogue overlaps the others' main loops, while the
// 2-stage glds kernel drains its DMA queue at every K-step barrier. Same 64-byte-row LDS image, source-side swizzle
// g ^ ((r >> 1) & 3), tap table behind the stages.
// ------------------------------------------------------------------------------------------------
// FASTK = false (Cs % 32 != 0, e.g. Inception's 48 / 80 / 160-channel inputs, padded to 8): a K-step spans taps, so
// every lane resolves the tap of its own 8-channel granule (kk = k0 + 8 * gsrc) from the LDS tap table and the K
// tail past Kdim loads zeros.
// BM = 256 (BIGDL_CONV_G4=6/7): 2 x 2 waves of 128 x 64, 32 MFMAs per wave between barriers instead of 16, 24 KB
// stages, 2 workgroups per CU.
// ABN = 1: timing ablation (BIGDL_G4_ABN=1 with ConvArgs::pre set; padding taps are not masked, so only 1x1 outputs
// are right) — the BN scale / shift + ReLU applied to every A fragment after its LDS read, coefficients loaded per
// K-step (what folding a BN apply into this tile's operand costs; round 4: +1.15 ms on the forward convs).
template <int BN, int NS, bool FASTK = true, int BM = 128, int ABN = 0>
// NS = 2 (short-K variant, BIGDL_CONV_SHORTK): Kdim <= 64, both K-steps issued up front, 32 KB of stages and four
// workgroups per CU for these one-DMA-round, epilogue-heavy tiles (the caller guarantees nk <= 2).
__global__ __launch_bounds__(256, NS == 2 ? 4 : ((NS == 3 && BM == 128) ? 3 : 2)) void conv_nt_g4_kernel(ConvArgs a) {
  constexpr int BKS = 32;
  constexpr bool SHORTK = NS == 2;
  constexpr int WGM = 2, WGN = 2;
  constexpr int TM = BM / WGM, TN = BN / WGN;      // 64 x 64 (or 64 x 32) per wave
  constexpr int MI = TM / 16, NI = TN / 16;
  constexpr int STAGE = (BM + BN) * BKS;
  constexpr int AI = BM / 64, BI = BN / 64;        // DMA instructions per thread per stage (4 waves x 16 rows)
  constexpr int L = AI + BI;
  // epilogue row chunks that fit the stages (4 at BM = 256: fewer prefetched epilogue rows in flight, no spills)
  constexpr int NH = BM == 256 ? 4 : (4 * TM * TN * 4 <= NS * STAGE * 2) ? 1 : 2;
  constexpr int SL = (TM / NH) * TN;
  static_assert(4 * SL * 4 <= NS * STAGE * 2, "epilogue chunk must fit the stages");
  __shared__ __attribute__((aligned(1024))) bf16_t lds[NS * STAGE + 3 * CONV_MAX_TAPS];
  short* taps = reinterpret_cast<short*>(lds + NS * STAGE);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int tiles_n = (a.Ncol + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nk = (a.Kdim + BKS - 1) / BKS;

  // DMA geometry: instruction j of wave w fills rows (j * 4 + w) * 16 .. +16 (64 B each); lane -> row + (lane >> 2),
  // slot lane & 3, which holds granule (lane & 3) ^ ((row >> 1) & 3)
  const int rsub = lane >> 2;
  const int gsrc = (lane & 3) ^ ((rsub >> 1) & 3);
  const int ps = a.pstride > 0 ? a.pstride : a.Cs;   // source pixel stride (ConvArgs::pstride)
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
  const bf16_t* wrow[BI];
  bool bvalid[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int n = n0 + (j * 4 + wave) * 16 + rsub;
    bvalid[j] = n < a.Ncol;
    wrow[j] = a.wt + (size_t)(bvalid[j] ? n : 0) * a.ldw + (FASTK ? gsrc * 8 : 0);
  }
  if (tid < a.ntaps) {
    taps[tid] = a.tap_h[tid];
    taps[CONV_MAX_TAPS + tid] = a.tap_w[tid];
    taps[2 * CONV_MAX_TAPS + tid] = a.tap_k[tid];
  }
  __syncthreads();   // tap table visible (no DMA outstanding yet)

  auto issue = [&](int kt, int buf) {
    const int k0 = kt * BKS;
    int th, tw, wk, c;
    bool kv = true;
    if constexpr (FASTK) {                  // the whole K-step lies in one tap
      const int t = k0 / a.Cs;
      const int cin = k0 - t * a.Cs;
      th = taps[t]; tw = taps[CONV_MAX_TAPS + t];
      wk = taps[2 * CONV_MAX_TAPS + t] * a.Cs + cin;
      c = cin + gsrc * 8;
    } else {                                // per-lane tap of granule kk
      const int kk = k0 + gsrc * 8;
      kv = kk < a.Kdim;
      const int kc = kv ? kk : 0;
      const int t = kc / a.Cs;
      c = kc - t * a.Cs;
      th = taps[t]; tw = taps[CONV_MAX_TAPS + t];
      wk = taps[2 * CONV_MAX_TAPS + t] * a.Cs + c;
    }
    bf16_t* A = lds + buf * STAGE;
    bf16_t* B = A + BM * BKS;
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int ch = a_h[j] + th, cw = a_w[j] + tw;
      const bool ok = kv && (unsigned)ch < (unsigned)a.Hs && (unsigned)cw < (unsigned)a.Ws;
      const bf16_t* src = ok ? a.src + (unsigned)((a_pix[j] + ch * a.Ws + cw) * ps + c) : g_zero_granule;
      glds16(src, (LDS_PTR(void))(A + (j * 4 + wave) * 16 * BKS));
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const bf16_t* src = (bvalid[j] && kv) ? wrow[j] + wk : g_zero_granule;
      glds16(src, (LDS_PTR(void))(B + (j * 4 + wave) * 16 * BKS));
    }
  };
  const int foff = (lane & 15) * BKS + ((((lane >> 4) ^ ((lane >> 1) & 3))) << 3);

  v4f acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  // prologue: K-steps 0 .. NS - 2 in flight; retire step 0
#pragma unroll
  for (int k = 0; k < (SHORTK ? 2 : NS - 1); ++k)
    if (k < nk) issue(k, k);
  {
    const int ahead = min(nk - 1, SHORTK ? 1 : NS - 2);     // steps in flight behind step 0
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * L) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // stage (kt + NS - 1) % NS == (kt - 1) % NS was last read in step kt - 1, before the barrier that ended it
    if (!SHORTK && kt + NS - 1 < nk) issue(kt + NS - 1, cur == 0 ? NS - 1 : cur - 1);
    const bf16_t* A = lds + cur * STAGE;
    const bf16_t* B = A + BM * BKS;
    v8s fa[MI], fb[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) fb[j] = *reinterpret_cast<const v8s*>(B + (wn * TN + j * 16) * BKS + foff);
#pragma unroll
    for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const v8s*>(A + (wm * TM + i * 16) * BKS + foff);
    if constexpr (ABN) {
      const int c0 = (kt * BKS) % a.Cs + 8 * (lane >> 4);
      const v4f s0 = *reinterpret_cast<const v4f*>(a.pre + c0), s1 = *reinterpret_cast<const v4f*>(a.pre + c0 + 4);
      const v4f t0 = *reinterpret_cast<const v4f*>(a.pre + a.Cs + c0), t1 = *reinterpret_cast<const v4f*>(a.pre + a.Cs + c0 + 4);
      const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
      const float sh[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        v4u u = __builtin_bit_cast(v4u, fa[i]);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          u[e] = pack2bf(fmaxf(lo_bf(u[e]) * sc[2 * e] + sh[2 * e], 0.f), fmaxf(hi_bf(u[e]) * sc[2 * e + 1] + sh[2 * e + 1], 0.f));
        fa[i] = __builtin_bit_cast(v8s, u);
      }
    }
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    // retire step kt + 1 (later steps stay in flight); order every wave's reads of this stage and its DMA before
    // anything after the barrier
    const int ahead = min(nk - 1, kt + NS - 1) - (kt + 1);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * L) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(L) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    cur = cur == NS - 1 ? 0 : cur + 1;
  }
  float* wl = reinterpret_cast<float*>(lds) + wave * SL;
  nt_epilogue_lds<MI, NI, TM, TN, NH, WGN * SL, WGM>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid, wl, wm);
}

// ------------------------------------------------------------------------------------------------
// 256 x 256 implicit-GEMM NT tile, BK = 64, 8 waves (2 M-halves x 4 N-quarters, 128 x 64 outputs per wave), one
// workgroup per CU, two 64 KB LDS buffers. Phase-interleaved K-loop after the 8-phase template of
// cdna_hip_programming.md §5: every K-tile is four phases; a phase is a LOAD segment (one LDS-DMA piece, fragment
// ds_reads, a counted vmcnt) + barrier + a COMPUTE segment of 16 MFMAs (one 64 x 32 quadrant of the wave's tile,
// K = 64) + barrier. The wave group of the second M-half runs one barrier behind the first, so on every SIMD one wave
// computes while its partner loads.
// A buffer holds a K-tile as four 16 KB pieces of 128 rows x 128 B (slot s of row r holds granule s ^ (r & 7), the
// swizzle applied on the DMA source side), cut by the phase that first reads them:
//   P0 = A rows of quadrant 0 of both M-halves, P1 = B rows of N-quadrant 0 of the four N-quarters,
//   P2 = A quadrant 1, P3 = B quadrant 1.
// Per K-tile t (reads from buffer t & 1; B fragments of both N-quadrants stay in registers through the tile):
//   ph0: DMA P3(t+1); read A q0 + B q0 (P0, P1); vmcnt -> P3(t) landed        -> MFMA (0, 0)
//   ph1: DMA P2(t+1); read B q1 (P3);            vmcnt -> P2(t) landed        -> MFMA (0, 1)
//   ph2: DMA P0(t+2); read A q1 (P2)                                          -> MFMA (1, 1)
//   ph3: DMA P1(t+2);                            vmcnt -> P0, P1(t+1) landed  -> MFMA (1, 0)
// so one DMA piece is issued per phase, each piece has 4-5 phases to land, and at most four pieces (eight DMA
// instructions per thread) are in flight. Hazards: a piece is waited for (counted vmcnt by every issuing wave) in the
// LOAD segment before the one that reads it, i.e. before a barrier both groups pass first; a piece of buffer b is
// overwritten at least two phases after its last read, by which time both groups retired that read (lgkmcnt(0) at
// the start of their COMPUTE segment). The wave tile and the epilogue are those of conv_nt_w8_kernel.
// FASTK only (Cs % 64 == 0: a K-tile lies in one tap). SPLIT: fp32 partials of a K range per blockIdx.y.
// ABL (diagnostic ablation builds, BIGDL_P8_ABL; wrong outputs): bit 0 no LDS-DMA inside the K-loop, bit 1 no fragment
// ds_reads after the first K-tile, bit 2 no wave-group stagger, bit 3 no MFMAs, bit 4 no A-operand DMA, bit 5 no
// B-operand DMA; bit 6 (64) is not an ablation: the one-tap K-tail mode (Cs % 64 != 0, granules past Kdim zero)
// SK (stream-K): gridDim.x persistent workgroups (one per CU) share the tiles x K-tiles iteration space evenly, so a
// small grid (ResNet-50's 14x14 / 7x7 layers: 98-392 tiles of 256 x 256 on 256 CUs) keeps every CU busy. A workgroup
// runs its range as segments (one tile's K sub-range each) through the same pipeline; a segment that covers a whole
// tile finishes it directly, otherwise it parks its fp32 accumulators (register order, write-through sc1 stores, one
// 256 KB slot per (tile, segment) in ws), drains them, and takes a ticket on the tile's counter; the workgroup that
// draws the last ticket reads every slot of the tile (sc1 loads) in segment order (the sum is independent of
// arrival order: deterministic), and runs the fused epilogue. Nobody waits on anybody: correct whatever the
// residency (the splitk-seam recipe of cdna_hip_programming.md §5 item 2, last-arriver form). a.ksplit = slots per
// tile; the tickets follow the slots in ws and are zeroed by a fill kernel before the launch.
template <bool SPLIT, int ABL = 0, bool SK = false>
__global__ __launch_bounds__(512, 2) void conv_nt_p8_kernel(ConvArgs a) {
  constexpr int BM = 256, BN = 256, BKT = 64;
  constexpr int WGM = 2, WGN = 4;
  constexpr int TM = BM / WGM, TN = BN / WGN;      // 128 x 64 per wave
  constexpr int MI = TM / 16, NI = TN / 16;        // 8 x 4 MFMA tiles
  constexpr int PIECE = 128 * BKT;                 // bf16 elements per piece (16 KB)
  constexpr int BUF = 4 * PIECE;                   // P0 P1 P2 P3 (64 KB)
  constexpr int NH = 4;                            // epilogue row chunks
  constexpr int SL = (TM / NH) * TN;
  static_assert(8 * SL * 4 <= 2 * BUF * 2, "epilogue chunk must fit the buffers");
  __shared__ __attribute__((aligned(1024))) bf16_t lds[2 * BUF + 3 * CONV_MAX_TAPS + 8];
  short* taps = reinterpret_cast<short*>(lds + 2 * BUF);
  int* skflag = reinterpret_cast<int*>(lds + 2 * BUF + 3 * CONV_MAX_TAPS);   // in the one LDS array (see above)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WGN, wn = wave % WGN;
  const int tiles_n = (a.Ncol + BN - 1) / BN;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  constexpr bool KTAIL = (ABL & 64) != 0;          // one tap, Cs % 64 != 0: granules past Kdim load zeros
  const int nk_all = KTAIL ? (a.Kdim + BKT - 1) / BKT : a.Kdim / BKT;
  if (tid < a.ntaps) {
    taps[tid] = a.tap_h[tid];
    taps[CONV_MAX_TAPS + tid] = a.tap_w[tid];
    taps[2 * CONV_MAX_TAPS + tid] = a.tap_k[tid];
  }
  __syncthreads();   // tap table visible (no DMA outstanding yet)

  // stream-K range of this workgroup in the (tile, K-tile) iteration space
  const long I = (long)nwg * nk_all;
  const long G = gridDim.x;
  long it = SK ? ((long)blockIdx.x * I) / G : 0;
  const long it_end = SK ? ((long)(blockIdx.x + 1) * I) / G : 1;
  auto wg_of = [&](long x) -> int {                // the workgroup whose range holds iteration x
    long w = (x * G) / I;
    while (w + 1 < G && ((w + 1) * I) / G <= x) ++w;
    while (w > 0 && (w * I) / G > x) --w;
    return (int)w;
  };

  for (;;) {
  int bid, tm, tn, kt0, nk;
  if constexpr (SK) {
    if (it >= it_end) break;
    const int tile = (int)(it / nk_all);
    kt0 = (int)(it - (long)tile * nk_all);
    nk = (int)min((long)(nk_all - kt0), it_end - it);
    it += nk;
    bid = tile;
    tm = tile / tiles_n; tn = tile % tiles_n;
  } else {
    bid = xcd_remap(blockIdx.x, nwg);
    tm = bid / tiles_n; tn = bid % tiles_n;
    kt0 = 0; nk = nk_all;
    if constexpr (SPLIT) {
      const int per = (nk_all + a.ksplit - 1) / a.ksplit;
      kt0 = blockIdx.y * per;
      nk = max(0, min(nk_all, kt0 + per) - kt0);
    }
  }
  const int m0 = tm * BM, n0 = tn * BN;

  // DMA geometry: instruction j of wave w fills piece rows (j * 8 + w) * 8 .. +8 (8 rows x 128 B); lane -> row
  // + (lane >> 3), slot lane & 7, which must hold granule (lane & 7) ^ (row & 7) = (lane & 7) ^ (lane >> 3).
  // Piece row lr of an A piece of quadrant q is tile row (lr >> 6) * 128 + q * 64 + (lr & 63); of a B piece of
  // quadrant q, tile column (lr >> 5) * 64 + q * 32 + (lr & 31). Slot q2 = q * 2 + j of the per-thread tables.
  const int gsrc = (lane & 7) ^ (lane >> 3);
  const int ohw = a.OH * a.OW;
  int a_pix[4], a_h[4], a_w[4];
  const bf16_t* wrow[4];
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
    wrow[q2] = a.wt + (size_t)(bvalid[q2] ? n : 0) * a.ldw + gsrc * 8;
  }
  // piece P (0 A q0, 1 B q0, 2 A q1, 3 B q1) of K-tile kt into buffer buf: 2 DMA instructions per thread
  auto issue = [&](int kt, int buf, int P) {
    const int k0 = kt * BKT;
    const int t = k0 / a.Cs;
    const int cin = k0 - t * a.Cs;
    bf16_t* base = lds + buf * BUF + P * PIECE;
    const int q = P >> 1;
    if ((ABL & 16) && (P & 1) == 0) return;
    if ((ABL & 32) && (P & 1) == 1) return;
    if ((P & 1) == 0) {
      const int th = taps[t], tw = taps[CONV_MAX_TAPS + t];
      const int c = cin + gsrc * 8;
      const bool kin = !KTAIL || c < a.Cs;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q2 = q * 2 + j;
        const int ch = a_h[q2] + th, cw = a_w[q2] + tw;
        const bool ok = kin && (unsigned)ch < (unsigned)a.Hs && (unsigned)cw < (unsigned)a.Ws;
        const bf16_t* src = ok ? a.src + (unsigned)((a_pix[q2] + ch * a.Ws + cw) * a.Cs + c) : g_zero_granule;
        glds16(src, (LDS_PTR(void))(base + (j * 8 + wave) * 8 * BKT));
      }
    } else {
      const int wk = taps[2 * CONV_MAX_TAPS + t] * a.Cs + cin;
      const bool kin = !KTAIL || cin + gsrc * 8 < a.Cs;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q2 = q * 2 + j;
        const bf16_t* src = (kin && bvalid[q2]) ? wrow[q2] + wk : g_zero_granule;
        glds16(src, (LDS_PTR(void))(base + (j * 8 + wave) * 8 * BKT));
      }
    }
  };
  // fragment slot of K-half kh: granule kh * 4 + (lane >> 4) of piece row (lane & 15) + 16 i lives at slot ^ (lane & 7)
  const int fo0 = (lane & 15) * BKT + (((lane >> 4)) ^ (lane & 7)) * 8;
  const int fo1 = (lane & 15) * BKT + ((4 + (lane >> 4)) ^ (lane & 7)) * 8;
  const int a_row = wm * 64 * BKT;                 // this wave's rows inside an A piece
  const int b_row = wn * 32 * BKT;                 // this wave's rows inside a B piece

  v4f acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};

  v8s fa[4][2], fb[NI][2];
  // 16 MFMAs of one 64 x 32 quadrant (rows ib .. ib + 3, columns jb, jb + 1), K-halves outermost so no two
  // consecutive MFMAs accumulate into the same tile
  auto quad = [&](int ib, int jb) {
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ib + i][jb + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[jb + j][kh], fa[i][kh], acc[ib + i][jb + j], 0, 0, 0);
  };
  auto read_a = [&](const bf16_t* P) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i][0] = *reinterpret_cast<const v8s*>(P + a_row + i * 16 * BKT + fo0);
      fa[i][1] = *reinterpret_cast<const v8s*>(P + a_row + i * 16 * BKT + fo1);
    }
  };
  auto read_b = [&](const bf16_t* P, int jb) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      fb[jb + j][0] = *reinterpret_cast<const v8s*>(P + b_row + j * 16 * BKT + fo0);
      fb[jb + j][1] = *reinterpret_cast<const v8s*>(P + b_row + j * 16 * BKT + fo1);
    }
  };
  auto compute = [&](int ib, int jb) {
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    if constexpr (!(ABL & 8)) quad(ib, jb);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  };

  // prologue: K-tile 0 whole, then P0, P1 of K-tile 1; retire P0, P1 of K-tile 0
  if (nk > 0) {
    issue(kt0, 0, 0); issue(kt0, 0, 1); issue(kt0, 0, 3); issue(kt0, 0, 2);
  }
  if (nk > 1) {
    issue(kt0 + 1, 1, 0); issue(kt0 + 1, 1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  if (!(ABL & 4) && wm == 1) __builtin_amdgcn_s_barrier();   // stagger: the second M-half runs one barrier behind

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bf16_t* L = lds + cur * BUF;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    // ---- phase 0
    if (!(ABL & 1) && n1) issue(kt0 + kt + 1, cur ^ 1, 3);
    if (!(ABL & 2) || kt == 0) { read_a(L); read_b(L + PIECE, 0); }
    if (n1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");          // P3(t) landed
    else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    compute(0, 0);
    // ---- phase 1
    if (!(ABL & 1) && n1) issue(kt0 + kt + 1, cur ^ 1, 2);
    if (!(ABL & 2) || kt == 0) read_b(L + 3 * PIECE, 2);
    if (n1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");          // P2(t) landed
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    compute(0, 2);
    // ---- phase 2
    if (!(ABL & 1) && n2) issue(kt0 + kt + 2, cur, 0);
    if (!(ABL & 2) || kt == 0) read_a(L + 2 * PIECE);
    compute(4, 2);
    // ---- phase 3
    if (!(ABL & 1) && n2) issue(kt0 + kt + 2, cur, 1);
    if (n2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");          // P0, P1(t+1) landed
    else if (n1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    compute(4, 0);
  }
  if (!(ABL & 4) && wm == 0) __builtin_amdgcn_s_barrier();   // balance the stagger: every wave has left the K-loop
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float* wl = reinterpret_cast<float*>(lds) + wave * SL;
  if constexpr (SK) {
    bool finish = kt0 == 0 && nk == nk_all;
    if (!finish) {
      const int tile = bid;
      const int w0 = wg_of((long)tile * nk_all), w1 = wg_of((long)(tile + 1) * nk_all - 1);
      const int nseg = w1 - w0 + 1, seg = (int)blockIdx.x - w0;
      constexpr int SLOT = MI * NI * 512 * 4;      // floats per (tile, segment) slot
      float* slots = a.ws + (size_t)tile * a.ksplit * SLOT;
      {
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(slots + (size_t)seg * SLOT, (short)0,
                                                                           SLOT * 4, 0x00020000);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, acc[i][j]), r, (((i * NI + j) * 512 + tid) * 4) * 4,
                                                   0, 16);   // sc1: write-through
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its slot stores have left
      __syncthreads();
      if (tid == 0) {
        unsigned* cnt = reinterpret_cast<unsigned*>(a.ws + (size_t)nwg * a.ksplit * SLOT) + tile;
        const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *skflag = (prev == (unsigned)(nseg - 1)) ? 1 : 0;
      }
      __syncthreads();
      finish = *skflag != 0;
      if (finish) {   // last arriver: every slot of the tile, in segment order
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
        for (int sgi = 0; sgi < nseg; ++sgi) {
          const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(slots + (size_t)sgi * SLOT, (short)0,
                                                                             SLOT * 4, 0x00020000);
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            if (i & 1) asm volatile("" ::: "memory");     // <= 8 slot loads in flight (VGPR budget)
#pragma unroll
            for (int j = 0; j < NI; ++j)
              acc[i][j] += __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(r, (((i * NI + j) * 512 + tid) * 4) * 4, 0, 16));
          }
        }
      }
    }
    if (finish) nt_epilogue_lds<MI, NI, TM, TN, NH, WGN * SL, WGM>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid, wl, wm);
    __syncthreads();   // the LDS is restaged by the next segment
  } else if constexpr (SPLIT) {
    store_partials_lds<MI, NI, TM, TN, NH>(a.ws + (size_t)blockIdx.y * a.M * a.Ncol, a.M, a.Ncol, acc,
                                           m0 + wm * TM, n0 + wn * TN, lane, wl);
  } else {
    nt_epilogue_lds<MI, NI, TM, TN, NH, WGN * SL, WGM>(a, acc, m0 + wm * TM, n0 + wn * TN, lane, bid, wl, wm);
  }
  if constexpr (!SK) break;
  }
}

// ------------------------------------------------------------------------------------------------
// Streaming 1x1 kernel for the HBM-bound one-tap GEMMs: identity pixel mapping (1x1, stride 1, no padding: A row m =
// source pixel m, dense rows of Kdim = Cs channels), Kdim in {64, 128}, Ncol % 64 == 0, identity output rows.
// ResNet-50's 64 -> 256 expansions, 128 -> 512, 64 -> 64 and the data gradients of the 256 -> 64 / 512 -> 128
// reductions are such GEMMs: 1-4 K-steps of MFMA per tile and a 2-8x wider output than input, so the per-tile kernel
// (conv_nt_g4: load, 2 K-steps, LDS epilogue, per-tile statistics atomics) ran them at 2-3 TB/s, latency- and
// issue-bound (layer 3 fwd: 43 % of wave time waiting, 1,300 VALU per wave). Here (measured on the standalone
// structure first, tools/ubench/nt_stream.hip: layer 3 fwd 202 -> 108 us = the 4.8 TB/s copy ceiling of its bytes):
//  * persistent: 2 workgroups per CU, each strides over pixel tiles of one fixed channel block, so every
//    per-channel quantity (the weight fragments, bias, BN mean / scale / shift, the statistics sums) is loaded or
//    reduced ONCE per workgroup instead of once per tile;
//  * wave w owns 64 output channels (cg = w % CG) of a BMW-pixel sub-tile (pg = w / CG); its weights live in VGPRs
//    as MFMA A fragments for the whole launch (K = 64: 32 VGPRs, K = 128: 64);
//  * A fragments are loaded straight from HBM into VGPRs (16 B per lane, no LDS staging: the tile is read once and
//    used by one wave), two tiles ahead of the one being computed (register triple buffer, static indices);
//  * epilogue: the wave parks its tile in its own LDS slice ([pixel][64 channels], 16-byte granules XOR-swizzled by
//    pixel; bf16 when nothing is added before rounding, else fp32), re-reads it row-wise (8 channels of one pixel per
//    lane) and writes whole 128-byte lines with 16-byte stores; addend / BN x / z rows for the consumer-BN backward
//    reduction are loaded before the tile's MFMAs (EXT);
//  * statistics (sum, sum of squares of the rounded output) or the consumer-BN backward sums accumulate in packed
//    2 x f32 registers across all tiles of the workgroup; one shuffle reduction and one slotted atomic per channel at
//    the end (same-address atomics serialise at the memory side: slots = block id % BIGDL_STAT_SLOTS).
// Semantics are nt_epilogue_lds's (bias + addend added in fp32 before rounding, ReLU, BN statistics of the rounded
// output, consumer-BN reduction of the rounded gradient with the z / affine ReLU mask).
template <int K, int CG, int BMW, bool F32T, bool EXT, bool PRE = false>
__global__ __launch_bounds__(256, K >= 256 ? 1 : 2) void conv_nt_s1_kernel(ConvArgs a) {
  constexpr int KF = K / 32, MI = BMW / 16, PGN = 4 / CG, BM = BMW * PGN;
  // EXT operands one tile ahead of their use (PF); K = 128 pays for the registers with a double instead of a triple
  // register buffer of A tiles (2 WG/CU: 256 VGPRs)
  constexpr bool PF = EXT && K >= 128;
  constexpr int NB = (EXT && K == 128) ? 2 : 3;
  constexpr int GPR = F32T ? 16 : 8;               // 16-byte granules per 64-channel row of the LDS slice
  constexpr int NR = BMW / 8;                      // row-phase passes (8 pixels x 8 lanes each)
  __shared__ __attribute__((aligned(16))) unsigned lds[4 * BMW * GPR * 4 + (PRE ? 2 * K : 0)];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cg = wave % CG, pg = wave / CG;
  const int nchb = a.Ncol / (64 * CG);
  const int chb = blockIdx.x % nchb, wgi = blockIdx.x / nchb, ngr = gridDim.x / nchb;
  const int c0 = (chb * CG + cg) * 64;
  const int ntiles = (a.M + BM - 1) / BM;
  unsigned* wl = lds + wave * BMW * GPR * 4;
  const int q = lane & 7;                          // row phase: channels c0 + 8 q .. + 7
  const int n = c0 + 8 * q;

  v8s wf[4][KF];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int kk = 0; kk < KF; ++kk)
      wf[j][kk] = *reinterpret_cast<const v8s*>(a.wt + (size_t)(c0 + 16 * j + (lane & 15)) * a.ldw + 32 * kk +
                                                8 * (lane >> 4));
  // PRE: the A operand is relu(x * scale[c] + shift[c]) of the producing BatchNorm (ConvArgs::pre): the [scale K |
  // shift K] table sits in LDS behind the wave slices (in VGPRs it spilled); a lane's fragment channels are
  // 32 kk + 8 (lane >> 4) + e
  const float* ptab = reinterpret_cast<const float*>(lds + 4 * BMW * GPR * 4);
  if constexpr (PRE) {
    for (int i = threadIdx.x; i < K / 2; i += 256)
      reinterpret_cast<v4f*>(lds + 4 * BMW * GPR * 4)[i] = reinterpret_cast<const v4f*>(a.pre)[i];
    __syncthreads();
  }
  float bs[8], bmu[8], bsc[8], bsh[8];
  const bool bnw = EXT && a.bnred && !a.stats;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bs[e] = (F32T && a.bias) ? a.bias[n + e] : 0.f;
    bmu[e] = bnw ? a.bnmean[n + e] : 0.f;
    bsc[e] = (bnw && a.bnaff) ? a.bnaff[n + e] : 0.f;
    bsh[e] = (bnw && a.bnaff) ? a.bnaff[a.Ncol + n + e] : 0.f;
  }
  typedef float v2f __attribute__((ext_vector_type(2)));
  v2f p1[4], p2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) p1[e] = p2[e] = v2f{0.f, 0.f};
  // EXT operands through buffer resources: an absent operand gets a 0-byte resource (its loads return zeros), so the
  // loads carry no branches — branch joins around loads made the compiler drain vmcnt before the stores (328
  // branches, 36 vmcnt(0) in the 64-channel EXT kernel); tail rows store through an out-of-range offset
  const size_t ob = EXT ? ((size_t)(a.M - 1) * a.ldo + a.Ncol) * 2 : 0;
  const __amdgpu_buffer_rsrc_t r_add = rsrc_of(a.addend, (EXT && a.addend) ? ob : 0);
  const __amdgpu_buffer_rsrc_t r_azm = rsrc_of(a.addzm, (EXT && a.addzm) ? ob / 16 : 0);
  const __amdgpu_buffer_rsrc_t r_bx = rsrc_of(a.bnx, bnw ? ob : 0);
  const __amdgpu_buffer_rsrc_t r_bzm = rsrc_of(a.bnzm, (bnw && a.bnzm) ? ob / 16 : 0);
  const __amdgpu_buffer_rsrc_t r_out = rsrc_of(a.out, ob);
  const int zmode = !bnw ? 0 : a.bnzm ? 1 : a.bnaff ? 3 : 0;     // a bf16 z mask is not taken (s1_applies)
  const bool azm = a.addzm != nullptr;

  auto load = [&](v8s (&af)[MI][KF], int t) {
    const int p0 = t * BM + pg * BMW;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int m = min(p0 + 16 * i + (lane & 15), a.M - 1);   // tail rows: any valid row (never stored)
#pragma unroll
      for (int kk = 0; kk < KF; ++kk)
        af[i][kk] = *reinterpret_cast<const v8s*>(a.src + (size_t)m * K + 32 * kk + 8 * (lane >> 4));
    }
  };

  // epilogue operands of a tile (EXT): addend / BN x rows and their mask bytes; with PF they are loaded one tile
  // ahead (issued before the previous tile's MFMAs) instead of at the start of the tile that consumes them
  // (mask bytes kept apart until use: combining them where they are loaded would wait for the loads there)
  struct ExtOps { v4u pad[EXT ? NR : 1], px[EXT ? NR : 1]; unsigned pza[EXT ? NR : 1], pzz[EXT ? NR : 1]; };
  auto load_ext = [&](ExtOps& e, int t) {
    if constexpr (EXT) {
      const int p0 = t * BM + pg * BMW;
#pragma unroll
      for (int rr = 0; rr < NR; ++rr) {
        const int m = min(p0 + rr * 8 + (lane >> 3), a.M - 1);
        const size_t off = (size_t)m * a.ldo + n;
        const unsigned eb = (unsigned)(off * 2), zo = (unsigned)(off >> 3);
        e.pad[rr] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r_add, eb, 0, 0));
        e.px[rr] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r_bx, eb, 0, 0));
        e.pza[rr] = __builtin_amdgcn_raw_buffer_load_b8(r_azm, zo, 0, 0);     // addend mask
        e.pzz[rr] = __builtin_amdgcn_raw_buffer_load_b8(r_bzm, zo, 0, 0);     // consumer-BN sign mask
      }
    }
  };

  auto compute_store = [&](v8s (&af)[MI][KF], ExtOps& eo, int t) {
    const int p0 = t * BM + pg * BMW;
    ExtOps el;
    if constexpr (EXT && !PF) load_ext(el, t);   // epilogue operands first: latency overlaps the MFMAs
    ExtOps& e = PF ? eo : el;
    auto& pad = e.pad;
    auto& px = e.px;
    v4f acc[MI][4];
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
    if constexpr (PRE) {     // BN apply + ReLU on the loaded operand (bn_apply_kernel's expression and rounding)
#pragma unroll
      for (int kk = 0; kk < KF; ++kk) {
        const int c = 32 * kk + 8 * (lane >> 4);
        const v4f s0 = *reinterpret_cast<const v4f*>(ptab + c), s1 = *reinterpret_cast<const v4f*>(ptab + c + 4);
        const v4f b0 = *reinterpret_cast<const v4f*>(ptab + K + c), b1 = *reinterpret_cast<const v4f*>(ptab + K + c + 4);
        const float sc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
        const float sh[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          v4u u = __builtin_bit_cast(v4u, af[i][kk]);
#pragma unroll
          for (int e = 0; e < 4; ++e)
            u[e] = pack2bf(fmaxf(lo_bf(u[e]) * sc[2 * e] + sh[2 * e], 0.f),
                           fmaxf(hi_bf(u[e]) * sc[2 * e + 1] + sh[2 * e + 1], 0.f));
          af[i][kk] = __builtin_bit_cast(v8s, u);
        }
      }
    }
#pragma unroll
    for (int kk = 0; kk < KF; ++kk)
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][kk], af[i][kk], acc[i][j], 0, 0, 0);
    // D[n][m]: lane holds channels 16 j + 4 (lane >> 4) + e of pixel 16 i + (lane & 15)
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = 16 * i + (lane & 15), qq = lane >> 4;
        if constexpr (F32T) {
          const int g = 4 * j + qq;
          *reinterpret_cast<v4f*>(wl + (p * GPR + (g ^ (p & 15))) * 4) = acc[i][j];
        } else {
          const int g = 2 * j + (qq >> 1);
          *reinterpret_cast<v2u*>(wl + (p * GPR + (g ^ (p & 7))) * 4 + (qq & 1) * 2) =
              v2u{pack2bf(acc[i][j][0], acc[i][j][1]), pack2bf(acc[i][j][2], acc[i][j][3])};
        }
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): wave-private slice
#pragma unroll
    for (int rr = 0; rr < NR; ++rr) {
      const int p = rr * 8 + (lane >> 3);
      const int m = p0 + p;
      v4u o;
      if constexpr (F32T) {
        const v4f lo = *reinterpret_cast<const v4f*>(wl + (p * GPR + ((2 * q) ^ (p & 15))) * 4);
        const v4f hi = *reinterpret_cast<const v4f*>(wl + (p * GPR + ((2 * q + 1) ^ (p & 15))) * 4);
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        if constexpr (EXT) {
          const v4u pa = azm ? (pad[rr] & mask8_to_and(e.pza[rr] & 0xffu)) : pad[rr];
#pragma unroll
          for (int e = 0; e < 4; ++e) { v[2 * e] += lo_bf(pa[e]); v[2 * e + 1] += hi_bf(pa[e]); }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float x0 = v[2 * e] + bs[2 * e], x1 = v[2 * e + 1] + bs[2 * e + 1];
          if (a.relu) { x0 = fmaxf(x0, 0.f); x1 = fmaxf(x1, 0.f); }
          o[e] = pack2bf(x0, x1);
        }
      } else {
        o = *reinterpret_cast<const v4u*>(wl + (p * GPR + (q ^ (p & 7))) * 4);
        if (a.relu) {
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] = pack2bf(fmaxf(lo_bf(o[e]), 0.f), fmaxf(hi_bf(o[e]), 0.f));
        }
      }
      if constexpr (EXT) {
        // branch-free: masks as selects, tail rows contribute zero and store out of range
        const float vm = m < a.M ? 1.f : 0.f;
        if (a.stats) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const v2f y = v2f{lo_bf(o[e]), hi_bf(o[e])} * vm;
            p1[e] += y;
            p2[e] = __builtin_elementwise_fma(y, y, p2[e]);
          }
        } else {
          const unsigned zb = e.pzz[rr] & 0xffu;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            v2f d = v2f{lo_bf(o[e]), hi_bf(o[e])} * vm;
            const v2f x = {lo_bf(px[rr][e]), hi_bf(px[rr][e])};
            bool k0 = true, k1 = true;
            if (zmode == 1) { k0 = (zb >> (2 * e)) & 1u; k1 = (zb >> (2 * e + 1)) & 1u; }
            else if (zmode == 3) { k0 = x[0] * bsc[2 * e] + bsh[2 * e] > 0.f; k1 = x[1] * bsc[2 * e + 1] + bsh[2 * e + 1] > 0.f; }
            d[0] = k0 ? d[0] : 0.f;
            d[1] = k1 ? d[1] : 0.f;
            p1[e] += d;
            p2[e] = __builtin_elementwise_fma(d, x - v2f{bmu[2 * e], bmu[2 * e + 1]}, p2[e]);
          }
        }
        const unsigned so = m < a.M ? (unsigned)(((size_t)m * a.ldo + n) * 2) : EOOB;
        __builtin_amdgcn_raw_buffer_store_b128(o, r_out, so, 0, 0);
      } else if (m < a.M) {
        if (a.stats) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const v2f y = {lo_bf(o[e]), hi_bf(o[e])};
            p1[e] += y;
            p2[e] = __builtin_elementwise_fma(y, y, p2[e]);
          }
        }
        *reinterpret_cast<v4u*>(a.out + (size_t)m * a.ldo + n) = o;
      }
    }
  };

  int t = wgi;
  if constexpr (NB == 2) {
    v8s a0[MI][KF], a1[MI][KF];
    ExtOps e0, e1;
    if (t < ntiles) load(a0, t);
    if constexpr (PF) load_ext(e0, t);       // rows are clamped: a tile past the end reads valid rows, unused
    for (; t < ntiles; t += 2 * ngr) {
      if (t + ngr < ntiles) load(a1, t + ngr);
      if constexpr (PF) load_ext(e1, t + ngr);
      compute_store(a0, e0, t);
      if (t + ngr >= ntiles) break;
      if (t + 2 * ngr < ntiles) load(a0, t + 2 * ngr);
      if constexpr (PF) load_ext(e0, t + 2 * ngr);
      compute_store(a1, e1, t + ngr);
    }
  } else {
    v8s a0[MI][KF], a1[MI][KF], a2[MI][KF];
    ExtOps e0, e1, e2;     // live only with PF (two at a time: the consumed tile's and the next one's)
    if (t < ntiles) load(a0, t);
    if (t + ngr < ntiles) load(a1, t + ngr);
    if constexpr (PF) load_ext(e0, t);
    for (; t < ntiles; t += 3 * ngr) {
      if (t + 2 * ngr < ntiles) load(a2, t + 2 * ngr);
      if constexpr (PF) load_ext(e1, t + ngr);
      compute_store(a0, e0, t);
      if (t + ngr >= ntiles) break;
      if (t + 3 * ngr < ntiles) load(a0, t + 3 * ngr);
      if constexpr (PF) load_ext(e2, t + 2 * ngr);
      compute_store(a1, e1, t + ngr);
      if (t + 2 * ngr >= ntiles) break;
      if (t + 4 * ngr < ntiles) load(a1, t + 4 * ngr);
      if constexpr (PF) load_ext(e0, t + 3 * ngr);
      compute_store(a2, e2, t + 2 * ngr);
    }
  }
  float* const red = a.stats ? a.stats : (bnw ? a.bnred : nullptr);
  if (red) {
    float s1[8], s2[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) { s1[2 * e] = p1[e][0]; s1[2 * e + 1] = p1[e][1]; s2[2 * e] = p2[e][0]; s2[2 * e + 1] = p2[e][1]; }
    // lanes l, l + 8, ... hold the same 8 channels: reduce over lane >> 3
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    if (lane < 8) {
      float* sp = red + (size_t)(blockIdx.x & (BIGDL_STAT_SLOTS - 1)) * 2 * a.Ncol;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        atomicAdd(sp + n + e, s1[e]);
        atomicAdd(sp + a.Ncol + n + e, s2[e]);
      }
    }
  }
}

// Grid of the split-K epilogue: (row blocks, 256-group channel chunks), ~8 rows per thread, <= 8192 blocks.
dim3 splitk_grid(long P, int C, long* rpb_out) {
  const int G = C >> 3;
  const int rpi = 256 / (G < 256 ? G : 256);
  const int gy = (G + 255) / 256;
  long rpb = (long)rpi * 8;
  long bx = (P + rpb - 1) / rpb;
  const long cap = 8192 / gy;
  if (bx > cap) {
    bx = cap;
    rpb = (P + bx - 1) / bx;
  }
  if (bx < 1) bx = 1;
  *rpb_out = rpb;
  return dim3((unsigned)bx, (unsigned)gy);
}

// Split-K epilogue: out = fused_epilogue(sum over splits of ws[s][m][n]) with exactly nt_epilogue_lds's semantics
// (+ bias, + addend, ReLU, bf16 store at the output placement, BN statistics of the rounded output or the consumer
// BN's backward reduction). Channel-stationary: a thread owns 8 channels of rows rsub, rsub + rpi, ...; per-channel
// sums are combined across the block's rows in LDS and added into the statistics slots with one atomic each.
__global__ __launch_bounds__(256) void conv_splitk_epilogue_kernel(ConvArgs a, long rpb) {
  __shared__ float sm[256 * 16];
  const int G = a.Ncol >> 3;
  const int gbase = blockIdx.y * 256;
  const int gcount = min(256, G - gbase);
  const int rpi = 256 / gcount;
  const int g = gbase + threadIdx.x % gcount, rsub = threadIdx.x / gcount;
  const bool act = rsub < rpi;
  const long rbeg = blockIdx.x * rpb, rend = min((long)a.M, rbeg + rpb);
  const int n = g * 8;
  const size_t plane = (size_t)a.M * a.Ncol;
  const int ohw = a.OH * a.OW;
  float bs[8], bmu[8], bsc[8], bsh[8], s1[8], s2[8];
  const bool bnw = a.bnred && !a.stats;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bs[e] = (act && a.bias) ? a.bias[n + e] : 0.f;
    bmu[e] = (act && bnw) ? a.bnmean[n + e] : 0.f;
    bsc[e] = (act && bnw && a.bnaff) ? a.bnaff[n + e] : 0.f;
    bsh[e] = (act && bnw && a.bnaff) ? a.bnaff[a.Ncol + n + e] : 0.f;
    s1[e] = s2[e] = 0.f;
  }
  if (act) {
    for (long m = rbeg + rsub; m < rend; m += rpi) {
      float v[8];
      const float* p = a.ws + (size_t)m * a.Ncol + n;
      {
        const v4f lo = *reinterpret_cast<const v4f*>(p), hi = *reinterpret_cast<const v4f*>(p + 4);
        v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3]; v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
      }
      for (int s = 1; s < a.ksplit; ++s) {
        const v4f lo = *reinterpret_cast<const v4f*>(p + s * plane), hi = *reinterpret_cast<const v4f*>(p + s * plane + 4);
        v[0] += lo[0]; v[1] += lo[1]; v[2] += lo[2]; v[3] += lo[3]; v[4] += hi[0]; v[5] += hi[1]; v[6] += hi[2]; v[7] += hi[3];
      }
      long orow = m;
      if (!a.ident_out) {
        const int nb = (int)(m / ohw), rem = (int)(m - (long)nb * ohw);
        const int oh = rem / a.OW, ow = rem - oh * a.OW;
        orow = ((long)nb * a.OHo + oh * a.omul_h + a.ooff_h) * a.OWo + ow * a.omul_w + a.ooff_w;
      }
      const size_t off = (size_t)orow * a.ldo + n;
      if (a.addend) {
        v4u q = *reinterpret_cast<const v4u*>(a.addend + off);
        if (a.addzm) q &= mask8_to_and(a.addzm[off >> 3]);
#pragma unroll
        for (int e = 0; e < 4; ++e) { v[2 * e] += lo_bf(q[e]); v[2 * e + 1] += hi_bf(q[e]); }
      }
      v4u o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x0 = v[2 * e] + bs[2 * e], x1 = v[2 * e + 1] + bs[2 * e + 1];
        if (a.relu) { x0 = fmaxf(x0, 0.f); x1 = fmaxf(x1, 0.f); }
        o[e] = pack2bf(x0, x1);
      }
      if (a.stats) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float y0 = lo_bf(o[e]), y1 = hi_bf(o[e]);
          s1[2 * e] += y0; s2[2 * e] += y0 * y0;
          s1[2 * e + 1] += y1; s2[2 * e + 1] += y1 * y1;
        }
      } else if (bnw) {
        const v4u px = *reinterpret_cast<const v4u*>(a.bnx + off);
        v4u pz = v4u{0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
        if (a.bnzm) pz = mask8_to_bf(a.bnzm[off >> 3]);
        else if (a.bnz) pz = *reinterpret_cast<const v4u*>(a.bnz + off);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float d0 = lo_bf(o[e]), d1 = hi_bf(o[e]);
          const float x0 = lo_bf(px[e]), x1 = hi_bf(px[e]);
          if (a.bnz || a.bnzm) {
            if (!(lo_bf(pz[e]) > 0.f)) d0 = 0.f;
            if (!(hi_bf(pz[e]) > 0.f)) d1 = 0.f;
          } else if (a.bnaff) {
            if (!(x0 * bsc[2 * e] + bsh[2 * e] > 0.f)) d0 = 0.f;
            if (!(x1 * bsc[2 * e + 1] + bsh[2 * e + 1] > 0.f)) d1 = 0.f;
          }
          s1[2 * e] += d0; s2[2 * e] += d0 * (x0 - bmu[2 * e]);
          s1[2 * e + 1] += d1; s2[2 * e + 1] += d1 * (x1 - bmu[2 * e + 1]);
        }
      }
      *reinterpret_cast<v4u*>(a.out + off) = o;
    }
  }
  float* const red = a.stats ? a.stats : a.bnred;
  if (red == nullptr) return;
#pragma unroll
  for (int e = 0; e < 8; ++e) { sm[threadIdx.x * 16 + e] = s1[e]; sm[threadIdx.x * 16 + 8 + e] = s2[e]; }
  __syncthreads();
  for (int w = threadIdx.x; w < gcount * 16; w += 256) {
    const int gg = w >> 4, slot = w & 15;
    float t = 0.f;
    for (int rs = 0; rs < rpi; ++rs) t += sm[(rs * gcount + gg) * 16 + slot];
    const int ch = (gbase + gg) * 8 + (slot & 7);
    atomicAdd(red + (size_t)(blockIdx.x & (BIGDL_STAT_SLOTS - 1)) * 2 * a.Ncol + (slot < 8 ? 0 : a.Ncol) + ch, t);
  }
}

template <int BM, int BN, int WM>
void launch_nt(const ConvArgs& a, bool fastk, hipStream_t st) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.Ncol + BN - 1) / BN);
  dim3 grid(nwg), block(256);
  if (fastk) conv_nt_kernel<BM, BN, WM, true><<<grid, block, 0, st>>>(a);
  else conv_nt_kernel<BM, BN, WM, false><<<grid, block, 0, st>>>(a);
}

template <int BM, int BN, int WM, bool FASTK = true, int NST = 2>
void launch_nt_glds(const ConvArgs& a, hipStream_t st) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.Ncol + BN - 1) / BN);
  conv_nt_glds_kernel<BM, BN, WM, FASTK, NST><<<dim3(nwg), dim3(256), 0, st>>>(a);
}

// single-stage kernel for Kdim == BK (BIGDL_CONV_ONESTAGE=0 disables it for A/B runs)
static bool conv_onestage() {
  static int v = [] { const char* e = getenv("BIGDL_CONV_ONESTAGE"); return e ? atoi(e) : 1; }();
  return v != 0;
}

// LDS-DMA path for Cs % 64 != 0 (BIGDL_CONV_GLDS_SLOWK=0 restores the register-staged kernel there)
static bool glds_slowk() {
  static int v = [] { const char* e = getenv("BIGDL_CONV_GLDS_SLOWK"); return e ? atoi(e) : 1; }();
  return v != 0;
}

template <int BM, int BN, int WM>
void launch_nt_pers(const ConvArgs& a, hipStream_t st) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.Ncol + BN - 1) / BN);
  const int grid = std::min(nwg, 2 * 256);
  conv_nt_pers_kernel<BM, BN, WM><<<dim3(grid), dim3(256), 0, st>>>(a);
}

template <int BN, int WGM, int WGN>
void launch_nt_p3(const ConvArgs& a, hipStream_t st) {
  const int nwg = ((a.M + 255) / 256) * ((a.Ncol + BN - 1) / BN);
  conv_nt_p3_kernel<BN, WGM, WGN><<<dim3(nwg), dim3(512), 0, st>>>(a);
}

// BIGDL_CONV_IMPL: 3 = persistent LDS-DMA kernel (next tile's loads overlap the epilogue) on grids of more
// than two tiles per CU, 2 = deep-pipelined 256-pixel kernel on grids that fill the chip,
// 1 (default) = LDS-DMA kernel where Cs % 64 == 0, 0 = register-staged kernel everywhere.
// 256 x 256 8-wave kernel (BIGDL_CONV_W8=0 disables it): fast-K over 32-channel steps, aligned bf16 output, at
// least 256 output channels, at least 4 K-steps of 32. Returns 0 (not picked) or the K split (1 = none): grids below
// one workgroup per CU are split along K (>= 8 K-steps per split) so every CU gets work.
static int w8_pick(const ConvArgs* a) {
  static const int on = [] { const char* e = getenv("BIGDL_CONV_W8"); return e ? atoi(e) : 0; }();
  if (!on || a->out32 || (a->Cs % 32) || (a->Ncol & 7) || (a->ldo & 7) || a->Ncol < 256 || a->Kdim < 128) return 0;
  const long tiles = (long)((a->M + 255) / 256) * ((a->Ncol + 255) / 256);
  const int nk = a->Kdim / 32;
  if (tiles >= 200 || on == 2) return 1;
  int split = (int)((320 + tiles - 1) / tiles);
  split = std::min(split, std::max(1, nk / 8));
  split = std::min(split, 8);
  return std::max(split, 1);
}

// BIGDL_CONV_P8: 0 = off, 1 (default) = the 256 x 256 phase-interleaved kernel on fast-K (Cs % 64 == 0) layers with
// Ncol >= 256 and Kdim >= 256, split over K when its grid would leave CUs idle; 2 = wherever it applies (tests).
// Returns 0 (not used), 1 (one pass) or the K split.
int g_conv_p8 = -1;
static int p8_pick(const ConvArgs* a) {
  if (g_conv_p8 < 0) {
    const char* e = getenv("BIGDL_CONV_P8");
    g_conv_p8 = e ? atoi(e) : 1;
  }
  const int on = g_conv_p8;
  const bool ktail = (a->Cs % 64) != 0 && a->ntaps == 1 && a->Cs % 8 == 0 && a->Kdim == a->Cs;   // p8_ktail()
  if (!on || a->out32 || ((a->Cs % 64) && !ktail) || (a->Ncol & 7) || (a->ldo & 7) || a->Kdim < 128) return 0;
  // auto: deep reductions only. Per layer (tools/conv_roofline.py, ResNet-50 b256) the one-workgroup-per-CU tile wins
  // from K = 1024 up (3x3 over 256 channels 101 -> 86 us) and loses below, where its prologue / epilogue are not
  // hidden by a co-resident workgroup (1x1 512 -> 1024 stride 2: 103 -> 147 us)
  if (on == 1 && (a->Ncol < 256 || a->Kdim < 1024)) return 0;
  const long tiles = (long)((a->M + 255) / 256) * ((a->Ncol + 255) / 256);
  const int nk = a->Kdim / 64;
  if (tiles >= 160) return 1;
  // split-K measured slower than the 256 x 128 deep-K kernel on the small ResNet grids (12544 x 512, K 4608:
  // 452 vs 544 TF/s, tools/gemm_ceiling.py): auto mode leaves grids under 160 tiles to the other kernels
  if (on == 1) return 0;
  int split = (int)((256 + tiles - 1) / tiles);
  split = std::min(split, std::max(1, nk / 4));
  split = std::min(split, 8);
  return std::max(split, 1);
}

// BIGDL_CONV_SK: stream-K for the 256 x 256 P8 kernel. 0 (default): off — it measured slower than the plain P8
// grid on every ResNet-50 layer its rule selects (profiles/r5_stream_k_ab.txt); 1 = on grids that leave CUs idle (a
// plain grid of tiles fills < 85 % of its last dispatch round) with deep reductions (Kdim >= BIGDL_CONV_SK_K, default
// 1024); 2 = wherever the P8 kernel applies (tests). Returns the (tile, segment) slots per tile, 0 when not used.
int g_conv_sk = -1;
int conv_impl();
static int sk_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}
static int sk_pick(const ConvArgs* a) {
  if (g_conv_sk < 0) {
    const char* e = getenv("BIGDL_CONV_SK");
    g_conv_sk = e ? atoi(e) : 0;
  }
  static const int kmin = [] { const char* e = getenv("BIGDL_CONV_SK_K"); return e ? atoi(e) : 1024; }();
  if (!g_conv_sk || conv_impl() != 1 || a->out32 || (a->Cs % 64) || (a->Ncol & 7) || (a->ldo & 7)) return 0;
  if (g_conv_p8 == 0) return 0;
  if (g_conv_sk == 1 && (a->Ncol < 256 || a->Kdim < kmin)) return 0;
  const long tiles = (long)((a->M + 255) / 256) * ((a->Ncol + 255) / 256);
  const int G = sk_cus();
  const int nk = a->Kdim / 64;
  const double eff = (double)tiles / (double)(((tiles + G - 1) / G) * G);
  if (g_conv_sk == 1 && eff >= 0.85) return 0;
  const long q = (tiles * nk) / G;
  if (q < 4) return 0;                      // ranges too short for the pipeline
  return (int)(nk / q + 2);
}

template <int BN, int NS, int BM = 128>
void launch_nt_g4(const ConvArgs& a, hipStream_t st) {
  const int nwg = ((a.M + BM - 1) / BM) * ((a.Ncol + BN - 1) / BN);
  static const int abn = [] { const char* e = getenv("BIGDL_G4_ABN"); return e ? atoi(e) : 0; }();
  if (abn && a.pre && BM == 128 && NS == 3 && a.Cs % 32 == 0)
    conv_nt_g4_kernel<BN, NS, true, BM, 1><<<dim3(nwg), dim3(256), 0, st>>>(a);
  else if (a.Cs % 32 == 0) conv_nt_g4_kernel<BN, NS, true, BM><<<dim3(nwg), dim3(256), 0, st>>>(a);
  else conv_nt_g4_kernel<BN, NS, false, BM><<<dim3(nwg), dim3(256), 0, st>>>(a);
}

// BIGDL_CONV_G4 (default 3): 0 = off, 4 = 4-stage (2 workgroups per CU), 3 = 3-stage (3 per CU) deep-pipelined 128-row kernel
// in place of the 2-stage LDS-DMA kernel on fast-K (Cs % 32 == 0), aligned-output layers; 5 = the 3-stage kernel
// also on the deep-K small-grid layers that otherwise take the 256-row 8-wave kernel; 6 = as 3, with the 256 x 128 tile
// for Ncol > 64 wherever its grid still gives every CU two workgroups; 7 = as 3, with the 256 x 128 tile always
// for Ncol > 64 (tests)
int g_conv_g4 = -1;
static int g4_pick() {
  if (g_conv_g4 < 0) {
    const char* e = getenv("BIGDL_CONV_G4");
    g_conv_g4 = e ? atoi(e) : 3;   // 3-stage default: ResNet-50 b256 27.35 -> 26.48 ms/step (profiles/r3_conv_g4_ab.txt)
  }
  return g_conv_g4;
}

// BIGDL_CONV_G4_SLOWK (default 1): the multi-stage kernel also for Cs % 32 != 0 (per-lane taps)
static bool g4_slowk() {
  static const int v = [] { const char* e = getenv("BIGDL_CONV_G4_SLOWK"); return e ? atoi(e) : 1; }();
  return v != 0;
}

// BIGDL_CONV_SHORTK (default 0): the two-stage, 4-workgroups-per-CU variant of the 128 x 64 multi-stage kernel when
// Kdim <= 64 and Ncol <= 64. Measured neutral on ResNet-50 b256 training (25.78 / 25.89 vs 25.81 / 25.91 ms,
// profiles/r4_shortk_ab.txt)
int g_conv_shortk = -1;
static bool conv_shortk() {
  if (g_conv_shortk < 0) {
    const char* e = getenv("BIGDL_CONV_SHORTK");
    g_conv_shortk = e ? atoi(e) : 0;
  }
  return g_conv_shortk != 0;
}

// BIGDL_CONV_S1 (default 2): the streaming 1x1 kernel (conv_nt_s1_kernel) wherever it applies, Kdim 64 / 128 / 256;
// 1 = Kdim 64 / 128 only (round 5; the 256-deep form runs one workgroup per CU with 128 weight VGPRs per wave:
// ResNet-50 22.62 -> 22.31 ms/step interleaved A/B, profiles/r6_iteration_log.txt); 0 = off (A/B)
int g_conv_s1 = -1;
static bool s1_applies(const ConvArgs* a) {
  if (g_conv_s1 < 0) {
    const char* e = getenv("BIGDL_CONV_S1");
    g_conv_s1 = e ? atoi(e) : 2;
  }
  if (!g_conv_s1 || a->out32 || !a->ident_out || a->ntaps != 1 || a->tap_h[0] || a->tap_w[0] || a->tap_k[0]) return false;
  if (a->mul_h != 1 || a->mul_w != 1 || a->Hs != a->OH || a->Ws != a->OW) return false;
  // BIGDL_CONV_S1 = 2 also takes Kdim 256 (128 VGPRs of weights per wave, 16-pixel wave tiles); 3 = Kdim 256 only
  // without the extended epilogue (addend / consumer-BN reduction: data gradients stay on the tile kernels)
  const bool ext = a->addend != nullptr || (a->bnred != nullptr && a->stats == nullptr);
  if ((a->Kdim != 64 && a->Kdim != 128 && !(a->Kdim == 256 && (g_conv_s1 == 2 || (g_conv_s1 == 3 && !ext)))) ||
      a->Cs != a->Kdim || (a->Ncol % 64) || (a->ldo % 8) || (a->ldw % 8))
    return false;
  // the epilogue operands go through 32-bit buffer offsets (bytes of an [M][ldo] bf16 tensor, below the OOB offset)
  if (((size_t)(a->M - 1) * a->ldo + a->Ncol) * 2 >= 0x7ff00000u) return false;
  // the consumer-BN ReLU mask as a bf16 z tensor (BIGDL_BN_ZMASK=0) is left to the tile kernels
  if (a->bnred && !a->stats && a->bnz && !a->bnzm) return false;
  // a BN applied on load (ConvArgs::pre) only with the forward epilogues (bias, statistics, ReLU; no addend)
  if (a->pre && (a->addend || (a->bnred && !a->stats))) return false;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return al(a->src) && al(a->wt) && al(a->out) && al(a->addend) && al(a->bnx) && al(a->bnz);
}

template <int K, int CG, int BMW, bool F32T, bool EXT, bool PRE = false>
void launch_s1(const ConvArgs& a, hipStream_t st) {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const int nchb = a.Ncol / (64 * CG);
  const int tiles = (a.M + BMW * (4 / CG) - 1) / (BMW * (4 / CG));
  constexpr int occ = K >= 256 ? 1 : 2;            // workgroups per CU (K = 256: 128 weight VGPRs per wave)
  int per = std::max(1, (occ * cus) / nchb);
  per = std::min(per, tiles);
  conv_nt_s1_kernel<K, CG, BMW, F32T, EXT, PRE><<<dim3(per * nchb), dim3(256), 0, st>>>(a);
}

template <int K, int CG>
void launch_s1_cg(const ConvArgs& a, hipStream_t st) {
  const bool ext = a.addend != nullptr || (a.bnred != nullptr && a.stats == nullptr);
  const bool f32t = ext || a.bias != nullptr;
  if constexpr (K == 256) {       // 128 VGPRs of weights per wave: 16-pixel wave tiles in every variant
    if (a.pre && f32t) launch_s1<K, CG, 16, true, false, true>(a, st);
    else if (a.pre) launch_s1<K, CG, 16, false, false, true>(a, st);
    else if (ext) launch_s1<K, CG, 16, true, true>(a, st);
    else if (f32t) launch_s1<K, CG, 16, true, false>(a, st);
    else launch_s1<K, CG, 16, false, false>(a, st);
  } else {
  constexpr int BW = K == 64 ? 64 : 32;            // pixels per wave tile (ubench: 64 / 32 best at K 64 / 128)
  // s1_applies: no bias / addend / BN reduction with pre; 32-pixel waves (the 64-pixel K = 64 tile spilled)
  if (a.pre && f32t) launch_s1<K, CG, BW / 2, true, false, true>(a, st);     // + bias (ResNet convs carry one)
  else if (a.pre) launch_s1<K, CG, 32, false, false, true>(a, st);
  else if (ext) launch_s1<K, CG, BW / 2, true, true>(a, st);
  else if (f32t) launch_s1<K, CG, BW / 2, true, false>(a, st);
  else launch_s1<K, CG, BW, false, false>(a, st);
  }
}

static void launch_s1_any(const ConvArgs& a, hipStream_t st) {
  const int cg = (a.Ncol % 256 == 0) ? 4 : (a.Ncol % 128 == 0) ? 2 : 1;
  if (a.Kdim == 64) {
    if (cg == 4) launch_s1_cg<64, 4>(a, st);
    else if (cg == 2) launch_s1_cg<64, 2>(a, st);
    else launch_s1_cg<64, 1>(a, st);
  } else if (a.Kdim == 128) {
    if (cg == 4) launch_s1_cg<128, 4>(a, st);
    else if (cg == 2) launch_s1_cg<128, 2>(a, st);
    else launch_s1_cg<128, 1>(a, st);
  } else {
    if (cg == 4) launch_s1_cg<256, 4>(a, st);
    else if (cg == 2) launch_s1_cg<256, 2>(a, st);
    else launch_s1_cg<256, 1>(a, st);
  }
}

int g_conv_impl = -1;
int conv_impl() {
  if (g_conv_impl < 0) {
    const char* e = getenv("BIGDL_CONV_IMPL");
    g_conv_impl = e ? atoi(e) : 1;
  }
  return g_conv_impl;
}

}  // namespace

extern "C" {

void bigdl_set_conv_impl(int impl) { g_conv_impl = impl; }
void bigdl_set_conv_s1(int v) { g_conv_s1 = v; }
void bigdl_set_conv_sk(int v) { g_conv_sk = v; }
void bigdl_set_conv_g4(int v) { g_conv_g4 = v; }
void bigdl_set_conv_shortk(int v) { g_conv_shortk = v; }
int g_wgrad_p8 = -1;
void bigdl_set_conv_p8(int v) { g_conv_p8 = v; }
void bigdl_set_wgrad_p8(int v) { g_wgrad_p8 = v; }
int bigdl_get_conv_g4() { return g4_pick(); }
int bigdl_get_conv_impl() { return conv_impl(); }

// Forward or data-gradient implicit GEMM. Returns 0 on success, negative on unsupported shapes.
long bigdl_conv_nt_plan(ConvArgs* a) {
  a->ksplit = 0;
  if (a->Cs % 8 != 0 || a->M <= 0 || conv_impl() < 1) return 0;
  if (a->pstride > 0 && a->pstride != a->Cs) return 0;   // overlapping windows: g4 only, no split-K
  if (conv_impl() == 1 && s1_applies(a)) return 0;
  if (conv_impl() == 1 && bigdl_conv_halo_applies(a)) return 0;
  if (conv_impl() == 1 && bigdl_stem_fwd_applies(a)) return 0;
  if (g_conv_p8 < 0) (void)p8_pick(a);      // reads BIGDL_CONV_P8 once
  const int sk = sk_pick(a);
  if (sk > 0) {
    a->ksplit = -sk;                        // stream-K: slots per tile (negative marks the mode)
    const long tiles = (long)((a->M + 255) / 256) * ((a->Ncol + 255) / 256);
    return tiles * sk * 65536L + tiles;     // fp32 slots + one ticket word per tile
  }
  const int p8 = conv_impl() == 1 ? p8_pick(a) : 0;
  if (p8 > 1) {
    a->ksplit = p8;
    return (long)p8 * a->M * a->Ncol;
  }
  if (p8 == 1) return 0;
  const int k = w8_pick(a);
  if (k > 1) {
    a->ksplit = k;
    return (long)k * a->M * a->Ncol;
  }
  return 0;
}

int bigdl_conv_pre_applies(const ConvArgs* a) {
  if (a->Cs % 8 != 0 || a->Kdim != a->ntaps * a->Cs || a->M <= 0 || a->pstride > 0 || conv_impl() != 1) return 0;
  if (bigdl_stem_fwd_applies(a)) return 0;
  return (s1_applies(a) || bigdl_conv_halo_applies(a)) ? 1 : 0;
}

int bigdl_conv_nt(const ConvArgs* a, hipStream_t st) {
  if (a->Cs % 8 != 0 || a->Kdim != a->ntaps * a->Cs || a->ntaps < 1 || a->ntaps > CONV_MAX_TAPS) return -1;
  if (a->pre) {     // a BN applied on load: only the kernels that implement it (the caller materialises otherwise)
    if (!bigdl_conv_pre_applies(a)) return -5;
    if (s1_applies(a)) launch_s1_any(*a, st);
    else if (bigdl_conv_halo(a, st) != 0) return -5;
    HIP_LAUNCH_CHECK();
    return 0;
  }
  // the BN-backward reduction lives in the LDS-transposed epilogue only
  if (a->bnred && (a->stats || a->bnx == nullptr || a->bnmean == nullptr || (a->Ncol & 7) || (a->ldo & 7))) return -2;
  // fp32 output exists in the LDS-transposed epilogue only (aligned columns), without stats / BN / ReLU / addend
  if (a->out32 && ((a->Ncol & 7) || (a->ldo & 7) || a->stats || a->bnred || a->relu || a->addend)) return -3;
  if (a->M <= 0) return 0;
  const bool fastk = (a->Cs % BK) == 0;
  const int impl = conv_impl();
  if (impl == 1 && bigdl_stem_fwd_applies(a) && bigdl_stem_fwd(a, st) == 0) {
    HIP_LAUNCH_CHECK();
    return 0;
  }
  if (a->pstride > 0 && a->pstride != a->Cs) {   // overlapping-window source: the g4 kernel is the one that reads it
    if ((a->Ncol & 7) || (a->ldo & 7) || a->out32 || a->ws || a->bnred || !(fastk || a->Kdim % 8 == 0)) return -4;
    if (a->Ncol <= 64) launch_nt_g4<64, 3>(*a, st);
    else launch_nt_g4<128, 3>(*a, st);
    HIP_LAUNCH_CHECK();
    return 0;
  }
  if (impl == 1 && s1_applies(a)) {
    launch_s1_any(*a, st);
    HIP_LAUNCH_CHECK();
    return 0;
  }
  if (impl == 1 && bigdl_conv_halo_applies(a) && bigdl_conv_halo(a, st) == 0) {
    HIP_LAUNCH_CHECK();
    return 0;
  }
  if (a->ksplit < 0 && a->ws != nullptr) {  // stream-K P8 (bigdl_conv_nt_plan)
    ConvArgs b = *a;
    b.ksplit = -a->ksplit;
    const long tiles = (long)((a->M + 255) / 256) * ((a->Ncol + 255) / 256);
    bigdl_fill_bytes(b.ws + tiles * b.ksplit * 65536L, 0, tiles * 4, st);   // tickets (a kernel: graph-safe)
    const dim3 grid((unsigned)std::min<long>(sk_cus(), tiles * (a->Kdim / 64)));
    conv_nt_p8_kernel<false, 0, true><<<grid, dim3(512), 0, st>>>(b);
    HIP_LAUNCH_CHECK();
    return 0;
  }
  const long p3_tiles = (long)((a->M + 255) / 256) * ((a->Ncol + 127) / 128);
  const long tiles128 = (long)((a->M + 127) / 128) * ((a->Ncol + (a->Ncol <= 64 ? 63 : 127)) / (a->Ncol <= 64 ? 64 : 128));
  const bool aligned_out = (a->Ncol & 7) == 0 && (a->ldo & 7) == 0;   // the persistent kernel has no fallback epilogue
  // deep-K layers on small pixel grids (ResNet stages 4-5: <= 50k output pixels, K >= 1024) run faster on the
  // 8-wave deep-pipelined kernel (tools/bench_conv.py, impl 1 vs 2); BIGDL_CONV_P3AUTO=0 keeps them on impl 1
  static const bool p3auto = [] { const char* e = getenv("BIGDL_CONV_P3AUTO"); return e ? atoi(e) != 0 : true; }();
  const bool p3_pick = impl == 2 || (impl == 1 && p3auto && a->M <= 50176 && a->Kdim >= 1024);
  const int p8 = impl == 1 ? p8_pick(a) : 0;
  const int w8 = (impl == 1 && p8 == 0) ? w8_pick(a) : 0;
  // K tail (one tap, Cs % 64 != 0, e.g. a 10000-word vocabulary projection's data gradient): granules past Kdim zero
  const bool p8_ktail = (a->Cs % 64) != 0;
  if (p8 > 1 && a->ksplit == p8 && a->ws != nullptr) {
    const int nwg = ((a->M + 255) / 256) * ((a->Ncol + 255) / 256);
    if (p8_ktail) conv_nt_p8_kernel<true, 64><<<dim3(nwg, p8), dim3(512), 0, st>>>(*a);
    else conv_nt_p8_kernel<true><<<dim3(nwg, p8), dim3(512), 0, st>>>(*a);
    long rpb = 0;
    const dim3 grid = splitk_grid(a->M, a->Ncol, &rpb);
    conv_splitk_epilogue_kernel<<<grid, dim3(256), 0, st>>>(*a, rpb);
  } else if (p8 == 1) {
    const int nwg = ((a->M + 255) / 256) * ((a->Ncol + 255) / 256);
    static const int abl = [] { const char* e = getenv("BIGDL_P8_ABL"); return e ? atoi(e) : 0; }();
    switch (p8_ktail ? 64 : abl) {
      case 64: conv_nt_p8_kernel<false, 64><<<dim3(nwg), dim3(512), 0, st>>>(*a); break;
      case 1: conv_nt_p8_kernel<false, 1><<<dim3(nwg), dim3(512), 0, st>>>(*a); break;
      case 2: conv_nt_p8_kernel<false, 2><<<dim3(nwg), dim3(512), 0, st>>>(*a); break;
      case 4: conv_nt_p8_kernel<false, 4><<<dim3(nwg), dim3(512), 0, st>>>(*a); break;
      case 8: conv_nt_p8_kernel<false, 8><<<dim3(nwg), dim3(512), 0, st>>>(*a); break;
      case 16: conv_nt_p8_kernel<false, 16><<<dim3(nwg), dim3(512), 0, st>>>(*a); break;
      case 32: conv_nt_p8_kernel<false, 32><<<dim3(nwg), dim3(512), 0, st>>>(*a); break;
      case 10: conv_nt_p8_kernel<false, 10><<<dim3(nwg), dim3(512), 0, st>>>(*a); break;
      default: conv_nt_p8_kernel<false><<<dim3(nwg), dim3(512), 0, st>>>(*a);
    }
  } else if (w8 > 1 && a->ksplit == w8 && a->ws != nullptr) {
    const int nwg = ((a->M + 255) / 256) * ((a->Ncol + 255) / 256);
    conv_nt_w8_kernel<true><<<dim3(nwg, w8), dim3(512), 0, st>>>(*a);
    long rpb = 0;
    const dim3 grid = splitk_grid(a->M, a->Ncol, &rpb);
    conv_splitk_epilogue_kernel<<<grid, dim3(256), 0, st>>>(*a, rpb);
  } else if (w8 == 1) {
    const int nwg = ((a->M + 255) / 256) * ((a->Ncol + 255) / 256);
    conv_nt_w8_kernel<false><<<dim3(nwg), dim3(512), 0, st>>>(*a);
  } else if (impl == 1 && g4_pick() && aligned_out && (a->Cs % 32 == 0 || (g4_slowk() && a->Kdim % 8 == 0)) &&
             (g4_pick() == 5 || !(p3_pick && fastk && p3_tiles >= 256))) {
    const long tiles256 = (long)((a->M + 255) / 256) * ((a->Ncol + 127) / 128);
    if (a->Ncol > 64 && (g4_pick() == 7 || (g4_pick() == 6 && tiles256 >= 512))) {
      launch_nt_g4<128, 3, 256>(*a, st);
    } else if (conv_shortk() && fastk && a->Kdim <= 64 && a->Ncol <= 64) {
      launch_nt_g4<64, 2>(*a, st);   // (the 128-wide tile needs 168 VGPRs: no fourth workgroup)
    } else if (g4_pick() != 4) {
      if (a->Ncol <= 64) launch_nt_g4<64, 3>(*a, st);
      else launch_nt_g4<128, 3>(*a, st);
    } else {
      if (a->Ncol <= 64) launch_nt_g4<64, 4>(*a, st);
      else launch_nt_g4<128, 4>(*a, st);
    }
  } else if (fastk && p3_pick && p3_tiles >= 256) {
    if (a->Ncol <= 64) launch_nt_p3<64, 8, 1>(*a, st);
    else launch_nt_p3<128, 4, 2>(*a, st);
  } else if (fastk && impl == 3 && aligned_out && tiles128 > 2 * 256) {
    if (a->Ncol <= 64) launch_nt_pers<128, 64, 2>(*a, st);
    else launch_nt_pers<128, 128, 2>(*a, st);
  } else if (fastk && impl >= 1 && a->Kdim == BK && aligned_out && conv_onestage()) {
    if (a->Ncol <= 64) launch_nt_glds<128, 64, 2, true, 1>(*a, st);
    else launch_nt_glds<128, 128, 2, true, 1>(*a, st);
  } else if (fastk && impl >= 1) {
    if (a->Ncol <= 64) launch_nt_glds<128, 64, 2>(*a, st);
    else launch_nt_glds<128, 128, 2>(*a, st);
  } else if (!fastk && impl >= 1 && glds_slowk()) {
    if (a->Ncol <= 64) launch_nt_glds<128, 64, 2, false>(*a, st);
    else launch_nt_glds<128, 128, 2, false>(*a, st);
  } else if (a->Ncol <= 64) {
    launch_nt<128, 64, 2>(*a, fastk, st);
  } else {
    launch_nt<128, 128, 2>(*a, fastk, st);
  }
  HIP_LAUNCH_CHECK();
  return 0;
}

// 64-wide output-channel layers with a deep reduction (stem 7x7, 3x3 over 64 channels) run half-empty 128x128
// tiles; the register-staged atomic kernel is faster there (measured per layer, profiles/r1_ab_wgrad.txt)
static bool wgrad_prefers_atomic(const WgradArgs* a) {
  // BIGDL_WGRAD_ATOMIC: 1 (default) this rule, 0 never, 2 always (per-layer A/B runs); never in deterministic mode
  static const int on = [] { const char* e = getenv("BIGDL_WGRAD_ATOMIC"); return e ? atoi(e) : 1; }();
  if (bigdl_deterministic()) return false;
  return on == 2 || (on == 1 && a->Ncol <= 64 && a->Kdim > 256);
}

int g_wgrad_g3 = -1;
// BIGDL_WGRAD_G3=1: the 3-stage counted-vmcnt weight-gradient kernel in place of the 2-stage one
static bool wgrad_g3() {
  if (g_wgrad_g3 < 0) {
    const char* e = getenv("BIGDL_WGRAD_G3");
    g_wgrad_g3 = e ? atoi(e) : 0;
  }
  return g_wgrad_g3 != 0;
}
void bigdl_set_wgrad_g3(int v) { g_wgrad_g3 = v; }
int bigdl_get_wgrad_g3() { return wgrad_g3() ? 1 : 0; }

// BIGDL_WGRAD_P8: 1 (default) = conv_wgrad_p8_kernel where it measured faster (below), 2 = on every layer with
// Ncol >= 256 and Kdim >= 256 (tests / A/B), 0 = off.
// Returns its pixel split (>= 1) or 0 when it does not apply; sets m_per_split.
static int p8w_pick(WgradArgs* a) {
  if (g_wgrad_p8 < 0) {
    const char* e = getenv("BIGDL_WGRAD_P8");
    g_wgrad_p8 = e ? atoi(e) : 1;
  }
  if (!g_wgrad_p8 || conv_impl() < 1 || a->Ncol < 256 || a->Kdim < 256 || (a->Cs % 8) ||
      (a->Ncol % 8) || (a->Kdim % 8) || a->M <= 0)
    return 0;
  const long tiles = (long)((a->Ncol + 255) / 256) * ((a->Kdim + 255) / 256);
  // Default: GEMM-shaped (1 x 1) weight gradients with >= 32 output tiles — Linear / LSTM projections, where it reads
  // dy and x in place (transposed LDS reads) instead of the two operand transposes of the NT GEMM path. In isolation
  // it also wins on ResNet-50's 3x3 layers with Kdim >= 2304 (-15..-25 %, profiles/r4_wgrad_p8_layers.txt), but
  // inside the training step its 128 KB-LDS workgroups on the weight-gradient side stream cost the concurrent data-
  // gradient chain more than they save (26.05 vs 25.72 ms/step, profiles/r4_wgrad_p8_ab.txt); on 1x1 layers with few
  // tiles its deep pixel split turns into fp32 partial traffic
  if (g_wgrad_p8 == 1 && !(a->R * a->S == 1 && tiles >= 32)) return 0;
  const long steps = (a->M + 63) / 64;
  // pixel split: one workgroup per CU, so pick the split (<= 8, >= 8 pixel steps each, <= 256 MB of fp32 partials)
  // whose grid fills its last dispatch round best (vocab 160 tiles: 2 splits = 320 workgroups = 1.25 rounds ran at
  // 326 TF/s; 3 = 480 fills 1.9 rounds)
  const long cap = std::max(1L, (256L << 20) / ((long)a->Ncol * a->Kdim * 4));
  const long smax = std::max(1L, std::min({8L, steps / 8, cap}));
  long splits = 1;
  double best = 0.0;
  for (long sp = 1; sp <= smax; ++sp) {
    const long wgs = tiles * sp;
    const double eff = (double)wgs / (double)(((wgs + 255) / 256) * 256);
    if (eff > best + 0.02) { best = eff; splits = sp; }
  }
  long mps = (a->M + splits - 1) / splits;
  mps = (mps + 63) / 64 * 64;
  splits = (a->M + mps - 1) / mps;
  a->m_per_split = (int)mps;
  return (int)splits;
}

int bigdl_conv_wgrad_uses_p8(const WgradArgs* a_in) {
  WgradArgs a = *a_in;
  return p8w_pick(&a) > 0 ? 1 : 0;
}

long bigdl_conv_wgrad_plan(WgradArgs* a) {
  if (conv_impl() >= 1) {
    const long sw = bigdl_stem_wgrad_plan(a);
    if (sw > 0) {
      a->splits = -1;                        // the pair-view stem kernel (stem_fwd.hip)
      return sw;
    }
  }
  const int hs = bigdl_wgrad_halo_plan(a);
  if (hs > 0) {
    a->splits = hs;
    return hs > 1 ? (long)hs * a->Ncol * a->Kdim + (a->dbias ? (long)hs * a->Ncol : 0) : 0;
  }
  const int p8w = p8w_pick(a);
  if (p8w > 0) {
    a->splits = p8w;
    return p8w > 1 ? (long)p8w * a->Ncol * a->Kdim : 0;
  }
  const int tiles = ((a->Ncol + WT - 1) / WT) * ((a->Kdim + WT - 1) / WT);
  if (conv_impl() < 1 || wgrad_prefers_atomic(a)) { a->splits = 0; return 0; }
  // workspace split-K: ~2 workgroups per CU (512; the kernel runs beside the dgrad chain on the side stream, so
  // fewer splits = less partial traffic wins: 26.37 vs 26.62 ms/step, profiles/r3_wgrad_wgs_ab.txt), >= 4 LDS stages per split
  // (BIGDL_WGRAD_WGS overrides the workgroup target for A/B runs: fewer splits = fewer partials to reduce)
  static const int target = [] { const char* e = getenv("BIGDL_WGRAD_WGS"); return e ? atoi(e) : 512; }();
  int splits = (target + tiles - 1) / tiles;
  const int maxsplit = (a->M + 8 * WBM - 1) / (8 * WBM);
  if (splits > maxsplit) splits = maxsplit;
  if (splits < 1) splits = 1;
  int mps = (a->M + splits - 1) / splits;
  mps = (mps + WBM - 1) / WBM * WBM;
  splits = (a->M + mps - 1) / mps;
  a->m_per_split = mps;
  a->splits = splits;
  return splits > 1 ? (long)splits * a->Ncol * a->Kdim : 0;
}

static int conv_wgrad_impl(const WgradArgs* a_in, hipStream_t st);

// Deterministic mode: the split kernels add their bias partials with one atomic per split, so the bias gradient is
// taken out of them and summed by a one-row-block column sum (one atomic per channel); the weight gradient always
// goes through the workspace partials + fixed-order reduce (no multi-split atomics, see bigdl_conv_wgrad_plan).
int bigdl_conv_wgrad(const WgradArgs* a_in, hipStream_t st) {
  if (bigdl_deterministic() && a_in->dbias != nullptr && (a_in->ldy % 8) == 0) {
    WgradArgs b = *a_in;
    b.dbias = nullptr;
    const int rc = conv_wgrad_impl(&b, st);
    if (rc == 0) bigdl_colsum_bf16_ld(a_in->dy, a_in->dbias, a_in->M, a_in->Ncol, a_in->ldy, st, a_in->det_ws);
    return rc;
  }
  return conv_wgrad_impl(a_in, st);
}

static int conv_wgrad_impl(const WgradArgs* a_in, hipStream_t st) {
  WgradArgs a = *a_in;
  if (a.pre) {      // a BN applied on load: the halo kernel only (the binding materialises everything else)
    WgradArgs b = a;
    const int hs = bigdl_wgrad_halo_plan(&b);
    if (hs <= 0 || hs != a.splits || (hs > 1 && a.ws == nullptr)) return -6;
    b.splits = hs;
    b.ws = hs > 1 ? a.ws : nullptr;
    const int rc = bigdl_wgrad_halo(&b, st);
    HIP_LAUNCH_CHECK();
    return rc;
  }
  if (a.splits == -1 && a.ws != nullptr && bigdl_stem_wgrad_plan(&a) > 0) {
    const int rc = bigdl_stem_wgrad(&a, st);
    HIP_LAUNCH_CHECK();
    return rc;
  }
  if (a.Cs % 8 != 0 || a.Ncol % 8 != 0 || a.Kdim % 8 != 0) return -1;
  {
    WgradArgs b = a;
    const int hs = bigdl_wgrad_halo_plan(&b);
    if (hs > 0 && hs == a.splits && (hs == 1 || a.ws != nullptr)) {
      b.splits = hs;
      b.ws = hs > 1 ? a.ws : nullptr;
      if (bigdl_wgrad_halo(&b, st) == 0) {
        HIP_LAUNCH_CHECK();
        return 0;
      }
    }
  }
  {
    WgradArgs b = a;
    const int p8w = p8w_pick(&b);
    if (p8w > 0 && p8w == a.splits && (p8w == 1 || a.ws != nullptr)) {
      b.splits = p8w;
      b.ws = a.ws;
      const int tiles = ((a.Ncol + 255) / 256) * ((a.Kdim + 255) / 256);
      const bool direct = a.R == 1 && a.S == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 && a.pw == 0 && a.Hs == a.OH &&
                          a.Ws == a.OW;
      if (direct) conv_wgrad_p8_kernel<true><<<dim3(tiles, p8w), dim3(512), 0, st>>>(b);
      else conv_wgrad_p8_kernel<false><<<dim3(tiles, p8w), dim3(512), 0, st>>>(b);
      if (p8w > 1) {
        const long n4 = (long)a.Ncol * a.Kdim / 4;
        const int blocks = (int)std::min<long>((n4 + 255) / 256, 8192);
        if ((reinterpret_cast<uintptr_t>(a.dw) & 15) == 0) wgrad_reduce_kernel<true><<<dim3(blocks, 1), 256, 0, st>>>(a.ws, a.dw, n4, p8w);
        else wgrad_reduce_kernel<false><<<dim3(blocks, 1), 256, 0, st>>>(a.ws, a.dw, n4, p8w);
      }
      HIP_LAUNCH_CHECK();
      return 0;
    }
  }
  if (a.ws != nullptr && a.splits > 1 && conv_impl() >= 1) {
    const int tiles = ((a.Ncol + WT - 1) / WT) * ((a.Kdim + WT - 1) / WT);
    const int spad = (a.splits + 7) / 8 * 8;
    if (wgrad_g3()) conv_wgrad_g3_kernel<<<dim3(tiles * spad), dim3(256), 0, st>>>(a);
    else conv_wgrad_glds_kernel<<<dim3(tiles * spad), dim3(256), 0, st>>>(a);
    const long n4 = (long)a.Ncol * a.Kdim / 4;
    const int blocks = (int)std::min<long>((n4 + 255) / 256, 8192);
    // ~2048 reduce workgroups in total, >= 4 splits per group, <= 64-way atomic contention
    const int groups = (blocks >= 256 || bigdl_deterministic()) ? 1
                                                               : std::max(1, std::min({2048 / blocks, a.splits / 4, 64}));
    const dim3 rgrid(blocks, groups);
    if ((reinterpret_cast<uintptr_t>(a.dw) & 15) == 0) wgrad_reduce_kernel<true><<<rgrid, 256, 0, st>>>(a.ws, a.dw, n4, a.splits);
    else wgrad_reduce_kernel<false><<<rgrid, 256, 0, st>>>(a.ws, a.dw, n4, a.splits);
    HIP_LAUNCH_CHECK();
    return 0;
  }
  a.ws = nullptr;
  const int tiles = ((a.Ncol + WT - 1) / WT) * ((a.Kdim + WT - 1) / WT);
  // ~2 workgroups per CU in one dispatch wave; every split adds a full fp32 atomic pass over its
  // tile, so also cap the atomic traffic (splits x |dW| x 4 B) at ~32 MB (~25 us at the chip rate).
  int splits = (512 + tiles - 1) / tiles;
  const long tile_bytes = (long)tiles * WT * WT * 4;
  static const long atomic_mb = [] { const char* e = getenv("BIGDL_WGRAD_ATOMIC_MB"); return e ? atol(e) : 32l; }();
  const int cap_atomic = (int)((atomic_mb << 20) / tile_bytes);
  if (splits > cap_atomic) splits = cap_atomic;
  const int maxsplit = (a.M + 4 * WBM - 1) / (4 * WBM);   // >= 4 LDS stages per split
  if (splits > maxsplit) splits = maxsplit;
  if (splits < 1 || bigdl_deterministic()) splits = 1;   // det: no workspace given -> one split, one atomic each
  int mps = (a.M + splits - 1) / splits;
  mps = (mps + WBM - 1) / WBM * WBM;
  splits = (a.M + mps - 1) / mps;
  a.m_per_split = mps;
  a.splits = splits;
  if (conv_impl() >= 1 && !wgrad_prefers_atomic(&a) && wgrad_g3())
    conv_wgrad_g3_kernel<<<dim3(tiles * ((splits + 7) / 8 * 8)), dim3(256), 0, st>>>(a);
  else if (conv_impl() >= 1 && !wgrad_prefers_atomic(&a))
    conv_wgrad_glds_kernel<<<dim3(tiles * ((splits + 7) / 8 * 8)), dim3(256), 0, st>>>(a);
  else conv_wgrad_kernel<<<dim3(tiles, splits), dim3(256), 0, st>>>(a);
  HIP_LAUNCH_CHECK();
  return 0;
}

void bigdl_transpose_krsc(const bf16_t* w, bf16_t* wt, int K, int RS, int C, hipStream_t st) {
  if (RS > 65535) return;
  if (K % 8 == 0 && C % 8 == 0 && (long)K * C >= (1L << 20) && (((uintptr_t)w | (uintptr_t)wt) & 15) == 0)
    transpose_krsc_v8_kernel<<<dim3((C + 63) / 64, (K + 63) / 64, RS), 256, 0, st>>>(w, wt, K, RS, C);
  else
    transpose_krsc_kernel<<<dim3((C + 31) / 32, (K + 31) / 32, RS), 256, 0, st>>>(w, wt, K, RS, C);
  HIP_LAUNCH_CHECK();
}

void bigdl_transpose_krsc_batched(const long* desc, int n, int total_tiles, hipStream_t st) {
  if (n <= 0 || total_tiles <= 0) return;
  transpose_krsc_batched_kernel<<<dim3(total_tiles), 256, 0, st>>>(desc, n);
  HIP_LAUNCH_CHECK();
}

}  // extern "C"
