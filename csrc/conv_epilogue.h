// Coalescing fused epilogue shared by the NT implicit-GEMM kernels (conv_igemm.hip, conv_halo.hip).
#pragma once
#include "common.h"
#include "kernels.h"

namespace {

// Output row of GEMM row m (-1: no output row). The default is the dense implicit-GEMM mapping: m is an output pixel
// (image, oh, ow) placed by (OHo, OWo, omul, ooff); conv_halo.hip maps its padded "virtual pixels" instead.
struct GemmRowMap {
  __device__ __forceinline__ long operator()(const ConvArgs& a, int m) const {
    if (m >= a.M) return -1;
    if (a.ident_out) return m;
    const int ohw = a.OH * a.OW;
    const int nb = m / ohw, rem = m - nb * ohw;
    const int oh = rem / a.OW, ow = rem - oh * a.OW;
    return ((long)nb * a.OHo + oh * a.omul_h + a.ooff_h) * a.OWo + ow * a.omul_w + a.ooff_w;
  }
};

// Coalescing epilogue (Ncol % 8 == 0, ldo % 8 == 0): each wave parks its fp32 TM x TN tile in its own
// slice of the (now idle) staging LDS — [pixel][channel], 16-byte granules XOR-swizzled by pixel so both
// the 16-byte writes (lanes of 16 consecutive pixels) and the 2 x 16-byte reads (lanes along a pixel row)
// are conflict-free — then re-reads it row-wise: a lane owns 8 channels of one pixel, so every store is
// 16 B and one wave instruction writes 64/(TN/8) whole pixel rows of TN channels. bias / addend / ReLU /
// BN statistics are applied in the row phase (the addend is read with the same 16-byte coalesced pattern).
// PAIR > 0 (= WGN * SL: every wave of the workgroup calls this with its slice at wave * SL, wave = wm * WGN + wn, and
// NWM pixel-row waves per channel range): the BN statistics / consumer-BN sums of all waves are combined through LDS
// and committed by the whole workgroup, one full-wave atomic per value (see the commit below).
template <int MI, int NI, int TM, int TN, int NH = 1, int PAIR = 0, int NWM = 2, class RowMap = GemmRowMap>
__device__ __forceinline__ void nt_epilogue_lds(const ConvArgs& a, v4f (&acc)[MI][NI], int mbase, int nbase,
                                                int lane, int bid, float* wl, int wm = 0, RowMap rowmap = {}) {
  constexpr int GR = TN / 4;            // 16-byte fp32 granules per pixel row
  constexpr int LPR = TN / 8;           // lanes per pixel row in the read phase
  constexpr int PPI = 64 / LPR;         // pixels per read instruction
  static_assert(TN % 8 == 0 && 64 % LPR == 0, "tile");
  auto gpos = [](int p, int g) { return (p * GR + (g ^ (p & (GR - 1)))) * 4; };
  const int q = lane % LPR;              // this lane's 8-channel group within the wave tile
  const int n = nbase + q * 8;
  const bool nok = n < a.Ncol;
  float bs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bs[e] = (a.bias && nok) ? a.bias[n + e] : 0.f;
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  float bmu[8], bsc[8], bsh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const bool on = a.bnred && !a.stats && nok;
    bmu[e] = on ? a.bnmean[n + e] : 0.f;
    bsc[e] = (on && a.bnaff) ? a.bnaff[n + e] : 0.f;
    bsh[e] = (on && a.bnaff) ? a.bnaff[a.Ncol + n + e] : 0.f;
  }
  // NH > 1: the accumulator tile goes through LDS in NH row chunks, so the wave slice is TM/NH x TN floats
  constexpr int NR = TM / PPI;
  constexpr int MIH = MI / NH, NRH = NR / NH;
  static_assert(MI % NH == 0 && NR % NH == 0, "row chunks");
  const bool bnw = a.bnred && !a.stats;
#pragma unroll
  for (int h = 0; h < NH; ++h) {
  // Phase 1: every global read of the chunk (addend, consumer-BN x / z) is issued before its first store:
  // `out` may alias them as far as the compiler knows, so loads left inside the store loop would be serialised
  // one round trip per row group.
  long orows[NRH];
  v4u pad[NRH], px[NRH], pz[NRH];
#pragma unroll
  for (int rr = 0; rr < NRH; ++rr) {
    const int m = mbase + (h * NRH + rr) * PPI + lane / LPR;
    const long orow = nok ? rowmap(a, m) : -1;
    orows[rr] = orow;
    const size_t off = (size_t)(orow < 0 ? 0 : orow) * a.ldo + n;
    pad[rr] = v4u{0u, 0u, 0u, 0u};
    px[rr] = v4u{0u, 0u, 0u, 0u};
    pz[rr] = v4u{0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
    if (orow >= 0) {
      if (a.addend) {
        pad[rr] = *reinterpret_cast<const v4u*>(a.addend + off);
        if (a.addzm) pad[rr] &= mask8_to_and(a.addzm[off >> 3]);
      }
      if (bnw) {
        px[rr] = *reinterpret_cast<const v4u*>(a.bnx + off);
        if (a.bnzm) pz[rr] = mask8_to_bf(a.bnzm[off >> 3]);
        else if (a.bnz) pz[rr] = *reinterpret_cast<const v4u*>(a.bnz + off);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < MIH; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int p = i * 16 + (lane & 15);
      const int g = j * 4 + (lane >> 4);
      *reinterpret_cast<v4f*>(wl + gpos(p, g)) = acc[h * MIH + i][j];
    }
  __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): this wave's LDS writes landed (wave-private slice)
#pragma unroll
  for (int rr = 0; rr < NRH; ++rr) {
    const int r = rr;
    const int p = rr * PPI + lane / LPR;
    const v4f lo = *reinterpret_cast<const v4f*>(wl + gpos(p, 2 * q));
    const v4f hi = *reinterpret_cast<const v4f*>(wl + gpos(p, 2 * q + 1));
    const long orow = orows[r];
    if (orow >= 0 && a.out32) {        // fp32 GEMM output (+ bias), optionally accumulated: 2 x 16-byte stores
      float* o32 = a.out32 + (size_t)orow * a.ldo + n;
      v4f p0 = {lo[0] + bs[0], lo[1] + bs[1], lo[2] + bs[2], lo[3] + bs[3]};
      v4f p1 = {hi[0] + bs[4], hi[1] + bs[5], hi[2] + bs[6], hi[3] + bs[7]};
      if (a.accum32) {
        p0 += *reinterpret_cast<const v4f*>(o32);
        p1 += *reinterpret_cast<const v4f*>(o32 + 4);
      }
      *reinterpret_cast<v4f*>(o32) = p0;
      *reinterpret_cast<v4f*>(o32 + 4) = p1;
      continue;
    }
    if (orow >= 0) {
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if (a.addend) {
#pragma unroll
        for (int e = 0; e < 4; ++e) { v[2 * e] += lo_bf(pad[r][e]); v[2 * e + 1] += hi_bf(pad[r][e]); }
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
        // consumer-BN backward reduction on the rounded gradient (what bn_bwd_reduce would read back)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float d0 = lo_bf(o[e]), d1 = hi_bf(o[e]);
          const float x0 = lo_bf(px[r][e]), x1 = hi_bf(px[r][e]);
          if (a.bnz || a.bnzm) {
            if (!(lo_bf(pz[r][e]) > 0.f)) d0 = 0.f;
            if (!(hi_bf(pz[r][e]) > 0.f)) d1 = 0.f;
          } else if (a.bnaff) {
            if (!(x0 * bsc[2 * e] + bsh[2 * e] > 0.f)) d0 = 0.f;
            if (!(x1 * bsc[2 * e + 1] + bsh[2 * e + 1] > 0.f)) d1 = 0.f;
          }
          s1[2 * e] += d0; s2[2 * e] += d0 * (x0 - bmu[2 * e]);
          s1[2 * e + 1] += d1; s2[2 * e + 1] += d1 * (x1 - bmu[2 * e + 1]);
        }
      }
      *reinterpret_cast<v4u*>(a.out + (size_t)orow * a.ldo + n) = o;
    }
  }
  }
  float* const red = a.stats ? a.stats : a.bnred;
  if (red) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
      for (int o = LPR; o < 64; o <<= 1) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    }
    if constexpr (PAIR > 0) {
      // Workgroup commit: every wave parks its TN channels' sums in its own (consumed) slice, then the whole workgroup
      // adds the NWM pixel-row partials of each of its channels and issues ONE atomic per value, with full waves.
      // A memory-side float atomic costs ~50 ns per wave-instruction per CU whatever its lane count, so the former
      // 8-lane atomics (16 wave-instructions per wave) bounded statistics-heavy tiles such as the 7x7 stem.
      // Slices are laid out as wave * SL floats with wave = wm * WGN + wn (PAIR = WGN * SL).
      if (lane < LPR) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { wl[lane * 16 + e] = s1[e]; wl[lane * 16 + 8 + e] = s2[e]; }
      }
      __syncthreads();
      const int nwv = (int)(blockDim.x >> 6), wgn = nwv / NWM, sl = PAIR / wgn;
      const int wave = (int)(threadIdx.x >> 6), wn = wave % wgn;
      const float* base = wl - wave * sl;
      const int n0 = nbase - wn * TN, nv = wgn * TN;
      float* sp = red + (size_t)(bid & (BIGDL_STAT_SLOTS - 1)) * 2 * a.Ncol;
      for (int t = (int)threadIdx.x; t < 2 * nv; t += (int)blockDim.x) {
        const int which = t >= nv ? 1 : 0, c = t - which * nv, w2 = c / TN, cl = c - w2 * TN;
        float v = 0.f;
#pragma unroll
        for (int k = 0; k < NWM; ++k) v += base[(k * wgn + w2) * sl + (cl >> 3) * 16 + which * 8 + (cl & 7)];
        if (n0 + c < a.Ncol) atomicAdd(sp + which * a.Ncol + n0 + c, v);
      }
      return;
    }
    if (lane < LPR && nok) {
      float* sp = red + (size_t)(bid & (BIGDL_STAT_SLOTS - 1)) * 2 * a.Ncol;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        atomicAdd(sp + n + e, s1[e]);
        atomicAdd(sp + a.Ncol + n + e, s2[e]);
      }
    }
  }
}

// ---- halo-style epilogues (conv_halo.hip, stem.hip). nt_epilogue_lds (its runtime-flag branches around every optional load put vmcnt(0) waits in front of
// its stores, and 7 row chunks per tile serialise on them: 42 of the 79 us of the 28x28 layer, BIGDL_CONV_HALO_ABL)
// is replaced by two branch-free forms; rows without an output pixel get a buffer offset past num_records (stores
// dropped, loads return 0).
constexpr unsigned EOOB = 0x7ffffff0u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p, size_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)(bytes < 0x7fffffffu ? bytes : 0x7fffffffu),
                                           0x00020000);
}

// Workgroup-level commit of per-wave channel sums: every wave parks its 64 channels' (s1, s2) in LDS, then one pass of
// the workgroup adds the WPX pixel-group partials of each of its KT channels and issues ONE atomic per value: 2 * KT /
// 256 full-wave atomic instructions per tile instead of 16-32 mostly-idle ones per wave (a memory-side float atomic
// costs ~50 ns per wave-instruction per CU whatever its lane count: that, not bandwidth, made the epilogue slow).
template <int WCH, int KT>
__device__ __forceinline__ void halo_commit(float* red, float* rl, int k0, int Ncol, int bid) {
  __syncthreads();
  const int t = threadIdx.x;
  if (t < 2 * KT) {
    const int which = t / KT, c = t - which * KT, wc = c / 64, cl = c & 63;
    float v = 0.f;
#pragma unroll
    for (int wp = 0; wp < 4 / WCH; ++wp) v += rl[(wp * WCH + wc) * 128 + which * 64 + cl];
    atomicAdd(red + (size_t)(bid & (BIGDL_STAT_SLOTS - 1)) * 2 * Ncol + which * Ncol + k0 + c, v);
  }
}

// Lean form (no addend / consumer-BN reduction: the forward with optional bias, ReLU and BN statistics): the wave's
// 64-channel tile goes through its LDS slice once as bf16 (bias added in fp32 before the rounding) ([pixel][8 granules], granule g of pixel p in slot g ^ (p & 7)),
// then 8 lanes store one pixel's whole 128-byte row (16-byte buffer stores); statistics of the rounded output.
// BNR: also the consumer-BN backward reduction of the rounded output (data gradients; no addend): every BN x row and
// mask byte of the wave's tile is loaded into registers BEFORE the first store, so no load waits behind a store.
template <int FM, int FN, int WCH, int KT, bool BNR = false, class RM>
__device__ __forceinline__ void halo_epi_lean(const ConvArgs& a, v4f (&acc)[FM][FN], int vbase, int nbase, int lane,
                                              int bid, unsigned char* sl, const RM& rm, float* rl0, int k0) {
  float* rl = rl0 + (threadIdx.x >> 6) * 128;
  static_assert(FN == 4, "64-channel wave tile");
  constexpr int TM = FM * 16;
  float bs[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) bs[j][e] = a.bias ? a.bias[nbase + j * 16 + 4 * (lane >> 4) + e] : 0.f;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int p = i * 16 + (lane & 15), g = 2 * j + (lane >> 5);
      const v2u w = {pack2bf(acc[i][j][0] + bs[j][0], acc[i][j][1] + bs[j][1]),
                     pack2bf(acc[i][j][2] + bs[j][2], acc[i][j][3] + bs[j][3])};
      *reinterpret_cast<v2u*>(sl + p * 128 + ((g ^ (p & 7)) << 4) + ((lane >> 4) & 1) * 8) = w;
    }
  const size_t rows = (size_t)a.Nb * a.OH * a.OW;
  const __amdgpu_buffer_rsrc_t ro = rsrc_of(a.out, ((rows - 1) * a.ldo + a.Ncol) * 2);
  const int q = lane & 7;
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s1[e] = s2[e] = 0.f;
  const bool relu = a.relu != 0, st = a.stats != nullptr;
  // consumer-BN operands (BNR): x rows, and the ReLU mask as z rows or sign-mask bytes, or from x * scale + shift
  constexpr int NRW = BNR ? TM / 8 : 1;
  // (a bf16 z is not taken here: the caller routes it to the full epilogue; the sign mask stays one byte per row)
  v4u px[NRW];
  unsigned zbm[NRW];
  float bmu[8], bsc[8], bsh[8];
  int zmode = 0;
  if constexpr (BNR) {
    const size_t nb2 = ((rows - 1) * a.ldo + a.Ncol) * 2;
    const __amdgpu_buffer_rsrc_t rbx = rsrc_of(a.bnx, nb2);
    const __amdgpu_buffer_rsrc_t rzm = rsrc_of(a.bnzm, a.bnzm ? nb2 / 16 : 0);
    zmode = a.bnzm ? 1 : a.bnaff ? 3 : 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = nbase + q * 8 + e;
      bmu[e] = a.bnmean[c];
      bsc[e] = a.bnaff ? a.bnaff[c] : 0.f;
      bsh[e] = a.bnaff ? a.bnaff[a.Ncol + c] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < NRW; ++r) {
      const long orow = rm(a, vbase + r * 8 + (lane >> 3));
      const size_t el = (size_t)(orow >= 0 ? orow : 0) * a.ldo + nbase + q * 8;
      const unsigned off = orow >= 0 ? (unsigned)(el * 2) : EOOB;
      px[r] = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(rbx, off, 0, 0));
      zbm[r] = zmode == 1 ? __builtin_amdgcn_raw_buffer_load_b8(rzm, orow >= 0 ? (unsigned)(el >> 3) : EOOB, 0, 0) : 0u;
    }
  }
#pragma unroll
  for (int r = 0; r < TM / 8; ++r) {
    const int p = r * 8 + (lane >> 3);
    v4u o = *reinterpret_cast<const v4u*>(sl + p * 128 + ((q ^ (p & 7)) << 4));
    const long orow = rm(a, vbase + p);
    if constexpr (BNR) {
      const float vm = orow >= 0 ? 1.f : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x0 = lo_bf(px[r][e]), x1 = hi_bf(px[r][e]);
        bool k0m = true, k1m = true;
        if (zmode == 1) { k0m = (zbm[r] >> (2 * e)) & 1u; k1m = (zbm[r] >> (2 * e + 1)) & 1u; }
        else if (zmode == 3) { k0m = x0 * bsc[2 * e] + bsh[2 * e] > 0.f; k1m = x1 * bsc[2 * e + 1] + bsh[2 * e + 1] > 0.f; }
        const float d0 = k0m ? lo_bf(o[e]) * vm : 0.f, d1 = k1m ? hi_bf(o[e]) * vm : 0.f;
        s1[2 * e] += d0; s2[2 * e] += d0 * (x0 - bmu[2 * e]);
        s1[2 * e + 1] += d1; s2[2 * e + 1] += d1 * (x1 - bmu[2 * e + 1]);
      }
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = pack2bf(fmaxf(lo_bf(o[e]), 0.f), fmaxf(hi_bf(o[e]), 0.f));
    }
    if (st) {
      const float vm = orow >= 0 ? 1.f : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float y0 = lo_bf(o[e]) * vm, y1 = hi_bf(o[e]) * vm;
        s1[2 * e] += y0; s2[2 * e] += y0 * y0;
        s1[2 * e + 1] += y1; s2[2 * e + 1] += y1 * y1;
      }
    }
    const unsigned off = orow >= 0 ? (unsigned)(((size_t)orow * a.ldo + nbase + q * 8) * 2) : EOOB;
    __builtin_amdgcn_raw_buffer_store_b128(o, ro, off, 0, 0);
  }
  if (st || BNR) {          // uniform: every wave of the workgroup takes this branch
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        s1[e] += __shfl_xor(s1[e], o, 64);
        s2[e] += __shfl_xor(s2[e], o, 64);
      }
    if (lane < 8) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { rl[q * 8 + e] = s1[e]; rl[64 + q * 8 + e] = s2[e]; }
    }
    halo_commit<WCH, KT>(BNR ? a.bnred : a.stats, rl0, k0, a.Ncol, bid);
  }
}


}  // namespace
