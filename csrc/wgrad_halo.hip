// Weight gradient of 3x3 / stride 1 / pad 1 convolutions from halo tiles (gfx950).
//
// dW[k][(r, s, c)] = sum over output pixels p of dy[p][k] * x[p + (r - 1, s - 1)][c]  (reference: the weight
// gradient of S/nn/SpatialConvolution.scala accGradParameters, MKL-DNN's backward-weights primitive there).
//
// The split-K im2col kernels (conv_igemm.hip, conv_wgrad_glds_kernel) DMA one x granule per (pixel, tap): every x
// element crosses the DMA engine 9 times and every DMA row costs ~10 VALU instructions of (image, row, column) and
// bounds arithmetic, so the ResNet-50 3x3 weight gradients ran at 6-9x their MFMA bound with MFMA busy ~22 %
// (profiles/r5_wgrad_glds_pmc_*.txt). Here a workgroup stages RB whole image rows at a time ("virtual pixels":
// the rows padded by one zero column on each side, RB * (W + 2) of them, rounded up to 32) together with a one-row
// halo above and below, ONCE, and reads the 9 shifted windows out of LDS:
//   * x tile: image rows oh0 - 1 .. oh0 + RB, each stored as W + 2 rows of 64 channels (128 B) with the zero pad
//     columns materialised, behind one guard row. Virtual pixel v = (rr, j) (j = padded column) reads tap (r, s) at
//     tile row v + r * (W + 2) + s (guard included): a constant shift per tap, no masks — pad columns and rows
//     outside the image are zero granules, and dy is zero at the padded columns, so wrapped reads multiply zeros.
//   * dy tile: the RB image rows of dy in the same padded virtual-pixel order (zero at the pad columns / tail).
//   * every DMA lane's source offset relative to the stage base is fixed for the whole kernel (precomputed); per
//     stage a lane adds one 64-bit base and picks the zero granule for halo rows outside the image.
//   * fragments come from ds_read_b64_tr_b16 (pixels down the rows); row swizzles f128 / f256 (slot g holds
//     granule g ^ f(row), applied on the DMA source side) keep every 32-lane transposed read conflict-free for ANY
//     row shift (checked exhaustively for shifts 0..199).
// Workgroup tile: 64 input channels x KB output channels x all 9 taps; KB / 16 waves = 4 channel blocks of 16 x
// KB / 64 output-channel groups of 64; a wave holds 9 x 4 16x16 accumulators (144 registers) and per 32 virtual
// pixels issues 36 MFMAs against 26 transposed LDS reads (8 dy + 18 x). NS LDS stages fill the LDS budget (80 KB by
// default, BIGDL_WGRAD_HALO_LDS); the DMA runs NS - 2 stages ahead with counted vmcnt waits and one barrier per stage.
// Splits over image-row stages give ~256 workgroups; partials go to the workspace and wgrad_reduce_kernel sums them
// in a fixed order (deterministic), one split adds into dW directly.
#include <algorithm>
#include <cstdlib>
#include <type_traits>
#include <utility>

#include "common.h"
#include "kernels.h"

namespace {

__device__ __forceinline__ int hf128(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }
__device__ __forceinline__ int hf256(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

template <int W, int RB, int KB, int LDSKB>
struct Halo {
  static constexpr int WP = W + 2;
  static constexpr int V = (RB * WP + 31) / 32 * 32;        // virtual pixels per stage
  static constexpr int NCH = V / 32;                        // MFMA reduction chunks per stage
  static constexpr int NW = KB / 16;                        // waves: 4 channel blocks x KB/64 k-groups
  static constexpr int NT = 64 * NW;
  static constexpr int XROWS = V + 2 * WP + 2;              // x tile rows any tap of any virtual pixel reads
  static constexpr int XG = (XROWS * 8 + NT - 1) / NT;      // x DMA instructions per thread per stage
  static constexpr int XR = XG * NT / 8;                    // x rows allocated (all DMA'd: finite)
  static constexpr int DG = V * KB / 8 / NT;                // dy DMA instructions per thread per stage
  static constexpr int DROW = KB * 2;                       // dy row bytes
  static constexpr int XBYTES = XR * 128;
  static constexpr int STAGE = XBYTES + V * DROW;
  static constexpr int NSR = (LDSKB * 1024) / STAGE;
  static constexpr int NS = NSR > 6 ? 6 : NSR;
  static constexpr int D = XG + DG;
  static_assert((V * KB / 8) % NT == 0, "dy tile must split evenly into DMA instructions");
  static_assert(NS >= 2, "need >= 2 LDS stages");
  static_assert(XG <= 8 && DG <= 4, "flag packing");
};

// ds_read_b64_tr_b16 pair (rows r and r + 4 of a fragment) -> one 8 x bf16 MFMA operand; OFF is a byte immediate
template <int OFF>
__device__ __forceinline__ v8s trd2(unsigned a0, unsigned a1) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset field");
  v4s lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(a0), "n"(OFF));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "n"(OFF));
  return v8s{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}
// wait until <= N LDS reads are outstanding; the operand tie keeps every use of `v` behind the wait
template <int N>
__device__ __forceinline__ void lgkm_wait(v8s& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}
template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int D, int MAXK>
__device__ __forceinline__ void vm_wait_stages(int k) {   // wait until <= k stages (k * D DMAs) are outstanding
  if constexpr (MAXK >= 4) { if (k >= 4) { vm_wait<4 * D>(); return; } }
  if constexpr (MAXK >= 3) { if (k == 3) { vm_wait<3 * D>(); return; } }
  if constexpr (MAXK >= 2) { if (k == 2) { vm_wait<2 * D>(); return; } }
  if constexpr (MAXK >= 1) { if (k == 1) { vm_wait<D>(); return; } }
  vm_wait<0>();
}

// PRE: x is the input of a training BatchNorm + ReLU (WgradArgs::pre): once a stage's DMAs have landed, each lane
// rewrites the x granules it staged as relu(x * scale + shift) rounded to bf16 (bn_apply_kernel's expression), before
// the barrier that publishes the stage; granules of pad columns / rows outside the image stay zero. The 64 channels'
// scale / shift sit in LDS behind the stages.
template <int W, int RB, int KB, int LDSKB, bool PRE = false>
__global__ __launch_bounds__(KB * 4, 1) void conv_wgrad_halo_kernel(WgradArgs a) {
  using H = Halo<W, RB, KB, LDSKB>;
  __shared__ __attribute__((aligned(1024))) unsigned char lds[H::NS * H::STAGE + (PRE ? 512 : 0)];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cw = wave & 3, kg = wave >> 2;
  const int C = a.Cs, K = a.Ncol, IH = a.Hs;
  const int tiles_c = C / 64, ntile = tiles_c * (K / KB);
  // split-major XCD order (as conv_wgrad_glds_kernel): a split's tiles share its x / dy rows in one XCD's L2
  const int L = blockIdx.x, kq = L >> 3;
  const int split = 8 * (kq / ntile) + (L & 7);
  const int t = kq % ntile;
  const int c0 = (t % tiles_c) * 64, k0 = (t / tiles_c) * KB;
  const int spi = IH / RB, nstage_all = a.Nb * spi;
  const int st0 = split * a.m_per_split;
  const int nst = min(nstage_all, st0 + a.m_per_split) - st0;
  if (split >= a.splits || nst <= 0) return;

  // ---- per-lane DMA sources: byte offsets from the stage's buffer-resource base, fixed for the whole kernel.
  // x base = stage pixel - W (so the top halo row is >= 0); a lane whose slot is padding, or a halo row outside the
  // image, gets an offset past num_records and the buffer unit returns (and the DMA writes) zeros. Variant v of the x
  // offsets = (top halo row outside the image) | (bottom halo row outside) << 1, picked per stage by a scalar branch.
  constexpr unsigned OOB = 0x7ffffff0u;
  unsigned xv[4][H::XG];
#pragma unroll
  for (int d = 0; d < H::XG; ++d) {
    const int slot = (d * H::NW + wave) * 64 + lane;
    const int row = slot >> 3;
    const int g = (slot & 7) ^ hf128(row);
    const int xr = row - 1;                                 // row 0 is the guard
    const int rr = xr >= 0 ? xr / H::WP : -1, j = xr - rr * H::WP;
    const bool ok = xr >= 0 && rr < RB + 2 && j >= 1 && j <= W;
    const unsigned off = (unsigned)((rr * W + (j - 1)) * C + c0 + g * 8) * 2u;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const bool bad = ((v & 1) && rr == 0) || ((v & 2) && rr == RB + 1);
      xv[v][d] = (ok && !bad) ? off : OOB;
    }
  }
  unsigned dv[H::DG];
#pragma unroll
  for (int d = 0; d < H::DG; ++d) {
    const int slot = (d * H::NW + wave) * 64 + lane;
    const int row = slot / (KB / 8);
    const int g = (slot % (KB / 8)) ^ (KB == 128 ? hf256(row) : hf128(row));
    const int rr = row / H::WP, j = row - rr * H::WP;
    const bool ok = rr < RB && j >= 1 && j <= W;
    dv[d] = ok ? (unsigned)((rr * W + (j - 1)) * a.ldy + k0 + g * 8) * 2u : OOB;
  }
  const bf16_t* xsrc = reinterpret_cast<const bf16_t*>(a.src);
  const bf16_t* dsrc = reinterpret_cast<const bf16_t*>(a.dy);
  const size_t xend = (size_t)a.Nb * IH * W * C, dend = (size_t)(a.M - 1) * a.ldy + K;

  float* const ptab = reinterpret_cast<float*>(lds + H::NS * H::STAGE);
  if constexpr (PRE) {                  // [scale 64 | shift 64] of channels c0 .. c0 + 63
    if (tid < 32) {
      const int h = tid >> 4, i = tid & 15;
      reinterpret_cast<v4f*>(ptab)[tid] = reinterpret_cast<const v4f*>(a.pre + h * C + c0)[i];
    }
    __syncthreads();
  }
  // stages are issued in order: walk (image, first row) instead of dividing the stage index each time
  int nx = st0 / spi, ohx = (st0 - nx * spi) * RB;
  auto issue = [&](int buf) {
    const int n = nx, oh0 = ohx;
    ohx += RB;
    if (ohx == IH) { ohx = 0; ++nx; }
    const size_t pix = ((size_t)n * IH + oh0) * W;
    const size_t xo = pix * C - (size_t)W * C;              // wraps below 0 only for n = oh0 = 0 (all OOB then)
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(xsrc + xo), (short)0, (int)((xend - xo) * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(dsrc + pix * a.ldy), (short)0, (int)((dend - pix * a.ldy) * 2), 0x00020000);
    unsigned char* X = lds + buf * H::STAGE;
    const int v = (oh0 == 0 ? 1 : 0) | (oh0 + RB == IH ? 2 : 0);
    auto xdma = [&](auto vc) {
      constexpr int V = decltype(vc)::value;
#pragma unroll
      for (int d = 0; d < H::XG; ++d)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (LDS_PTR(void))(X + (d * H::NW + wave) * 64 * 16), 16,
                                                 (int)xv[V][d], 0, 0, 0);
    };
    switch (v) {
      case 0: xdma(std::integral_constant<int, 0>{}); break;
      case 1: xdma(std::integral_constant<int, 1>{}); break;
      case 2: xdma(std::integral_constant<int, 2>{}); break;
      default: xdma(std::integral_constant<int, 3>{}); break;
    }
    unsigned char* Dt = X + H::XBYTES;
#pragma unroll
    for (int d = 0; d < H::DG; ++d)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rd, (LDS_PTR(void))(Dt + (d * H::NW + wave) * 64 * 16), 16,
                                               (int)dv[d], 0, 0, 0);
  };

  // ---- per-lane LDS read offsets (bytes within a stage; + chunk * 32 rows as immediates)
  const int G = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  int xa[9][2], da[4][2];
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 8 * G + q + 4 * h + (tp / 3) * H::WP + (tp % 3);
      xa[tp][h] = row * 128 + (((cw * 2 + (p >> 1)) ^ hf128(row)) << 4) + (p & 1) * 8;
    }
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int row = 8 * G + q + 4 * h;
      const int gr = kg * 8 + kb * 2 + (p >> 1);
      da[kb][h] = H::XBYTES + row * H::DROW + ((gr ^ (KB == 128 ? hf256(row) : hf128(row))) << 4) + (p & 1) * 8;
    }

  const unsigned lds_base = (unsigned)(uintptr_t)(LDS_PTR(unsigned char))lds;
  v4f acc[9][4], accb[4];
#pragma unroll
  for (int i = 0; i < 9; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j) accb[j] = v4f{0.f, 0.f, 0.f, 0.f};
  // bias gradient (sum of dy over the pixels): the channel-block-0 waves of the first channel tile multiply their dy
  // fragments by a ones operand as well (every row of the product is the column sum)
  const bool bias = a.dbias != nullptr && c0 == 0 && cw == 0;
  const v8s ones = {(short)0x3f80, (short)0x3f80, (short)0x3f80, (short)0x3f80,
                    (short)0x3f80, (short)0x3f80, (short)0x3f80, (short)0x3f80};

  // prologue: stages 0 .. NS-2 in flight
#pragma unroll
  for (int s = 0; s < H::NS - 1; ++s)
    if (s < nst) issue(s);

  for (int i = 0; i < nst; ++i) {
    // stage i landed (this wave's DMAs), then every wave's (barrier); the barrier also retires stage i-1's reads
    vm_wait_stages<H::D, H::NS - 2>(min(H::NS - 2, nst - 1 - i));
    if constexpr (PRE) {
      const int sg = st0 + i, oh0 = (sg % spi) * RB;
      const int v = (oh0 == 0 ? 1 : 0) | (oh0 + RB == IH ? 2 : 0);
      const unsigned xb = (unsigned)(uintptr_t)(LDS_PTR(unsigned char))lds + (unsigned)((i % H::NS) * H::STAGE);
      // inline asm LDS accesses (a plain load here would make the compiler drain every in-flight stage DMA): every
      // granule's read issued at once, one wait, then branch-free rewrites (pad / out-of-image granules keep zero).
      // A lane's granule g = (slot & 7) ^ hf128(row) with slot & 7 = lane & 7 and row = slot >> 3, so g depends on d:
      // its 8 scale / shift pairs are read per granule.
      constexpr int PG = H::XG < 4 ? H::XG : 4;            // granules per batch (8 at once spilled)
#pragma unroll
      for (int d0 = 0; d0 < H::XG; d0 += PG) {
        v4u u[PG];
        v4f s0[PG], s1[PG], b0[PG], b1[PG];
#pragma unroll
        for (int q = 0; q < PG; ++q) {
          const int d = d0 + q;
          if (d >= H::XG) break;
          const int slot = (d * H::NW + wave) * 64 + lane;
          const int g = (slot & 7) ^ hf128(slot >> 3);
          const unsigned ta = (unsigned)(uintptr_t)(LDS_PTR(float))ptab + (unsigned)(g * 32);
          const unsigned addr = xb + (unsigned)(slot * 16);
          asm volatile("ds_read_b128 %0, %5\n\tds_read_b128 %1, %6 offset:0\n\tds_read_b128 %2, %6 offset:16\n\t"
                       "ds_read_b128 %3, %6 offset:256\n\tds_read_b128 %4, %6 offset:272"
                       : "=v"(u[q]), "=v"(s0[q]), "=v"(s1[q]), "=v"(b0[q]), "=v"(b1[q]) : "v"(addr), "v"(ta) : "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // tie the loaded values to volatile asms behind the wait (their arithmetic cannot be hoisted above it)
#pragma unroll
        for (int q = 0; q < PG; ++q) asm volatile("" : "+v"(u[q]), "+v"(s0[q]), "+v"(s1[q]), "+v"(b0[q]), "+v"(b1[q]));
#pragma unroll
        for (int q = 0; q < PG; ++q) {
          const int d = d0 + q;
          if (d >= H::XG) break;
          const unsigned off = v == 0 ? xv[0][d] : v == 1 ? xv[1][d] : v == 2 ? xv[2][d] : xv[3][d];
          const int slot = (d * H::NW + wave) * 64 + lane;
          const unsigned addr = xb + (unsigned)(slot * 16);
          const float sc[8] = {s0[q][0], s0[q][1], s0[q][2], s0[q][3], s1[q][0], s1[q][1], s1[q][2], s1[q][3]};
          const float sh[8] = {b0[q][0], b0[q][1], b0[q][2], b0[q][3], b1[q][0], b1[q][1], b1[q][2], b1[q][3]};
          v4u t;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            t[e] = pack2bf(fmaxf(lo_bf(u[q][e]) * sc[2 * e] + sh[2 * e], 0.f),
                           fmaxf(hi_bf(u[q][e]) * sc[2 * e + 1] + sh[2 * e + 1], 0.f));
          const v4u o = off != OOB ? t : u[q];
          asm volatile("ds_write_b128 %0, %1" ::"v"(addr), "v"(o) : "memory");
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (i + H::NS - 1 < nst) issue((i + H::NS - 1) % H::NS);
    // fragment reads as inline asm (counted lgkmcnt waits below): hipcc's waitcnt pass treats a transposed-read
    // builtin as aliasing every in-flight LDS DMA and drains vmcnt to 0 before it, which would serialise the stages
    const unsigned sb = lds_base + (unsigned)((i % H::NS) * H::STAGE);
    unsigned xad[9][2], dad[4][2];
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) { xad[tp][0] = sb + xa[tp][0]; xad[tp][1] = sb + xa[tp][1]; }
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) { dad[kb][0] = sb + da[kb][0]; dad[kb][1] = sb + da[kb][1]; }
    sfor<H::NCH>([&](auto chc) {
      constexpr int ch = decltype(chc)::value;
      constexpr int XO = ch * 32 * 128, DO = ch * 32 * H::DROW;
      v8s fd[4], fx[3];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) fd[kb] = trd2<DO>(dad[kb][0], dad[kb][1]);
      fx[0] = trd2<XO>(xad[0][0], xad[0][1]);
      fx[1] = trd2<XO>(xad[1][0], xad[1][1]);
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        if (tp + 2 < 9) fx[(tp + 2) % 3] = trd2<XO>(xad[tp + 2][0], xad[tp + 2][1]);
        // tap tp's reads (and at tp == 0 the dy fragments) retired; 2 taps' reads stay in flight
        if (tp + 2 < 9) lgkm_wait<4>(fx[tp % 3]);
        else if (tp + 1 < 9) lgkm_wait<2>(fx[tp % 3]);
        else lgkm_wait<0>(fx[tp % 3]);
        if (tp == 0) {
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) lgkm_wait<4>(fd[kb]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
          acc[tp][kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fx[tp % 3], fd[kb], acc[tp][kb], 0, 0, 0);
        if (tp == 0 && bias) {
#pragma unroll
          for (int kb = 0; kb < 4; ++kb) accb[kb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, fd[kb], accb[kb], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    });
  }

  // ---- bias: lanes 0..15 hold the column sums of k = k0 + kg * 64 + kb * 16 + lane (row 0 of the product)
  if (bias && lane < 16) {
    float* bp = a.ws ? a.ws + (size_t)a.splits * K * a.Kdim + (size_t)split * K : a.dbias;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int k = k0 + kg * 64 + kb * 16 + lane;
      if (a.ws) bp[k] = accb[kb][0];
      else if (a.splits > 1) unsafeAtomicAdd(bp + k, accb[kb][0]);
      else bp[k] += accb[kb][0];
    }
  }
  // ---- out: lane holds dW[k][tap * C + c .. c + 3] (4 consecutive c of one k) per accumulator
  const int Kd = a.Kdim;
  float* base = a.ws ? a.ws + (size_t)split * K * Kd : a.dw;
  const bool aligned = ((reinterpret_cast<uintptr_t>(base) | (unsigned)Kd * 4u) & 15) == 0;
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      const int k = k0 + kg * 64 + kb * 16 + (lane & 15);
      float* o = base + (size_t)k * Kd + tp * C + c0 + cw * 16 + 4 * G;
      if (a.ws) {
        *reinterpret_cast<v4f*>(o) = acc[tp][kb];
      } else if (a.splits > 1) {    // atomic mode (halo_atomic): the splits meet in dW through fp32 atomics
#pragma unroll
        for (int e = 0; e < 4; ++e) unsafeAtomicAdd(o + e, acc[tp][kb][e]);
      } else if (aligned) {
        *reinterpret_cast<v4f*>(o) += acc[tp][kb];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] += acc[tp][kb][e];
      }
    }
}

// dw[i] += sum over splits of ws[split][i], in a fixed order (deterministic): a workgroup owns 16 float4 columns and
// its 16 thread rows stride the splits (coalesced 256-byte rows), then a fixed-order sum of the 16 row partials.
// ~n4 / 16 workgroups keep the chip busy even for a 64 x 576 weight with 256 splits (the per-column loop of
// wgrad_reduce_kernel ran 36 workgroups there: 38 us for 38 MB).
__global__ __launch_bounds__(256) void halo_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw, long n4,
                                                         int splits, int aligned) {
  __shared__ v4f red[16][17];
  const int e = threadIdx.x & 15, g = threadIdx.x >> 4;
  const long i = (long)blockIdx.x * 16 + e;
  v4f s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f}, s2 = s0, s3 = s0;
  if (i < n4) {
    const v4f* w4 = reinterpret_cast<const v4f*>(ws);
    int sp = g;
    // four independent loads in flight per trip (the partial rows are read once: latency, not bandwidth, bound)
    for (; sp + 48 < splits; sp += 64) {
      const v4f a0 = w4[(long)sp * n4 + i], a1 = w4[(long)(sp + 16) * n4 + i];
      const v4f a2 = w4[(long)(sp + 32) * n4 + i], a3 = w4[(long)(sp + 48) * n4 + i];
      s0 += a0; s1 += a1; s2 += a2; s3 += a3;
    }
    for (; sp < splits; sp += 16) s0 += w4[(long)sp * n4 + i];
  }
  red[g][e] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && i < n4) {
    v4f t = red[0][e];
#pragma unroll
    for (int r = 1; r < 16; ++r) t += red[r][e];
    if (aligned) {
      reinterpret_cast<v4f*>(dw)[i] += t;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) dw[4 * i + k] += t[k];
    }
  }
}

template <int W, int RB, int LDSKB>
void launch_halo(const WgradArgs& a, hipStream_t st) {
  const int ntile = (a.Cs / 64) * (a.Ncol / (a.Ncol % 128 == 0 ? 128 : 64));
  const int spad = (a.splits + 7) / 8 * 8;
  if (a.pre) {     // (launch_halo_lds: the 80 KB budget, so the channel table fits behind the stages)
    if constexpr (LDSKB <= 80) {
      if (a.Ncol % 128 == 0) conv_wgrad_halo_kernel<W, RB, 128, LDSKB, true><<<dim3(ntile * spad), dim3(512), 0, st>>>(a);
      else conv_wgrad_halo_kernel<W, RB, 64, LDSKB, true><<<dim3(ntile * spad), dim3(256), 0, st>>>(a);
    }
  } else if (a.Ncol % 128 == 0) {
    conv_wgrad_halo_kernel<W, RB, 128, LDSKB><<<dim3(ntile * spad), dim3(512), 0, st>>>(a);
  } else {
    conv_wgrad_halo_kernel<W, RB, 64, LDSKB><<<dim3(ntile * spad), dim3(256), 0, st>>>(a);
  }
}

template <int W, int RB>
void launch_halo_lds(const WgradArgs& a, int lds, hipStream_t st) {
  if (lds <= 80 || a.pre) launch_halo<W, RB, 80>(a, st);
  else launch_halo<W, RB, 160>(a, st);
}

int halo_rb(int W) { return W == 56 ? 1 : W == 28 ? 2 : W == 14 ? 2 : W == 7 ? 7 : 0; }

int g_wgrad_halo = -1;
// BIGDL_WGRAD_HALO_LDS: LDS budget per workgroup in KB. 80 (default) leaves half a CU's LDS to the data-gradient
// chain running beside the weight gradient on the other stream and measured as fast in isolation as 160 (fewer
// stages in flight, same MFMA rate: profiles/r5_wgrad_halo_ab.txt)
int halo_lds() {
  static const int v = [] { const char* e = getenv("BIGDL_WGRAD_HALO_LDS"); return e ? atoi(e) : 80; }();
  return v;
}
// BIGDL_WGRAD_HALO_ATOMIC=1: with splits > 1 the splits add into dW / dbias with fp32 atomics instead of writing
// workspace partials for halo_reduce_kernel (one fp32 copy of dW per split written and re-read); never in
// deterministic mode (atomic order)
bool halo_atomic() {
  static const int v = [] { const char* e = getenv("BIGDL_WGRAD_HALO_ATOMIC"); return e ? atoi(e) : 0; }();
  return v != 0 && !bigdl_deterministic();
}
int halo_wgs() {
  static const int v = [] { const char* e = getenv("BIGDL_WGRAD_HALO_WGS"); return e ? atoi(e) : 256; }();
  return v;
}

}  // namespace

extern "C" {

void bigdl_set_wgrad_halo(int v) { g_wgrad_halo = v; }

// Splits (>= 1) when the halo kernel takes this weight gradient (sets a->m_per_split = image-row stages per
// split), 0 otherwise. BIGDL_WGRAD_HALO=0 turns it off.
int bigdl_wgrad_halo_plan(WgradArgs* a) {
  if (g_wgrad_halo < 0) {
    const char* e = getenv("BIGDL_WGRAD_HALO");
    g_wgrad_halo = e ? atoi(e) : 1;
  }
  if (!g_wgrad_halo) return 0;
  const int rb = halo_rb(a->Ws);
  if (rb == 0 || a->R != 3 || a->S != 3 || a->sh != 1 || a->sw != 1 || a->ph != 1 || a->pw != 1 || a->dh != 1 ||
      a->dwl != 1 || a->OH != a->Hs || a->OW != a->Ws || (a->Hs % rb) || (a->Cs % 64) || (a->Ncol % 64) ||
      a->Kdim != 9 * a->Cs || a->ldy != a->Ncol || a->M != a->Nb * a->OH * a->OW || a->M <= 0)
    return 0;
  const long stages = (long)a->Nb * (a->Hs / rb);
  const int ntile = (a->Cs / 64) * (a->Ncol / (a->Ncol % 128 == 0 ? 128 : 64));
  const long x_bytes = (long)a->Nb * a->Hs * a->Ws * a->Cs * 2, dy_bytes = (long)a->M * a->ldy * 2;
  if (x_bytes >= (1L << 30) || dy_bytes >= (1L << 30)) return 0;    // 32-bit buffer offsets
  long splits = std::max(1L, std::min(stages, ((long)halo_wgs() + ntile - 1) / ntile));
  const long sps = (stages + splits - 1) / splits;
  splits = (stages + sps - 1) / sps;
  a->m_per_split = (int)sps;
  return (int)splits;
}

int bigdl_wgrad_pre_applies(const WgradArgs* a) {
  WgradArgs b = *a;
  return bigdl_wgrad_halo_plan(&b) > 0 ? 1 : 0;
}

// Launch (a->splits / m_per_split from bigdl_wgrad_halo_plan; a->ws = [splits][Ncol][Kdim] partials when splits > 1,
// then [splits][Ncol] bias partials when a->dbias, summed into a->dw / a->dbias in split order, else the kernel adds
// into a->dw / a->dbias).
int bigdl_wgrad_halo(const WgradArgs* a_in, hipStream_t st) {
  const int lds = halo_lds();
  WgradArgs b = *a_in;
  if (b.splits > 1 && halo_atomic()) b.ws = nullptr;
  const WgradArgs* a = &b;
  switch (a->Ws) {
    case 56: launch_halo_lds<56, 1>(*a, lds, st); break;
    case 28: launch_halo_lds<28, 2>(*a, lds, st); break;
    case 14: launch_halo_lds<14, 2>(*a, lds, st); break;
    case 7: launch_halo_lds<7, 7>(*a, lds, st); break;
    default: return -1;
  }
  if (a->splits > 1 && a->ws != nullptr) {
    const long n4 = (long)a->Ncol * a->Kdim / 4;
    const int aligned = (reinterpret_cast<uintptr_t>(a->dw) & 15) == 0;
    halo_reduce_kernel<<<dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, st>>>(a->ws, a->dw, n4, a->splits, aligned);
    if (a->dbias)      // [splits][Ncol] bias partials: the same split-parallel reduce (Ncol % 4 == 0)
      halo_reduce_kernel<<<dim3((unsigned)((a->Ncol / 4 + 15) / 16)), dim3(256), 0, st>>>(
          a->ws + (size_t)a->splits * a->Ncol * a->Kdim, a->dbias, a->Ncol / 4, a->splits,
          (reinterpret_cast<uintptr_t>(a->dbias) & 15) == 0);
  }
  return 0;
}

// dw[i] += sum over s of ws[s * n + i] (n % 4 == 0) in a fixed order, split-parallel: the stem weight gradient's
// per-workgroup partials (csrc/stem_fwd.hip) use the same reduce as the halo weight gradient
void bigdl_split_reduce_f32(const float* ws, float* dw, long n, int splits, hipStream_t st) {
  const long n4 = n / 4;
  halo_reduce_kernel<<<dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, st>>>(
      ws, dw, n4, splits, (reinterpret_cast<uintptr_t>(dw) & 15) == 0);
  HIP_LAUNCH_CHECK();
}

}  // extern "C"
