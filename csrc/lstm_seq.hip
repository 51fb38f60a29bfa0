// Whole-sequence LSTM recurrence as ONE persistent launch per direction (gfx950).
//
// Reference: the fused whole-sequence MKL-DNN RNN primitive S/nn/mkldnn/RNN.scala:167-320 (forward + backward over
// all time steps in one call), cell math S/nn/LSTM.scala:77-185 (gates i, g, f, o; c' = f*c + i*g; h' = o*tanh(c')).
//
// MI355X design. The per-step kernels of lstm.hip pay, every time step, a kernel boundary plus a re-read of their
// weight slice from L2 and of the previous state from other XCDs. Here the launch holds the recurrent weight for the
// whole sequence and only the state crosses workgroups:
//  * grid = 8 batch groups x M = H / 32 workgroups (256 for H = 1024: one 512-thread workgroup per CU). Group g =
//    blockIdx % 8 owns batch rows [g * Bg, (g + 1) * Bg) (Bg <= 16): under the round-robin dispatch its workgroups sit
//    on one XCD, so the per-step exchange is L2-local (placement only changes speed, never correctness: every
//    hand-off is an agent-scope protocol).
//  * member m owns hidden units [32 m, 32 m + 32); each of its 8 waves keeps its slice of W (16 gate rows x H for the
//    forward, 16 units x one gate block of W^T for the backward) in VGPRs as MFMA A fragments: KS = H / 32 fragments,
//    128 VGPRs at H = 1024, loaded once.
//  * per step a workgroup waits for its group's counter, pulls the group's previous state (bf16, 16 rows) into LDS
//    with write-through (sc1) 16-byte loads, runs KS MFMAs per wave on two accumulator chains, applies the cell in
//    registers, publishes its 16 x 32 slice of the new state with sc1 16-byte stores, drains them (vmcnt(0)) and adds
//    1 to the group counter (agent-scope atomic). This is the write-through hand-off of the CDNA4 programming guide's
//    inter-workgroup rule: every handed-off byte is stored sc1 and drained before the counter add, every load of it is
//    an sc1 load to registers behind the poll, and no other load reads bytes written in the launch.
//  * counters are zeroed by a fill kernel ahead of every launch (graph-replay safe: no memset node, see
//    bigdl_fill_bytes); every spin is bounded (2 s of the 100 MHz wall clock by default, bigdl_set_seq_timeout_us):
//    on timeout the workgroup sets the launch's error word AND a process-wide host-mapped word, poisons EVERY output
//    element it owns (remaining steps) with NaN and leaves. The host reads the mapped word without a device sync
//    (bigdl_persistent_error: TrainStep.throttle and every persistent-kernel call check it and raise).
//  * residency: correctness needs all 8 x H/32 workgroups co-resident. The launch is refused (per-step fallback) when
//    the occupancy query of the exact kernel instantiation admits less than one 512-thread workgroup per CU or the
//    grid exceeds the CU count; workgroups that are resident but wait on ones held back by OTHER streams' kernels
//    just spin until those finish (nothing those kernels wait on depends on this launch), bounded by the timeout.
// Forward per step: gates = W h_{t-1} (+ xg, the input projection computed beforehand as one GEMM), c and h in
// fp32, h16 bf16 hand-off (also the B operand of the weight-gradient GEMM). Backward per step: dh = dout + dg_{t+1} W
// (K = 4H split over the 4 gate blocks = 4 waves per unit tile, partials summed in LDS), the cell backward per
// (unit, batch) thread, dg_t as fp32 (input-projection gradients) and bf16 (hand-off + weight gradient); one extra
// round after t = 0 produces dh0 = dg_0 W, so no transposed weight copy is ever made.
#include "common.h"
#include "kernels.h"

namespace {

typedef __attribute__((address_space(1))) unsigned gu32;

constexpr int NGRP = 8;                          // batch groups (= XCDs)
constexpr int CNT_STRIDE = 32;                   // one 128-byte line per group counter
unsigned long long g_spin_ticks = 200000000ull;         // 2 s at 100 MHz (bigdl_set_seq_timeout_us)

struct LstmSeqArgs {
  const bf16_t* W16;       // [4H][H] gate blocks i, g, f, o
  const void* xg;          // fwd: [B][T][4H] gate pre-activations from the input projection (f32 or bf16: BIO)
  const float* c0;         // [B][H] or null
  const void* dout;        // bwd: [B][T][H] or null (f32 or bf16: BIO)
  const float* dhT;        // bwd: [B][H] or null
  const float* dcT;        // bwd: [B][H] or null
  bf16_t* h16;             // [T + 1][B][H]: h_{-1} .. h_{T-1}
  void* out;               // fwd: [B][T][H] (f32 or bf16: BIO)
  float* hT;               // fwd: [B][H] f32 last hidden state, or null
  float* cs;               // [T][B][H]
  float* acts;             // [T][B][4H]
  bf16_t* dg16;            // bwd: [T][B][4H]
  void* dxg;               // bwd: [B][T][4H] (f32 or bf16: BIO)
  float* dc0;              // bwd: [B][H] (dc flowing into c0)
  float* dh0;              // bwd: [B][H]
  unsigned* sync;          // NGRP counters (CNT_STRIDE apart) + error word
  unsigned* herr;          // process-wide host-mapped error word (device address)
  unsigned long long spin; // bound of every wait, wall-clock ticks (100 MHz)
  int B, H, T, Bg;
  int late;                // the publishing wave stores its outputs after the hand-off (BIGDL_LSTM_LATE)
};

// Host-mapped (fine-grained, coherent) error word shared by every persistent kernel of the process: a timeout stores
// to it with system scope, so the host can see the failure without synchronising the device.
unsigned* g_herr_host = nullptr;
unsigned* g_herr_dev = nullptr;
unsigned* host_err_dev() {
  if (g_herr_dev == nullptr) {
    void* h = nullptr;
    if (hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) != hipSuccess) return nullptr;
    for (int i = 0; i < 16; ++i) static_cast<volatile unsigned*>(h)[i] = 0u;
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess) return nullptr;
    g_herr_host = static_cast<unsigned*>(h);
    g_herr_dev = static_cast<unsigned*>(d);
  }
  return g_herr_dev;
}

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  const float e = __expf(-2.f * fabsf(x));
  const float t = (1.f - e) / (1.f + e);
  return x < 0.f ? -t : t;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
// 16-byte write-through load / store (aux 16 = sc1)
__device__ __forceinline__ v4u ld_sc1(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}
__device__ __forceinline__ void st_sc1(v4u v, __amdgpu_buffer_rsrc_t r, int off) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}

// One lane polls the group counter (relaxed agent-scope load = global_load sc1) until it reaches target.
__device__ __noinline__ bool wait_count(unsigned* cnt, unsigned target, unsigned* err, unsigned* herr,
                                       unsigned long long spin) {
  const unsigned long long t0 = wall_clock64();
  while (__hip_atomic_load((gu32*)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
    __builtin_amdgcn_s_sleep(1);
    if (wall_clock64() - t0 > spin) {
      __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (herr) {
        __hip_atomic_store(herr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      }
      return false;
    }
  }
  return true;
}

// Wave 0 polls, the verdict goes to every wave through LDS. Returns false when the group timed out.
__device__ __forceinline__ bool group_wait(unsigned* cnt, unsigned target, const LstmSeqArgs& a, int* flag, int wave,
                                           int lane) {
  if (wave == 0 && lane == 0) *flag = wait_count(cnt, target, a.sync + NGRP * CNT_STRIDE, a.herr, a.spin) ? 0 : 1;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keeps the sc1 state loads below the poll
  __syncthreads();
  return *flag == 0;
}

__device__ __forceinline__ void signal(unsigned* cnt) {
  __hip_atomic_fetch_add((gu32*)cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------------------------------------ forward
__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float((unsigned)v << 16); }

// BIO: xg / out (forward) and dout / dxg (backward) are bf16 (the projection GEMMs' own dtype; no f32 round trip)
// NT: 16-row batch tiles per group (1: B <= 128, 2: B <= 256). The weight fragments in VGPRs serve every tile: a
// second tile doubles the MFMAs per step and the state exchanged, not the weight traffic.
template <int KS, bool BIO, int NT>
__global__ __launch_bounds__(512, 1) void lstm_seq_fwd_kernel(LstmSeqArgs a) {
  constexpr int H = KS * 32;
  constexpr int HP = H + 8;                      // LDS row pitch: consecutive batch rows 4 banks apart
  constexpr int R = 16 * NT;                     // batch rows per group
  constexpr int CH = R * H / 8 / 512;            // 16-byte chunks of h_{t-1} per thread
  __shared__ __attribute__((aligned(16))) bf16_t hs[R * HP];
  __shared__ __attribute__((aligned(16))) bf16_t hst[R * 32];    // this workgroup's h_t slice [batch][unit]
  __shared__ int flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x % NGRP, m = blockIdx.x / NGRP, M = gridDim.x / NGRP;
  const int b_lo = g * a.Bg, nb = min(a.Bg, a.B - b_lo);
  if (nb <= 0) return;                            // no rows: nobody waits on this group
  const int G = lane >> 4, col = lane & 15;
  const int ub = m * 32 + wave * 4;               // the wave's 4 units; A row r = unit (r >> 2), gate (r & 3)
  const int j = ub + G;                           // this lane's unit in D (rows 4G .. 4G + 3 = its 4 gates)
  bool live[NT];
  int b[NT];
  float c[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    live[tt] = tt * 16 + col < nb;
    b[tt] = b_lo + (live[tt] ? tt * 16 + col : 0);
    c[tt] = a.c0 ? a.c0[(size_t)b[tt] * H + j] : 0.f;
  }
  v8s wa[KS];
  {
    const bf16_t* wp = a.W16 + (size_t)((col & 3) * H + ub + (col >> 2)) * H + 8 * G;
#pragma unroll
    for (int s = 0; s < KS; ++s) wa[s] = *reinterpret_cast<const v8s*>(wp + s * 32);
  }
  unsigned* cnt = a.sync + g * CNT_STRIDE;
  const size_t slab = (size_t)a.B * H;            // one time step of h16

  for (int t = 0; t < a.T; ++t) {
    float x[NT][4];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      const size_t xo = ((size_t)b[tt] * a.T + t) * 4 * H + j;
      if constexpr (BIO) {
        const bf16_t* xp = static_cast<const bf16_t*>(a.xg) + xo;
        x[tt][0] = bf2f(xp[0]); x[tt][1] = bf2f(xp[H]); x[tt][2] = bf2f(xp[2 * H]); x[tt][3] = bf2f(xp[3 * H]);
      } else {
        const float* xp = static_cast<const float*>(a.xg) + xo;
        x[tt][0] = xp[0]; x[tt][1] = xp[H]; x[tt][2] = xp[2 * H]; x[tt][3] = xp[3 * H];
      }
    }
    if (t > 0 && !group_wait(cnt, (unsigned)(M * t), a, &flag, wave, lane)) {
      // every element this lane owns from step t on: out, h16 (the weight-gradient operand), cs, acts, hT
      const float nan = __builtin_nanf("");
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        if (!live[tt]) continue;
        const int bt = b[tt];
        for (int u = t; u < a.T; ++u) {
          if constexpr (BIO) static_cast<bf16_t*>(a.out)[((size_t)bt * a.T + u) * H + j] = 0x7fc0;
          else static_cast<float*>(a.out)[((size_t)bt * a.T + u) * H + j] = nan;
          a.h16[(u + 1) * slab + (size_t)bt * H + j] = 0x7fc0;
          a.cs[((size_t)u * a.B + bt) * H + j] = nan;
          float* ap = a.acts + ((size_t)u * a.B + bt) * 4 * H + j;
          ap[0] = nan; ap[H] = nan; ap[2 * H] = nan; ap[3 * H] = nan;
        }
        if (a.hT) a.hT[(size_t)bt * H + j] = nan;
      }
      return;
    }
    {   // h_{t-1} of the group's rows -> LDS (rows past the group read as zero)
      const __amdgpu_buffer_rsrc_t r = rsrc(a.h16 + t * slab + (size_t)b_lo * H, nb * H * 2);
      v4u v[CH];
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int q = tid + 512 * i, row = q / (H / 8), c8 = q % (H / 8);
        v[i] = ld_sc1(r, (row * H + c8 * 8) * 2);
      }
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int q = tid + 512 * i, row = q / (H / 8), c8 = q % (H / 8);
        *reinterpret_cast<v4u*>(hs + row * HP + c8 * 8) = v[i];
      }
    }
    __syncthreads();
    // CH independent accumulator chains per batch tile (4 with one tile: a dependent MFMA waits out the previous
    // one's passes, so two chains left the matrix core idle between issues)
    constexpr int CH = NT == 1 ? 4 : 2;
    v4f acc[CH][NT];
#pragma unroll
    for (int q = 0; q < CH; ++q)
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) acc[q][tt] = v4f{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; s += CH) {
      if ((s & (8 / NT - 1)) == 0) asm volatile("" ::: "memory");     // <= 8 fragment reads in flight (VGPRs)
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        const bf16_t* hb = hs + (tt * 16 + col) * HP + 8 * G;
#pragma unroll
        for (int q = 0; q < CH; ++q) {
          const v8s hq = *reinterpret_cast<const v8s*>(hb + (s + q) * 32);
          acc[q][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[s + q], hq, acc[q][tt], 0, 0, 0);
        }
      }
    }
    // the publishing wave (0) stores its outputs AFTER the hand-off: its drain (vmcnt(0) before the counter add)
    // then waits for the state stores only, not for the scattered c / gate-activation stores (a.late; 0 = before)
    const bool late = wave == 0 && NT == 1 && a.late;   // (two-tile groups measured slower: B 256)
    float kh[NT], kc[NT], ka[NT][4];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      v4f gs = acc[0][tt];
#pragma unroll
      for (int q = 1; q < CH; ++q) gs += acc[q][tt];
      const float ig = sigm(gs[0] + x[tt][0]), gg = tanh_f(gs[1] + x[tt][1]), fg = sigm(gs[2] + x[tt][2]),
                  og = sigm(gs[3] + x[tt][3]);
      c[tt] = fg * c[tt] + ig * gg;
      const float h = og * tanh_f(c[tt]);
      kh[tt] = h; kc[tt] = c[tt];
      ka[tt][0] = ig; ka[tt][1] = gg; ka[tt][2] = fg; ka[tt][3] = og;
      if (live[tt] && !late) {
        const int bt = b[tt];
        if constexpr (!BIO) static_cast<float*>(a.out)[((size_t)bt * a.T + t) * H + j] = h;
        if (t == a.T - 1 && a.hT) a.hT[(size_t)bt * H + j] = h;
        a.cs[((size_t)t * a.B + bt) * H + j] = c[tt];
        float* ap = a.acts + ((size_t)t * a.B + bt) * 4 * H + j;
        ap[0] = ig; ap[H] = gg; ap[2 * H] = fg; ap[3 * H] = og;
      }
      hst[(tt * 16 + col) * 32 + wave * 4 + G] = f2bf(h);
    }
    __syncthreads();
    if (wave == 0) {   // publish: R rows x 64 B, lane -> (row, 16-byte quarter); drained before the counter add
      const __amdgpu_buffer_rsrc_t r = rsrc(a.h16 + (t + 1) * slab, (int)(slab * 2));
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        const int row = tt * 16 + (lane >> 2), qq = lane & 3;
        if (row < nb) {
          const v4u hv = *reinterpret_cast<const v4u*>(hst + row * 32 + qq * 8);
          st_sc1(hv, r, (int)(((b_lo + row) * H + m * 32 + qq * 8) * 2));
          if constexpr (BIO)   // the layer output is the same bf16 h: one plain 16-byte store per lane
            if (!(NT == 1 && a.late))
              *reinterpret_cast<v4u*>(static_cast<bf16_t*>(a.out) + ((size_t)(b_lo + row) * a.T + t) * H + m * 32 + qq * 8) = hv;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) signal(cnt);
      if (NT == 1 && a.late) {      // wave 0's outputs, behind the hand-off
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
          const int row = tt * 16 + (lane >> 2), qq = lane & 3;
          if constexpr (BIO)   // re-read from LDS: hst is not rewritten before this wave reaches the next barrier
            if (row < nb)
              *reinterpret_cast<v4u*>(static_cast<bf16_t*>(a.out) + ((size_t)(b_lo + row) * a.T + t) * H + m * 32 + qq * 8) =
                  *reinterpret_cast<const v4u*>(hst + row * 32 + qq * 8);
          if (live[tt]) {
            const int bt = b[tt];
            if constexpr (!BIO) static_cast<float*>(a.out)[((size_t)bt * a.T + t) * H + j] = kh[tt];
            if (t == a.T - 1 && a.hT) a.hT[(size_t)bt * H + j] = kh[tt];
            a.cs[((size_t)t * a.B + bt) * H + j] = kc[tt];
            float* ap = a.acts + ((size_t)t * a.B + bt) * 4 * H + j;
            ap[0] = ka[tt][0]; ap[H] = ka[tt][1]; ap[2 * H] = ka[tt][2]; ap[3 * H] = ka[tt][3];
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------ backward
// Wave w: unit tile ut = w & 1 (16 units), gate block q = w >> 1 (K chunk of H). A[unit][k] = W[q H + k][unit]
// gathered once; B = dg_{t+1}[batch][q H + k] from LDS; D[unit][batch] partials summed over q in LDS. With NT = 2
// the two 16-row batch tiles go through the one 16-row LDS image in turn (16 x 4H bf16 = 128 KB at H = 1024).
template <int KS, bool BIO, int NT>
__global__ __launch_bounds__(512, 1) void lstm_seq_bwd_kernel(LstmSeqArgs a) {
  constexpr int H = KS * 32, G4 = 4 * H;
  constexpr int DP = G4 + 8;
  constexpr int CH = 16 * G4 / 8 / 512;          // 16-byte chunks of one tile's dg_{t+1} per thread
  constexpr int R = 16 * NT;
  __shared__ __attribute__((aligned(16))) bf16_t dgs[16 * DP];
  __shared__ float red[4][32][17];               // [gate block][unit][batch]
  __shared__ __attribute__((aligned(16))) bf16_t dst[R * 4 * 32];    // dg_t slice [batch][gate][unit]
  __shared__ int flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x % NGRP, m = blockIdx.x / NGRP, M = gridDim.x / NGRP;
  const int b_lo = g * a.Bg, nb = min(a.Bg, a.B - b_lo);
  if (nb <= 0) return;
  const int G = lane >> 4, col = lane & 15;
  const int ut = wave & 1, q = wave >> 1;
  v8s wa[KS];
  {
    const bf16_t* wp = a.W16 + (size_t)(q * H + 8 * G) * H + m * 32 + ut * 16 + col;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      v4u f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        f[i] = (unsigned)wp[(size_t)(s * 32 + 2 * i) * H] | ((unsigned)wp[(size_t)(s * 32 + 2 * i + 1) * H] << 16);
      asm volatile("" : "+v"(f) :: "memory");   // packed per fragment: 8 loads in flight, 4 VGPRs kept
      wa[s] = __builtin_bit_cast(v8s, f);
    }
  }
  // cell thread: unit jj, batch rows bb + 16 tt
  const int jj = tid >> 4, bb = tid & 15;
  const int j = m * 32 + jj;
  bool live[NT];
  int b[NT];
  float dc[NT];
#pragma unroll
  for (int tt = 0; tt < NT; ++tt) {
    live[tt] = tt * 16 + bb < nb;
    b[tt] = b_lo + (live[tt] ? tt * 16 + bb : 0);
    dc[tt] = a.dcT ? a.dcT[(size_t)b[tt] * H + j] : 0.f;
  }
  unsigned* cnt = a.sync + g * CNT_STRIDE;
  const size_t slab = (size_t)a.B * G4;          // one time step of dg16

  // round i handles t = T-1-i; round T computes dh0 from dg_0
  for (int i = 0; i <= a.T; ++i) {
    const int t = a.T - 1 - i;
    float dh[NT], ig[NT], gg[NT], fg[NT], og[NT], cv[NT], cp[NT];
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      dh[tt] = ig[tt] = gg[tt] = fg[tt] = og[tt] = cv[tt] = cp[tt] = 0.f;
      if (t >= 0) {
        const int bt = b[tt];
        if (a.dout) {
          const size_t o = ((size_t)bt * a.T + t) * H + j;
          dh[tt] = BIO ? bf2f(static_cast<const bf16_t*>(a.dout)[o]) : static_cast<const float*>(a.dout)[o];
        }
        if (i == 0 && a.dhT) dh[tt] += a.dhT[(size_t)bt * H + j];
        const float* ap = a.acts + ((size_t)t * a.B + bt) * G4 + j;
        ig[tt] = ap[0]; gg[tt] = ap[H]; fg[tt] = ap[2 * H]; og[tt] = ap[3 * H];
        cv[tt] = a.cs[((size_t)t * a.B + bt) * H + j];
        cp[tt] = t > 0 ? a.cs[((size_t)(t - 1) * a.B + bt) * H + j] : (a.c0 ? a.c0[(size_t)bt * H + j] : 0.f);
      }
    }
    if (i > 0) {
      if (!group_wait(cnt, (unsigned)(M * i), a, &flag, wave, lane)) {
        // every element this thread owns from step t down: dxg, dg16 (the weight-gradient operand), dc0, dh0
        const float nan = __builtin_nanf("");
#pragma unroll
        for (int tt = 0; tt < NT; ++tt) {
          if (!live[tt]) continue;
          const int bt = b[tt];
          for (int u = t; u >= 0; --u) {
            const size_t go = ((size_t)bt * a.T + u) * G4 + j;
            bf16_t* dp = a.dg16 + u * slab + (size_t)bt * G4 + j;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              if constexpr (BIO) static_cast<bf16_t*>(a.dxg)[go + k * H] = 0x7fc0;
              else static_cast<float*>(a.dxg)[go + k * H] = nan;
              dp[k * H] = 0x7fc0;
            }
          }
          a.dh0[(size_t)bt * H + j] = nan;
          a.dc0[(size_t)bt * H + j] = nan;
        }
        return;
      }
#pragma unroll
      for (int tt = 0; tt < NT; ++tt) {
        {   // dg_{t+1} of this tile's rows of the group -> LDS (rows past the group read as zero)
          const int rows = max(0, min(16, nb - tt * 16));
          const __amdgpu_buffer_rsrc_t r = rsrc(a.dg16 + (t + 1) * slab + (size_t)(b_lo + tt * 16) * G4, rows * G4 * 2);
          // U loads per batch (VGPR budget: W takes 128), two batches in flight: batch h + 1 is issued before
          // batch h is written to LDS, so the CH / U batches do not each pay a full L2 round trip
          constexpr int U = CH < 4 ? CH : 4;
          auto ld = [&](v4u (&v)[U], int h) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int qc = tid + 512 * (h + u), row = qc / (G4 / 8), c8 = qc % (G4 / 8);
              v[u] = ld_sc1(r, (row * G4 + c8 * 8) * 2);
            }
          };
          auto st = [&](const v4u (&v)[U], int h) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
              const int qc = tid + 512 * (h + u), row = qc / (G4 / 8), c8 = qc % (G4 / 8);
              *reinterpret_cast<v4u*>(dgs + row * DP + c8 * 8) = v[u];
            }
          };
          if constexpr (NT == 1) {
            v4u va[U], vb[U];
            ld(va, 0);
#pragma unroll
            for (int h = 0; h < CH; h += 2 * U) {
              if (h + U < CH) ld(vb, h + U);
              st(va, h);
              if (h + U >= CH) break;
              if (h + 2 * U < CH) ld(va, h + 2 * U);
              st(vb, h + U);
            }
          } else {       // (two 16-row tiles: no registers for a second batch)
#pragma unroll
            for (int h = 0; h < CH; h += U) {
              v4u v[U];
              ld(v, h);
              st(v, h);
            }
          }
        }
        __syncthreads();
        v4f acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
        const bf16_t* db = dgs + col * DP + q * H + 8 * G;
#pragma unroll
        for (int s = 0; s < KS; s += 2) {
          const v8s d0 = *reinterpret_cast<const v8s*>(db + s * 32), d1 = *reinterpret_cast<const v8s*>(db + (s + 1) * 32);
          acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[s], d0, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[s + 1], d1, acc1, 0, 0, 0);
          if ((s & 7) == 6) asm volatile("" ::: "memory");   // <= 8 fragment reads in flight (VGPR budget)
        }
        const v4f p = acc0 + acc1;
#pragma unroll
        for (int e = 0; e < 4; ++e) red[q][ut * 16 + 4 * G + e][col] = p[e];
        __syncthreads();   // every wave's reads of dgs are done (they fed p) and red is complete
        dh[tt] += red[0][jj][bb] + red[1][jj][bb] + red[2][jj][bb] + red[3][jj][bb];
      }
    }
    if (t < 0) {   // final round: dh0 = dg_0 W
#pragma unroll
      for (int tt = 0; tt < NT; ++tt)
        if (live[tt]) a.dh0[(size_t)b[tt] * H + j] = dh[tt];
      break;
    }
#pragma unroll
    for (int tt = 0; tt < NT; ++tt) {
      const float tc = tanh_f(cv[tt]);
      const float dcv = dh[tt] * og[tt] * (1.f - tc * tc) + dc[tt];
      const float di = dcv * gg[tt] * ig[tt] * (1.f - ig[tt]);
      const float dgg = dcv * ig[tt] * (1.f - gg[tt] * gg[tt]);
      const float df = dcv * cp[tt] * fg[tt] * (1.f - fg[tt]);
      const float dog = dh[tt] * tc * og[tt] * (1.f - og[tt]);
      dc[tt] = dcv * fg[tt];
      if (!BIO && live[tt]) {
        float* gp = static_cast<float*>(a.dxg) + ((size_t)b[tt] * a.T + t) * G4 + j;
        gp[0] = di; gp[H] = dgg; gp[2 * H] = df; gp[3 * H] = dog;
      }
      const int row = tt * 16 + bb;
      dst[(row * 4 + 0) * 32 + jj] = f2bf(di);
      dst[(row * 4 + 1) * 32 + jj] = f2bf(dgg);
      dst[(row * 4 + 2) * 32 + jj] = f2bf(df);
      dst[(row * 4 + 3) * 32 + jj] = f2bf(dog);
    }
    __syncthreads();
    if (wave == 0) {   // publish R rows x 4 gates x 64 B; drained before the counter add
      const __amdgpu_buffer_rsrc_t r = rsrc(a.dg16 + t * slab, (int)(slab * 2));
#pragma unroll
      for (int k = 0; k < 4 * NT; ++k) {
        const int cidx = lane + 64 * k, row = cidx >> 4, gt = (cidx >> 2) & 3, qq = cidx & 3;
        if (row < nb) {
          const v4u gv = *reinterpret_cast<const v4u*>(dst + (row * 4 + gt) * 32 + qq * 8);
          st_sc1(gv, r, (int)(((b_lo + row) * G4 + gt * H + m * 32 + qq * 8) * 2));
          if constexpr (BIO)   // the input-projection gradient is the same bf16 dg: plain 16-byte store
            if (!(NT == 1 && a.late))
              *reinterpret_cast<v4u*>(static_cast<bf16_t*>(a.dxg) + ((size_t)(b_lo + row) * a.T + t) * G4 + gt * H +
                                      m * 32 + qq * 8) = gv;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) signal(cnt);
      if constexpr (BIO) {
        if (NT == 1 && a.late) {   // (as in the forward) the dxg copy behind the hand-off, re-read from LDS: the tile is not
                        // rewritten before this wave reaches the next step's barrier
#pragma unroll
          for (int k = 0; k < 4 * NT; ++k) {
            const int cidx = lane + 64 * k, row = cidx >> 4, gt = (cidx >> 2) & 3, qq = cidx & 3;
            if (row < nb)
              *reinterpret_cast<v4u*>(static_cast<bf16_t*>(a.dxg) + ((size_t)(b_lo + row) * a.T + t) * G4 + gt * H +
                                      m * 32 + qq * 8) = *reinterpret_cast<const v4u*>(dst + (row * 4 + gt) * 32 + qq * 8);
          }
        }
      }
    }
  }
#pragma unroll
  for (int tt = 0; tt < NT; ++tt)
    if (live[tt]) a.dc0[(size_t)b[tt] * H + j] = dc[tt];
}

// ------------------------------------------------------------------------------------------------ GRU
// Whole-sequence GRU recurrence, one persistent launch per direction (reference: the fused MKL-DNN RNN primitive
// with VanillaGru, S/nn/mkldnn/RNN.scala:213-219; cell S/nn/GRU.scala: r = s(x_r + U_r h), z = s(x_z + U_z h),
// n = tanh(x_n + U_n (r * h)), h' = (1 - z) n + z h). Same grid, group / member split, write-through hand-off and
// bounded waits as the LSTM kernels above; a GRU step has TWO dependent recurrent GEMMs (the candidate's operand
// r * h spans every unit), so every step makes two hand-offs through the group counter (2 M signals per step).
// Forward, member m (units 32 m .. + 31), 8 waves:
//   rz GEMM (K = H): wave w owns rz tile w & 3 (16 member-local rows = 8 units x {r, z}) over K half w >> 2;
//   n  GEMM (K = H): wave w owns unit tile w & 1 (16 units) over K quarter w >> 1;
//   W fragments for both stay in VGPRs (H = 1024: 16 + 8 fragments = 96 VGPRs); partials meet in LDS.
// A thread (unit uu = tid >> 4, batch bb = tid & 15) keeps h_{t-1} in fp32 across steps.
// Backward (reverse sweep + one round for dh0 = drz_0 U_rz): S2 (K = 2H) dh = drz_{t+1} U_rz + carried z / r paths
// + dout -> dz, dn (hand-off of dn) ; S1 (K = H) d(r h) = dn U_n -> dr, r-path of dh_{t-1} (hand-off of drz_t).
struct GruSeqArgs {
  const bf16_t* Wrz16;   // [2H][H] gate blocks r, z
  const bf16_t* Wn16;    // [H][H]
  const float* xg;       // fwd: [B][T][3H] preTopology output (r | z | n)
  const float* h0;       // [B][H] or null
  bf16_t* h16;           // [T + 1][B][H]: h_{-1} .. h_{T-1} (bf16 operands, row 0 filled by the host)
  bf16_t* rh16;          // [T][B][H]: r * h_{t-1} (the candidate GEMM operand)
  float* gates;          // [3][T][B][H] r, z, n
  float* out;            // fwd: [B][T][H]
  const float* dout;     // bwd: [B][T][H] or null
  const float* dhT;      // bwd: [B][H] or null
  float* dx;             // bwd: [B][T][3H]
  bf16_t* dn16;          // bwd: [T][B][H]
  bf16_t* drz16;         // bwd: [T][B][2H] (dr | dz)
  float* dh0;            // bwd: [B][H]
  unsigned* sync;
  unsigned* herr;
  unsigned long long spin;
  int B, H, T, Bg;
};

__device__ __forceinline__ bool gru_wait(unsigned* cnt, unsigned target, const GruSeqArgs& a, int* flag, int wave,
                                         int lane) {
  if (wave == 0 && lane == 0) *flag = wait_count(cnt, target, a.sync + NGRP * CNT_STRIDE, a.herr, a.spin) ? 0 : 1;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
  return *flag == 0;
}

// rows x (K) bf16 of one time step, group rows [b_lo, b_lo + nb) -> LDS image [16][K + 8] (sc1 loads; rows past the
// group read as zero)
template <int K>
__device__ __forceinline__ void stage_rows(bf16_t* dstl, const bf16_t* src, int nb, int tid) {
  constexpr int KP = K + 8, CH = 16 * K / 8 / 512, U = CH < 4 ? CH : 4;
  const __amdgpu_buffer_rsrc_t r = rsrc(src, nb * K * 2);
#pragma unroll
  for (int h = 0; h < CH; h += U) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = tid + 512 * (h + u), row = q / (K / 8), c8 = q % (K / 8);
      v[u] = ld_sc1(r, (row * K + c8 * 8) * 2);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int q = tid + 512 * (h + u), row = q / (K / 8), c8 = q % (K / 8);
      *reinterpret_cast<v4u*>(dstl + row * KP + c8 * 8) = v[u];
    }
  }
}

// publish a 16 x 32 bf16 slice (LDS [16][32]) to dst rows b_lo.. (row stride ld elements) at column col0; wave 0
// only, drained before the counter add
__device__ __forceinline__ void publish_slice(const bf16_t* sl, bf16_t* dst, size_t dst_elems, int ld, int col0,
                                              int b_lo, int nb, int lane, unsigned* cnt) {
  const __amdgpu_buffer_rsrc_t r = rsrc(dst, (int)(dst_elems * 2));
  const int row = lane >> 2, qq = lane & 3;
  if (row < nb) {
    const v4u hv = *reinterpret_cast<const v4u*>(sl + row * 32 + qq * 8);
    st_sc1(hv, r, (int)(((b_lo + row) * ld + col0 + qq * 8) * 2));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) signal(cnt);
}

template <int KS>
__global__ __launch_bounds__(512, 1) void gru_seq_fwd_kernel(GruSeqArgs a) {
  constexpr int H = KS * 32, HP = H + 8;
  constexpr int KH = KS / 2, KQ = KS / 4;        // fragments per wave: rz (K half), n (K quarter)
  __shared__ __attribute__((aligned(16))) bf16_t hs[16 * HP];
  __shared__ float red_rz[2][64][17];
  __shared__ float red_n[4][32][17];
  __shared__ __attribute__((aligned(16))) bf16_t sl[16 * 32];
  __shared__ int flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x % NGRP, m = blockIdx.x / NGRP, M = gridDim.x / NGRP;
  const int b_lo = g * a.Bg, nb = min(a.Bg, a.B - b_lo);
  if (nb <= 0) return;
  const int G = lane >> 4, col = lane & 15;
  // rz role: local row lr = 16 rt + (lane & 15): unit 8 rt + (lr >> 1) of the member, gate lr & 1
  const int rt = wave & 3, kh = wave >> 2;
  // n role
  const int nt = wave & 1, kq = wave >> 1;
  v8s wrz[KH], wn[KQ];
  {
    const int lr = (col);
    const int unit = m * 32 + 8 * rt + (lr >> 1), gate = lr & 1;
    const bf16_t* wp = a.Wrz16 + (size_t)(gate * H + unit) * H + kh * (H / 2) + 8 * G;
#pragma unroll
    for (int s = 0; s < KH; ++s) wrz[s] = *reinterpret_cast<const v8s*>(wp + s * 32);
    const bf16_t* wq = a.Wn16 + (size_t)(m * 32 + 16 * nt + col) * H + kq * (H / 4) + 8 * G;
#pragma unroll
    for (int s = 0; s < KQ; ++s) wn[s] = *reinterpret_cast<const v8s*>(wq + s * 32);
  }
  // cell thread
  const int uu = tid >> 4, bb = tid & 15;
  const int j = m * 32 + uu;
  const bool live = bb < nb;
  const int b = b_lo + (live ? bb : 0);
  float hp = a.h0 ? a.h0[(size_t)b * H + j] : 0.f;
  unsigned* cnt = a.sync + g * CNT_STRIDE;
  const size_t slab = (size_t)a.B * H;
  const size_t gslab = (size_t)a.T * a.B * H;

  for (int t = 0; t < a.T; ++t) {
    const float* xp = a.xg + ((size_t)b * a.T + t) * 3 * H + j;
    const float xr = xp[0], xz = xp[H], xn = xp[2 * H];
    if (t > 0 && !gru_wait(cnt, (unsigned)(2 * M * t), a, &flag, wave, lane)) {
      if (live)
        for (int u = t; u < a.T; ++u) {
          a.out[((size_t)b * a.T + u) * H + j] = __builtin_nanf("");
          a.h16[(u + 1) * slab + (size_t)b * H + j] = 0x7fc0;
          a.rh16[u * slab + (size_t)b * H + j] = 0x7fc0;
          for (int k = 0; k < 3; ++k) a.gates[k * gslab + ((size_t)u * a.B + b) * H + j] = __builtin_nanf("");
        }
      return;
    }
    stage_rows<H>(hs, a.h16 + t * slab + (size_t)b_lo * H, nb, tid);
    __syncthreads();
    {   // rz GEMM partials
      v4f acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const bf16_t* hb = hs + col * HP + kh * (H / 2) + 8 * G;
#pragma unroll
      for (int s = 0; s < KH; s += 2) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wrz[s], *reinterpret_cast<const v8s*>(hb + s * 32), acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wrz[s + 1], *reinterpret_cast<const v8s*>(hb + (s + 1) * 32), acc1, 0, 0, 0);
      }
      const v4f p = acc0 + acc1;
#pragma unroll
      for (int e = 0; e < 4; ++e) red_rz[kh][16 * rt + 4 * G + e][col] = p[e];
    }
    __syncthreads();
    // local rz row of (unit uu, gate q): 16 (uu >> 3) + 2 (uu & 7) + q
    const int lr0 = 16 * (uu >> 3) + 2 * (uu & 7);
    const float r = sigm(red_rz[0][lr0][bb] + red_rz[1][lr0][bb] + xr);
    const float z = sigm(red_rz[0][lr0 + 1][bb] + red_rz[1][lr0 + 1][bb] + xz);
    sl[bb * 32 + uu] = f2bf(r * hp);
    if (live) {
      a.gates[((size_t)t * a.B + b) * H + j] = r;
      a.gates[gslab + ((size_t)t * a.B + b) * H + j] = z;
    }
    __syncthreads();
    if (wave == 0) publish_slice(sl, a.rh16 + t * slab, slab, H, m * 32, b_lo, nb, lane, cnt);
    if (!gru_wait(cnt, (unsigned)(2 * M * t + M), a, &flag, wave, lane)) {
      if (live)
        for (int u = t; u < a.T; ++u) {
          a.out[((size_t)b * a.T + u) * H + j] = __builtin_nanf("");
          a.h16[(u + 1) * slab + (size_t)b * H + j] = 0x7fc0;
          a.gates[2 * gslab + ((size_t)u * a.B + b) * H + j] = __builtin_nanf("");
        }
      return;
    }
    stage_rows<H>(hs, a.rh16 + t * slab + (size_t)b_lo * H, nb, tid);
    __syncthreads();
    {   // n GEMM partials
      v4f acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const bf16_t* hb = hs + col * HP + kq * (H / 4) + 8 * G;
#pragma unroll
      for (int s = 0; s < KQ; s += 2) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wn[s], *reinterpret_cast<const v8s*>(hb + s * 32), acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wn[s + 1], *reinterpret_cast<const v8s*>(hb + (s + 1) * 32), acc1, 0, 0, 0);
      }
      const v4f p = acc0 + acc1;
#pragma unroll
      for (int e = 0; e < 4; ++e) red_n[kq][16 * nt + 4 * G + e][col] = p[e];
    }
    __syncthreads();
    const float n = tanh_f(red_n[0][uu][bb] + red_n[1][uu][bb] + red_n[2][uu][bb] + red_n[3][uu][bb] + xn);
    const float h = (1.f - z) * n + z * hp;
    hp = h;
    if (live) {
      a.gates[2 * gslab + ((size_t)t * a.B + b) * H + j] = n;
      a.out[((size_t)b * a.T + t) * H + j] = h;
    }
    sl[bb * 32 + uu] = f2bf(h);
    __syncthreads();
    if (wave == 0) publish_slice(sl, a.h16 + (t + 1) * slab, slab, H, m * 32, b_lo, nb, lane, cnt);
  }
}

template <int KS>
__global__ __launch_bounds__(512, 1) void gru_seq_bwd_kernel(GruSeqArgs a) {
  constexpr int H = KS * 32, H2 = 2 * H;
  constexpr int DP = H2 + 8;                     // LDS row pitch of the drz image (the dn image uses H + 8)
  constexpr int K2 = (2 * KS) / 4, K1 = KS / 4;  // fragments per wave: S2 (K = 2H quarter), S1 (K = H quarter)
  __shared__ __attribute__((aligned(16))) bf16_t ds[16 * DP];
  __shared__ float red[4][32][17];
  __shared__ __attribute__((aligned(16))) bf16_t sl[16 * 32];
  __shared__ __attribute__((aligned(16))) bf16_t sl2[16 * 64];
  __shared__ int flag;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = blockIdx.x % NGRP, m = blockIdx.x / NGRP, M = gridDim.x / NGRP;
  const int b_lo = g * a.Bg, nb = min(a.Bg, a.B - b_lo);
  if (nb <= 0) return;
  const int G = lane >> 4, col = lane & 15;
  const int ut = wave & 1, kq = wave >> 1;       // unit tile (16 units), K quarter
  const int unit = m * 32 + 16 * ut + col;       // A row of this lane's fragments
  v8s w2[K2], w1[K1];
  {   // A[unit][k] = Urz[k][unit] (k in this wave's quarter of 2H), Un[k][unit] (quarter of H): gathered once
    const bf16_t* wp = a.Wrz16 + (size_t)(kq * (H2 / 4) + 8 * G) * H + unit;
#pragma unroll
    for (int s = 0; s < K2; ++s) {
      v4u f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        f[i] = (unsigned)wp[(size_t)(s * 32 + 2 * i) * H] | ((unsigned)wp[(size_t)(s * 32 + 2 * i + 1) * H] << 16);
      asm volatile("" : "+v"(f) :: "memory");
      w2[s] = __builtin_bit_cast(v8s, f);
    }
    const bf16_t* wq = a.Wn16 + (size_t)(kq * (H / 4) + 8 * G) * H + unit;
#pragma unroll
    for (int s = 0; s < K1; ++s) {
      v4u f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        f[i] = (unsigned)wq[(size_t)(s * 32 + 2 * i) * H] | ((unsigned)wq[(size_t)(s * 32 + 2 * i + 1) * H] << 16);
      asm volatile("" : "+v"(f) :: "memory");
      w1[s] = __builtin_bit_cast(v8s, f);
    }
  }
  const int uu = tid >> 4, bb = tid & 15;
  const int j = m * 32 + uu;
  const bool live = bb < nb;
  const int b = b_lo + (live ? bb : 0);
  float dhp = a.dhT ? a.dhT[(size_t)b * H + j] : 0.f;   // carried z- / r-paths of dh (plus dhT at the start)
  unsigned* cnt = a.sync + g * CNT_STRIDE;
  const size_t slab = (size_t)a.B * H;
  const size_t gslab = (size_t)a.T * a.B * H;

  for (int i = 0; i <= a.T; ++i) {
    const int t = a.T - 1 - i;
    float S2 = 0.f;
    if (i > 0) {   // S2 = drz_{t+1} . U_rz for (unit j, batch b)
      if (!gru_wait(cnt, (unsigned)(2 * M * i), a, &flag, wave, lane)) {
        if (live) {
          for (int u = t; u >= 0; --u) {
            float* dx = a.dx + ((size_t)b * a.T + u) * 3 * H + j;
            dx[0] = dx[H] = dx[2 * H] = __builtin_nanf("");
            a.dn16[u * slab + (size_t)b * H + j] = 0x7fc0;
            a.drz16[(size_t)u * a.B * H2 + (size_t)b * H2 + j] = 0x7fc0;
            a.drz16[(size_t)u * a.B * H2 + (size_t)b * H2 + H + j] = 0x7fc0;
          }
          a.dh0[(size_t)b * H + j] = __builtin_nanf("");
        }
        return;
      }
      {
        constexpr int CH = 16 * H2 / 8 / 512, U = CH < 4 ? CH : 4;
        const __amdgpu_buffer_rsrc_t r = rsrc(a.drz16 + (size_t)(t + 1) * a.B * H2 + (size_t)b_lo * H2, nb * H2 * 2);
#pragma unroll
        for (int h = 0; h < CH; h += U) {
          v4u v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int q = tid + 512 * (h + u), row = q / (H2 / 8), c8 = q % (H2 / 8);
            v[u] = ld_sc1(r, (row * H2 + c8 * 8) * 2);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int q = tid + 512 * (h + u), row = q / (H2 / 8), c8 = q % (H2 / 8);
            *reinterpret_cast<v4u*>(ds + row * DP + c8 * 8) = v[u];
          }
        }
      }
      __syncthreads();
      v4f acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const bf16_t* db = ds + col * DP + kq * (H2 / 4) + 8 * G;
#pragma unroll
      for (int s = 0; s < K2; s += 2) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2[s], *reinterpret_cast<const v8s*>(db + s * 32), acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w2[s + 1], *reinterpret_cast<const v8s*>(db + (s + 1) * 32), acc1, 0, 0, 0);
      }
      const v4f p = acc0 + acc1;
#pragma unroll
      for (int e = 0; e < 4; ++e) red[kq][16 * ut + 4 * G + e][col] = p[e];
      __syncthreads();
      S2 = red[0][uu][bb] + red[1][uu][bb] + red[2][uu][bb] + red[3][uu][bb];
    }
    if (t < 0) {   // final round: dh0 = drz_0 . U_rz + carried paths
      if (live) a.dh0[(size_t)b * H + j] = S2 + dhp;
      break;
    }
    const size_t go = ((size_t)t * a.B + b) * H + j;
    const float r = a.gates[go], z = a.gates[gslab + go], n = a.gates[2 * gslab + go];
    const float hprev = t > 0 ? a.out[((size_t)b * a.T + (t - 1)) * H + j] : (a.h0 ? a.h0[(size_t)b * H + j] : 0.f);
    float dh = S2 + dhp;
    if (a.dout) dh += a.dout[((size_t)b * a.T + t) * H + j];
    const float dn = dh * (1.f - z) * (1.f - n * n);
    const float dz = dh * (hprev - n) * z * (1.f - z);
    dhp = dh * z;                                  // z-path of dh_{t-1}
    float* dx = a.dx + ((size_t)b * a.T + t) * 3 * H + j;
    if (live) { dx[H] = dz; dx[2 * H] = dn; }
    sl[bb * 32 + uu] = f2bf(dn);
    __syncthreads();
    if (wave == 0) publish_slice(sl, a.dn16 + t * slab, slab, H, m * 32, b_lo, nb, lane, cnt);
    if (!gru_wait(cnt, (unsigned)(2 * M * i + M), a, &flag, wave, lane)) {
      if (live) {
        for (int u = t; u >= 0; --u) {
          float* dxx = a.dx + ((size_t)b * a.T + u) * 3 * H + j;
          dxx[0] = __builtin_nanf("");
          a.drz16[(size_t)u * a.B * H2 + (size_t)b * H2 + j] = 0x7fc0;
          a.drz16[(size_t)u * a.B * H2 + (size_t)b * H2 + H + j] = 0x7fc0;
        }
        a.dh0[(size_t)b * H + j] = __builtin_nanf("");
      }
      return;
    }
    stage_rows<H>(ds, a.dn16 + t * slab + (size_t)b_lo * H, nb, tid);   // [16][H + 8] image in the same buffer
    __syncthreads();
    {
      v4f acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      const bf16_t* db = ds + col * (H + 8) + kq * (H / 4) + 8 * G;
#pragma unroll
      for (int s = 0; s < K1; s += 2) {
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[s], *reinterpret_cast<const v8s*>(db + s * 32), acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w1[s + 1], *reinterpret_cast<const v8s*>(db + (s + 1) * 32), acc1, 0, 0, 0);
      }
      const v4f p = acc0 + acc1;
#pragma unroll
      for (int e = 0; e < 4; ++e) red[kq][16 * ut + 4 * G + e][col] = p[e];
    }
    __syncthreads();
    const float drh = red[0][uu][bb] + red[1][uu][bb] + red[2][uu][bb] + red[3][uu][bb];
    const float dr = drh * hprev * r * (1.f - r);
    dhp += drh * r;                                // r-path of dh_{t-1}
    if (live) dx[0] = dr;
    sl2[bb * 64 + uu] = f2bf(dr);
    sl2[bb * 64 + 32 + uu] = f2bf(dz);
    __syncthreads();
    if (wave == 0) {   // drz_t slice: dr at columns 32 m.., dz at H + 32 m..
      const __amdgpu_buffer_rsrc_t rr = rsrc(a.drz16 + (size_t)t * a.B * H2, (int)((size_t)a.B * H2 * 2));
      const int row = lane >> 2, qq = lane & 3;
      if (row < nb) {
        const v4u v0 = *reinterpret_cast<const v4u*>(sl2 + row * 64 + qq * 8);
        const v4u v1 = *reinterpret_cast<const v4u*>(sl2 + row * 64 + 32 + qq * 8);
        st_sc1(v0, rr, (int)(((b_lo + row) * H2 + m * 32 + qq * 8) * 2));
        st_sc1(v1, rr, (int)(((b_lo + row) * H2 + H + m * 32 + qq * 8) * 2));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) signal(cnt);
    }
  }
}

int g_lstm_seq = -1;   // BIGDL_LSTM_SEQ: 1 (default) persistent whole-sequence kernels, 0 = per-step kernels
int seq_enabled() {
  if (g_lstm_seq < 0) {
    const char* e = getenv("BIGDL_LSTM_SEQ");
    g_lstm_seq = e ? atoi(e) : 1;
  }
  return g_lstm_seq;
}

int cu_count() {
  static const int n = [] {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return cus;
  }();
  return n;
}

// Occupancy of every instantiation the launch may pick for this H: at least one 512-thread workgroup per CU.
template <int KS, int NT>
bool occ_ok_ks() {
  static const bool ok = [] {
    int n = 0;
    const void* ks[4] = {reinterpret_cast<const void*>(&lstm_seq_fwd_kernel<KS, true, NT>),
                         reinterpret_cast<const void*>(&lstm_seq_fwd_kernel<KS, false, NT>),
                         reinterpret_cast<const void*>(&lstm_seq_bwd_kernel<KS, true, NT>),
                         reinterpret_cast<const void*>(&lstm_seq_bwd_kernel<KS, false, NT>)};
    for (const void* k : ks) {
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 512, 0) != hipSuccess || n < 1) return false;
    }
    return true;
  }();
  return ok;
}

bool seq_shape_ok(int B, int H) {
  if (!seq_enabled() || B <= 0 || (H != 256 && H != 512 && H != 1024)) return false;
  const int bg = (B + NGRP - 1) / NGRP;
  if (bg > 32) return false;                         // two 16-row batch tiles per group at most
  if (NGRP * (H / 32) > cu_count()) return false;   // one workgroup per CU, all resident
  bool occ;
  if (bg > 16) occ = H == 1024 ? occ_ok_ks<32, 2>() : H == 512 ? occ_ok_ks<16, 2>() : occ_ok_ks<8, 2>();
  else occ = H == 1024 ? occ_ok_ks<32, 1>() : H == 512 ? occ_ok_ks<16, 1>() : occ_ok_ks<8, 1>();
  return occ && host_err_dev() != nullptr;
}

template <int KS>
bool gru_occ_ok() {
  static const bool ok = [] {
    int n = 0;
    const void* ks[2] = {reinterpret_cast<const void*>(&gru_seq_fwd_kernel<KS>),
                         reinterpret_cast<const void*>(&gru_seq_bwd_kernel<KS>)};
    for (const void* k : ks)
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 512, 0) != hipSuccess || n < 1) return false;
    return true;
  }();
  return ok;
}

bool gru_shape_ok(int B, int H) {
  if (!seq_enabled() || B <= 0 || (H != 256 && H != 512 && H != 1024)) return false;
  if ((B + NGRP - 1) / NGRP > 16) return false;
  if (NGRP * (H / 32) > cu_count()) return false;
  const bool occ = H == 1024 ? gru_occ_ok<32>() : H == 512 ? gru_occ_ok<16>() : gru_occ_ok<8>();
  return occ && host_err_dev() != nullptr;
}

}  // namespace

extern "C" {

int bigdl_gru_seq_supported(int B, int H) { return gru_shape_ok(B, H) ? 1 : 0; }

int bigdl_gru_seq(int bwd, const uint16_t* Wrz16, const uint16_t* Wn16, const float* xg, const float* h0,
                  uint16_t* h16, uint16_t* rh16, float* gates, float* out, const float* dout, const float* dhT,
                  float* dx, uint16_t* dn16, uint16_t* drz16, float* dh0, unsigned* sync, int B, int H, int T,
                  hipStream_t st) {
  if (!gru_shape_ok(B, H) || T <= 0) return -1;
  GruSeqArgs a{};
  a.Wrz16 = Wrz16; a.Wn16 = Wn16; a.xg = xg; a.h0 = h0; a.h16 = h16; a.rh16 = rh16; a.gates = gates; a.out = out;
  a.dout = dout; a.dhT = dhT; a.dx = dx; a.dn16 = dn16; a.drz16 = drz16; a.dh0 = dh0; a.sync = sync;
  a.B = B; a.H = H; a.T = T; a.Bg = (B + NGRP - 1) / NGRP;
  a.herr = host_err_dev(); a.spin = g_spin_ticks;
  bigdl_fill_bytes(sync, 0, (long)sizeof(unsigned) * bigdl_lstm_seq_sync_words(), st);   // kernel: graph-safe
  const dim3 grid(NGRP * (H / 32));
#define GRU_L(K) do { if (bwd) gru_seq_bwd_kernel<K><<<grid, 512, 0, st>>>(a); else gru_seq_fwd_kernel<K><<<grid, 512, 0, st>>>(a); } while (0)
  if (H == 1024) GRU_L(32);
  else if (H == 512) GRU_L(16);
  else GRU_L(8);
#undef GRU_L
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_lstm_seq_supported(int B, int H) { return seq_shape_ok(B, H) ? 1 : 0; }
void bigdl_set_lstm_seq(int v) { g_lstm_seq = v; }
int bigdl_lstm_seq_sync_words() { return NGRP * CNT_STRIDE + CNT_STRIDE; }

// Timeouts recorded by persistent kernels since the last clear (host-mapped word: no device synchronisation).
int bigdl_persistent_error(int clear) { return bigdl_host_word(0, clear); }
// Process-wide host-mapped words (16 x 4 B, fine-grained): slot 0 persistent-kernel timeouts, slot 1 index-range
// errors of the TensorMath index kernels. Device address for kernels; host reads need no synchronisation.
unsigned* bigdl_host_word_dev(int slot) {
  unsigned* d = host_err_dev();
  return (d && slot >= 0 && slot < 16) ? d + slot : nullptr;
}
int bigdl_host_word(int slot, int clear) {
  if (g_herr_host == nullptr || slot < 0 || slot >= 16) return 0;
  volatile unsigned* p = g_herr_host + slot;
  const unsigned v = *p;
  if (clear && v) *p = 0u;
  return (int)v;
}
// Bound of every persistent-kernel wait (tests force a timeout with a small value); <= 0 restores the default.
void bigdl_set_seq_timeout_us(double us) { g_spin_ticks = us > 0 ? (unsigned long long)(us * 100.0) : 200000000ull; }
unsigned* bigdl_persistent_err_dev() { return host_err_dev(); }
unsigned long long bigdl_seq_spin_ticks() { return g_spin_ticks; }

int bigdl_lstm_seq_fwd(const uint16_t* W16, const void* xg, const float* c0, uint16_t* h16, void* out, float* hT,
                       float* cs, float* acts, unsigned* sync, int B, int H, int T, int bf16io, hipStream_t st) {
  if (!seq_shape_ok(B, H) || T <= 0) return -1;
  LstmSeqArgs a{};
  a.W16 = W16; a.xg = xg; a.c0 = c0; a.h16 = h16; a.out = out; a.hT = hT; a.cs = cs; a.acts = acts; a.sync = sync;
  a.B = B; a.H = H; a.T = T; a.Bg = (B + NGRP - 1) / NGRP;
  a.herr = host_err_dev(); a.spin = g_spin_ticks;
  static const int late = [] { const char* e = getenv("BIGDL_LSTM_LATE"); return e ? atoi(e) : 1; }();
  a.late = late;
  bigdl_fill_bytes(sync, 0, (long)sizeof(unsigned) * bigdl_lstm_seq_sync_words(), st);   // kernel: graph-safe
  const dim3 grid(NGRP * (H / 32));
#define SEQ_FWD(K)                                                                       \
  do {                                                                                   \
    if (a.Bg > 16) {                                                                     \
      if (bf16io) lstm_seq_fwd_kernel<K, true, 2><<<grid, 512, 0, st>>>(a);             \
      else lstm_seq_fwd_kernel<K, false, 2><<<grid, 512, 0, st>>>(a);                   \
    } else {                                                                             \
      if (bf16io) lstm_seq_fwd_kernel<K, true, 1><<<grid, 512, 0, st>>>(a);             \
      else lstm_seq_fwd_kernel<K, false, 1><<<grid, 512, 0, st>>>(a);                   \
    }                                                                                    \
  } while (0)
  if (H == 1024) SEQ_FWD(32);
  else if (H == 512) SEQ_FWD(16);
  else SEQ_FWD(8);
#undef SEQ_FWD
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_lstm_seq_bwd(const uint16_t* W16, const void* dout, const float* dhT, const float* dcT, const float* acts,
                       const float* cs, const float* c0, uint16_t* dg16, void* dxg, float* dc0, float* dh0,
                       unsigned* sync, int B, int H, int T, int bf16io, hipStream_t st) {
  if (!seq_shape_ok(B, H) || T <= 0) return -1;
  LstmSeqArgs a{};
  a.W16 = W16; a.dout = dout; a.dhT = dhT; a.dcT = dcT; a.acts = const_cast<float*>(acts);
  a.cs = const_cast<float*>(cs); a.c0 = c0; a.dg16 = dg16; a.dxg = dxg; a.dc0 = dc0; a.dh0 = dh0; a.sync = sync;
  a.B = B; a.H = H; a.T = T; a.Bg = (B + NGRP - 1) / NGRP;
  a.herr = host_err_dev(); a.spin = g_spin_ticks;
  static const int late = [] { const char* e = getenv("BIGDL_LSTM_LATE"); return e ? atoi(e) : 1; }();
  a.late = late;
  bigdl_fill_bytes(sync, 0, (long)sizeof(unsigned) * bigdl_lstm_seq_sync_words(), st);   // kernel: graph-safe
  const dim3 grid(NGRP * (H / 32));
#define SEQ_BWD(K)                                                                       \
  do {                                                                                   \
    if (a.Bg > 16) {                                                                     \
      if (bf16io) lstm_seq_bwd_kernel<K, true, 2><<<grid, 512, 0, st>>>(a);             \
      else lstm_seq_bwd_kernel<K, false, 2><<<grid, 512, 0, st>>>(a);                   \
    } else {                                                                             \
      if (bf16io) lstm_seq_bwd_kernel<K, true, 1><<<grid, 512, 0, st>>>(a);             \
      else lstm_seq_bwd_kernel<K, false, 1><<<grid, 512, 0, st>>>(a);                   \
    }                                                                                    \
  } while (0)
  if (H == 1024) SEQ_BWD(32);
  else if (H == 512) SEQ_BWD(16);
  else SEQ_BWD(8);
#undef SEQ_BWD
  HIP_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
