// Fused LSTM time-step kernels for gfx950: one launch per step does the recurrent GEMM on the bf16 MFMA
// and the whole cell (forward) / cell backward + next recurrent-gradient GEMM (backward).
//
// Reference: S/nn/LSTM.scala:77-185 (gates i, g, f, o; c' = f*c + i*g; h' = o*tanh(c')), recurrent loop
// S/nn/Recurrent.scala:283-305, fused whole-sequence MKL-DNN RNN S/nn/mkldnn/RNN.scala:36-501.
//
// Why one launch per step and not a persistent kernel: every step is an all-to-all seam (each workgroup needs
// the whole h_{t-1}); on MI355X a grid barrier costs ~4-5 us at 256 workgroups vs ~1.5 us for a kernel
// boundary (MI355X_MICROARCH price list: barrier-xcd vs boundary), and the HIP-graph-captured step loop has no
// host overhead. What the fusion removes is everything else: the gate pre-activations never touch HBM, the
// cell math runs in the GEMM epilogue, and the weight slice each workgroup reads is the same every step, so
// it stays hot in that XCD's L2.
//
// Both steps are bound by reading the previous step's bf16 state (h_{t-1} or dg_{t+1}) written on all XCDs,
// so tiles are sized to cut that cross-XCD traffic (measured with tools/lstm_micro.py):
// Forward step, workgroup = 16 hidden units x 16 batch rows: MFMA 16x16x32 bf16, A = gate rows of W ordered
//   row = unit*4 + gate, B = h_{t-1}^T; the 4 gates of a (unit, batch) pair meet in LDS, the cell math runs
//   coalesced along the hidden dimension, c stays fp32.
// Backward step, workgroup = 16 batch rows x 64 hidden units: dh_t = dout_t + dg_{t+1} . W as
//   D[batch][unit] = A(dg16 rows) x B(W^T rows), then the cell backward of each (batch, unit) pair emits
//   dg_t (fp32 for the weight-gradient GEMM, bf16 as the next step's A operand) and dc_{t-1} (in place).
#include "common.h"
#include "kernels.h"

namespace {

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  const float e = __expf(-2.f * fabsf(x));
  const float t = (1.f - e) / (1.f + e);
  return x < 0.f ? -t : t;
}

__device__ __forceinline__ v8s ld8(const bf16_t* p) { return *(const v8s*)p; }

// K is consumed in groups of 8 k-steps whose loads are all issued before the group's MFMAs, so a wave pays about
// one memory round trip per group; the step kernels split K over many waves so that each wave has one or two groups
// (a long per-wave chain of L2/MALL round trips was the measured bottleneck, tools/lstm_micro.py).

// K-split factor: chunks of >= 256 (8 k-steps), at most `cap` waves per output tile.
__host__ __device__ inline int ksplit(int K, int cap) {
  int ks = K / 256;
  if (ks < 1) ks = 1;
  if (ks > cap) ks = cap;
  while (ks > 1 && (K % (ks * 32)) != 0) --ks;
  return ks;
}

// NS x NV output tiles: acc[i][n] += S[i] x V[n] (SFIRST: S is the MFMA's first operand) over K, every fragment
// loaded once per k-step and used by all the tiles of its row / column (NV = 2 halves the weight traffic per output).
template <int NS, int NV, bool SFIRST>
__device__ __forceinline__ void mfma_tiles(const bf16_t* const (&ps)[NS], const bf16_t* const (&pv)[NV], int K,
                                           v4f (&acc)[NS][NV]) {
  constexpr int CH = NS * NV > 2 ? 4 : 8;
  const int steps = K / 32, full = steps / CH * CH;
  for (int s = 0; s < full; s += CH) {
    v8s a[NS][CH], b[NV][CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
#pragma unroll
      for (int u = 0; u < NS; ++u) a[u][i] = ld8(ps[u] + (s + i) * 32);
#pragma unroll
      for (int n = 0; n < NV; ++n) b[n][i] = ld8(pv[n] + (s + i) * 32);
    }
#pragma unroll
    for (int i = 0; i < CH; ++i)
#pragma unroll
      for (int u = 0; u < NS; ++u)
#pragma unroll
        for (int n = 0; n < NV; ++n)
          acc[u][n] = SFIRST ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u][i], b[n][i], acc[u][n], 0, 0, 0)
                             : __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[n][i], a[u][i], acc[u][n], 0, 0, 0);
  }
  for (int s = full; s < steps; ++s) {
    v8s a[NS], b[NV];
#pragma unroll
    for (int u = 0; u < NS; ++u) a[u] = ld8(ps[u] + s * 32);
#pragma unroll
    for (int n = 0; n < NV; ++n) b[n] = ld8(pv[n] + s * 32);
#pragma unroll
    for (int u = 0; u < NS; ++u)
#pragma unroll
      for (int n = 0; n < NV; ++n)
        acc[u][n] = SFIRST ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b[n], acc[u][n], 0, 0, 0)
                           : __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[n], a[u], acc[u][n], 0, 0, 0);
  }
}

// Forward step. Workgroup = 16 hidden units x 16 batch rows, 4*KS waves: wave w owns units j0+4(w&3)..+3 as
// one 16-row MFMA tile (row = unit*4 + gate) over K chunk w>>2; all waves of a chunk share the batch tile's
// h_{t-1} fragments (L1). The 64 gate rows a workgroup reads are the same every step (L2-resident on its
// XCD). Gates are summed over the K chunks in LDS, then the cell update and all its loads / stores run
// coalesced along the hidden dimension (16 consecutive units per batch row).
template <int NB>
__global__ void __launch_bounds__(1024) lstm_fwd_step_kernel(
    const bf16_t* __restrict__ W16, const bf16_t* __restrict__ h16_prev, const float* __restrict__ xg, long ldx,
    const float* __restrict__ c_prev, float* __restrict__ c_out, float* __restrict__ h_out, long ldh,
    bf16_t* __restrict__ h16_out, float* __restrict__ acts, long lda, int B, int H, int KS) {
  __shared__ float gl[NB][4][16][16][5];                     // [batch tile][K chunk][batch][unit][gate] (+1 pad)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kh = lane >> 4;
  const int mt = wave & 3, kc = wave >> 2;
  const int j0 = blockIdx.x * 16, b0 = blockIdx.y * 16 * NB;
  const bool cell = threadIdx.x < 256 * NB;
  // cell element of threads 0..256*NB-1: (batch b0 + 16 * tile + m, unit j0 + n); operands loaded before the GEMM
  const int tile = threadIdx.x >> 8;
  const int m = (threadIdx.x >> 4) & 15, n = threadIdx.x & 15;
  const int b = b0 + tile * 16 + m, j = j0 + n;
  const bool live = cell && b < B;
  const int bs = b < B ? b : 0;
  float x0 = 0.f, x1 = 0.f, x2 = 0.f, x3 = 0.f, cp = 0.f;
  if (cell) {
    const float* x = xg + (long)bs * ldx + j;
    x0 = x[0]; x1 = x[H]; x2 = x[2 * H]; x3 = x[3 * H];
    cp = c_prev != nullptr ? c_prev[(long)bs * H + j] : 0.f;
  }
  v4f acc[1][NB];
#pragma unroll
  for (int t = 0; t < NB; ++t) acc[0][t] = v4f{0.f, 0.f, 0.f, 0.f};
  if (h16_prev != nullptr) {
    const int kl = H / KS;
    const int grow = (r & 3) * H + j0 + mt * 4 + (r >> 2);          // A row r = unit*4 + gate
    // batch rows past B read row 0: a batch column only feeds its own output column, never stored
    const bf16_t* pv[NB];
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const int bl = b0 + t * 16 + r;
      pv[t] = h16_prev + (long)(bl < B ? bl : 0) * H + kc * kl + kh * 8;
    }
    const bf16_t* pw[1] = {W16 + (long)grow * H + kc * kl + kh * 8};
    mfma_tiles<1, NB, true>(pw, pv, kl, acc);
  }
#pragma unroll
  for (int t = 0; t < NB; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) gl[t][kc][r][mt * 4 + kh][i] = acc[0][t][i];   // D[row = unit*4+gate][col = batch]
  __syncthreads();
  if (!live) return;
  float g[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = 0.f;
    for (int k = 0; k < KS; ++k) v += gl[tile][k][m][n][i];
    g[i] = v;
  }
  const float ig = sigm(g[0] + x0), gg = tanh_f(g[1] + x1), fg = sigm(g[2] + x2), og = sigm(g[3] + x3);
  const float c = fg * cp + ig * gg;
  const float h = og * tanh_f(c);
  c_out[(long)b * H + j] = c;
  h_out[(long)b * ldh + j] = h;
  h16_out[(long)b * H + j] = f2bf(h);
  float* a = acts + (long)b * lda + j;
  a[0] = ig; a[H] = gg; a[2 * H] = fg; a[3 * H] = og;
}

// Forward step, fragment-shared form: workgroup = 16 hidden units (64 gate rows) x 16*NB batch rows, KS waves,
// wave kc owning K chunk kc of kl = H / KS. Per k-step a wave loads the 4 W fragments (row tiles mt = 0..3) and the
// NB h fragments once and issues 4*NB MFMAs, so no fragment is loaded twice inside the workgroup: per step the grid
// moves (H/16) * (B/16/NB) * (64 + 16 NB) rows of K instead of (H/16) * (B/16) * (64 + 4 * 16) (the per-step time
// tracks those bytes: tools/lstm_micro.py, ~0.12 us per MB at H = 1024).
template <int NB, int KSMAX>
__global__ void __launch_bounds__(1024) lstm_fwd_step_ws_kernel(
    const bf16_t* __restrict__ W16, const bf16_t* __restrict__ h16_prev, const float* __restrict__ xg, long ldx,
    const float* __restrict__ c_prev, float* __restrict__ c_out, float* __restrict__ h_out, long ldh,
    bf16_t* __restrict__ h16_out, float* __restrict__ acts, long lda, int B, int H, int KS) {
  __shared__ float gl[KSMAX][16 * NB][16][5];                // [K chunk][batch][unit][gate] (+1 pad)
  const int lane = threadIdx.x & 63, kc = threadIdx.x >> 6;
  const int r = lane & 15, kh = lane >> 4;
  const int j0 = blockIdx.x * 16, b0 = blockIdx.y * 16 * NB;
  const bool cell = threadIdx.x < 256 * NB;
  const int tile = threadIdx.x >> 8;
  const int m = (threadIdx.x >> 4) & 15, n = threadIdx.x & 15;
  const int b = b0 + tile * 16 + m, j = j0 + n;
  const bool live = cell && b < B;
  const int bs = b < B ? b : 0;
  float x0 = 0.f, x1 = 0.f, x2 = 0.f, x3 = 0.f, cp = 0.f;
  if (cell) {
    const float* x = xg + (long)bs * ldx + j;
    x0 = x[0]; x1 = x[H]; x2 = x[2 * H]; x3 = x[3 * H];
    cp = c_prev != nullptr ? c_prev[(long)bs * H + j] : 0.f;
  }
  v4f acc[4][NB];
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int t = 0; t < NB; ++t) acc[mt][t] = v4f{0.f, 0.f, 0.f, 0.f};
  if (h16_prev != nullptr) {
    const int kl = H / KS, steps = kl / 32;
    const bf16_t* pw[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)                                   // A row r = unit*4 + gate
      pw[mt] = W16 + (long)((r & 3) * H + j0 + mt * 4 + (r >> 2)) * H + kc * kl + kh * 8;
    const bf16_t* pv[NB];
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const int bl = b0 + t * 16 + r;        // batch rows past B read row 0: their columns are never stored
      pv[t] = h16_prev + (long)(bl < B ? bl : 0) * H + kc * kl + kh * 8;
    }
    constexpr int G = 4;
    int s = 0;
    for (; s + G <= steps; s += G) {
      v8s a[G][4], v[NB][G];
#pragma unroll
      for (int i = 0; i < G; ++i) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) a[i][mt] = ld8(pw[mt] + (s + i) * 32);
#pragma unroll
        for (int t = 0; t < NB; ++t) v[t][i] = ld8(pv[t] + (s + i) * 32);
      }
#pragma unroll
      for (int i = 0; i < G; ++i)
#pragma unroll
        for (int mt = 0; mt < 4; ++mt)
#pragma unroll
          for (int t = 0; t < NB; ++t)
            acc[mt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][mt], v[t][i], acc[mt][t], 0, 0, 0);
    }
    for (; s < steps; ++s) {
      v8s a[4], v[NB];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) a[mt] = ld8(pw[mt] + s * 32);
#pragma unroll
      for (int t = 0; t < NB; ++t) v[t] = ld8(pv[t] + s * 32);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int t = 0; t < NB; ++t)
          acc[mt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], v[t], acc[mt][t], 0, 0, 0);
    }
  }
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int t = 0; t < NB; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) gl[kc][t * 16 + r][mt * 4 + kh][i] = acc[mt][t][i];   // D[unit*4+gate][batch]
  __syncthreads();
  if (!live) return;
  float g[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = 0.f;
    for (int k = 0; k < KS; ++k) v += gl[k][tile * 16 + m][n][i];
    g[i] = v;
  }
  const float ig = sigm(g[0] + x0), gg = tanh_f(g[1] + x1), fg = sigm(g[2] + x2), og = sigm(g[3] + x3);
  const float c = fg * cp + ig * gg;
  const float h = og * tanh_f(c);
  c_out[(long)b * H + j] = c;
  h_out[(long)b * ldh + j] = h;
  h16_out[(long)b * H + j] = f2bf(h);
  float* a = acts + (long)b * lda + j;
  a[0] = ig; a[H] = gg; a[2 * H] = fg; a[3 * H] = og;
}

// Backward step. Workgroup = 16 batch rows x 16 hidden units, KS waves splitting K = 4H: dh_t = dout_t +
// dg_{t+1} . W as D[batch][unit] = A(dg16 rows) x B(W^T rows), partials summed in LDS, then the cell backward
// of each (batch, unit) pair emits dg_t (fp32 for the weight-gradient GEMM, bf16 as the next step's A
// operand) and dc_{t-1} (in place).
template <int NB, int NU>
__global__ void __launch_bounds__(1024) lstm_bwd_step_kernel(
    const bf16_t* __restrict__ WT16, const bf16_t* __restrict__ dg16_next, const float* __restrict__ dout, long ldd,
    const float* __restrict__ dh_ext, const float* __restrict__ acts, long lda, const float* __restrict__ c_prev,
    const float* __restrict__ c_t, float* __restrict__ dc, float* __restrict__ dg_out, long ldg,
    bf16_t* __restrict__ dg16_out, int B, int H, int KS) {
  __shared__ float red[NU * NB][16][16][17];                 // [unit tile x batch tile][K chunk][batch][unit]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kh = lane >> 4;
  const int j0 = blockIdx.x * 16 * NU, b0 = blockIdx.y * 16 * NB;
  const bool cell = threadIdx.x < 256 * NB * NU;
  const int tile = threadIdx.x >> 8, tb = tile % NB, tu = tile / NB;
  const int m = (threadIdx.x >> 4) & 15, n = threadIdx.x & 15;
  const int b = b0 + tb * 16 + m, j = j0 + tu * 16 + n;
  const bool live = cell && b < B;
  const long bj = (long)(b < B ? b : 0) * H + j;
  float dh = 0.f, ig = 0.f, gg = 0.f, fg = 0.f, og = 0.f, c = 0.f, cp = 0.f, dcn = 0.f;
  if (cell) {                        // cell operands in flight while the GEMM runs
    if (dout != nullptr) dh += dout[(long)(b < B ? b : 0) * ldd + j];
    if (dh_ext != nullptr) dh += dh_ext[bj];
    const float* a = acts + (long)(b < B ? b : 0) * lda + j;
    ig = a[0]; gg = a[H]; fg = a[2 * H]; og = a[3 * H];
    c = c_t[bj];
    cp = c_prev != nullptr ? c_prev[bj] : 0.f;
    dcn = dc[bj];
  }
  v4f acc[NU][NB];
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int t = 0; t < NB; ++t) acc[u][t] = v4f{0.f, 0.f, 0.f, 0.f};
  if (dg16_next != nullptr) {
    const long G = 4L * H;
    const int kl = (int)(G / KS);
    // batch rows past B read row 0: an A row only feeds its own output row, whose thread never stores
    const bf16_t* pv[NB];
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const int ba = b0 + t * 16 + r;
      pv[t] = dg16_next + (long)(ba < B ? ba : 0) * G + (long)wave * kl + kh * 8;
    }
    const bf16_t* pw[NU];
#pragma unroll
    for (int u = 0; u < NU; ++u) pw[u] = WT16 + (long)(j0 + u * 16 + r) * G + (long)wave * kl + kh * 8;
    mfma_tiles<NU, NB, false>(pw, pv, kl, acc);
  }
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int t = 0; t < NB; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) red[u * NB + t][wave][kh * 4 + i][r] = acc[u][t][i];  // D[row = batch][col = unit]
  __syncthreads();
  if (!live) return;
  for (int k = 0; k < KS; ++k) dh += red[tu * NB + tb][k][m][n];
  const float tc = tanh_f(c);
  const float dcv = dh * og * (1.f - tc * tc) + dcn;
  const float di = dcv * gg * ig * (1.f - ig);
  const float dgg = dcv * ig * (1.f - gg * gg);
  const float df = dcv * cp * fg * (1.f - fg);
  const float dog = dh * tc * og * (1.f - og);
  dc[bj] = dcv * fg;                                     // flows into c_{t-1}; same thread reads and writes
  float* g = dg_out + (long)b * ldg + j;
  g[0] = di; g[H] = dgg; g[2 * H] = df; g[3 * H] = dog;
  bf16_t* g16 = dg16_out + (long)b * 4 * H + j;
  g16[0] = f2bf(di); g16[H] = f2bf(dgg); g16[2 * H] = f2bf(df); g16[3 * H] = f2bf(dog);
}

// Batch tiles per workgroup: 2 once the 1-tile grid exceeds one workgroup per CU (a second dispatch round costs a
// whole extra step latency, and the pair shares every weight fragment); BIGDL_LSTM_NB forces 1 or 2.
int lstm_nb(int H, int B, int KS, int per_tile_threads) {
  static const int env = [] { const char* e = getenv("BIGDL_LSTM_NB"); return e ? atoi(e) : 0; }();
  if (KS * per_tile_threads < 512) return 1;     // the cell phase needs 256 threads per batch tile
  if (env == 1 || env == 2) return env;
  return (long)(H / 16) * ((B + 15) / 16) > 256 ? 2 : 1;
}

}  // namespace

int bigdl_lstm_fwd_step(const uint16_t* W16, const uint16_t* h16_prev, const float* xg, long ldx, const float* c_prev,
                        float* c_out, float* h_out, long ldh, uint16_t* h16_out, float* acts, long lda, int B, int H,
                        hipStream_t st) {
  if (H % 32 != 0 || B <= 0) return -1;
  static const bool ws = [] { const char* e = getenv("BIGDL_LSTM_WS"); return e ? atoi(e) != 0 : true; }();
  if (ws) {
    // fragment-shared kernel: K chunks of >= 32 over at most 16 (NB = 1) / 8 (NB = 2) waves, 256 cell threads per tile
    int NB = lstm_nb(H, B, 16, 64);
    int KSw = 0;
    for (int k = NB == 2 ? 8 : 16; k >= 1 && !KSw; --k)
      if (H % (k * 32) == 0) KSw = k;
    if (KSw * 64 < 256 * NB) NB = 1;
    if (KSw * 64 >= 256 * NB) {
      dim3 grid(H / 16, (B + 16 * NB - 1) / (16 * NB));
      if (NB == 2)
        lstm_fwd_step_ws_kernel<2, 8><<<grid, 64 * KSw, 0, st>>>(W16, h16_prev, xg, ldx, c_prev, c_out, h_out, ldh,
                                                                 h16_out, acts, lda, B, H, KSw);
      else
        lstm_fwd_step_ws_kernel<1, 16><<<grid, 64 * KSw, 0, st>>>(W16, h16_prev, xg, ldx, c_prev, c_out, h_out, ldh,
                                                                  h16_out, acts, lda, B, H, KSw);
      HIP_LAUNCH_CHECK();
      return 0;
    }
  }
  const int KS = ksplit(H, 4);
  const int NB = lstm_nb(H, B, KS, 256);
  dim3 grid(H / 16, (B + 16 * NB - 1) / (16 * NB));
  if (NB == 2)
    lstm_fwd_step_kernel<2><<<grid, 256 * KS, 0, st>>>(W16, h16_prev, xg, ldx, c_prev, c_out, h_out, ldh, h16_out,
                                                       acts, lda, B, H, KS);
  else
    lstm_fwd_step_kernel<1><<<grid, 256 * KS, 0, st>>>(W16, h16_prev, xg, ldx, c_prev, c_out, h_out, ldh, h16_out,
                                                       acts, lda, B, H, KS);
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_lstm_bwd_step(const uint16_t* WT16, const uint16_t* dg16_next, const float* dout, long ldd,
                        const float* dh_ext, const float* acts, long lda, const float* c_prev, const float* c_t,
                        float* dc, float* dg_out, long ldg, uint16_t* dg16_out, int B, int H, hipStream_t st) {
  if (H % 32 != 0 || B <= 0) return -1;
  const int KS = ksplit(4 * H, 16) < 4 ? 4 : ksplit(4 * H, 16);     // >= 4 waves so all 256 cell threads exist
  const int NB = lstm_nb(H, B, KS, 64);
  // 32 hidden units per workgroup too once the 2-batch-tile grid still exceeds one workgroup per CU (B = 256, H = 1024:
  // 27.7 -> 19.6 us per step; at 256 workgroups or fewer the halved grid loses, B = 128: 15.4 -> 19.0 us); needs 1024
  // cell threads (KS = 16). BIGDL_LSTM_NU forces 1 or 2.
  static const int nu_env = [] { const char* e = getenv("BIGDL_LSTM_NU"); return e ? atoi(e) : 0; }();
  const bool nu_ok = NB == 2 && KS == 16;
  const int NU = !nu_ok ? 1 : (nu_env == 1 || nu_env == 2) ? nu_env
                                                             : ((long)(H / 16) * ((B + 31) / 32) > 256 ? 2 : 1);
  dim3 grid(H / (16 * NU), (B + 16 * NB - 1) / (16 * NB));
  if (NU == 2)
    lstm_bwd_step_kernel<2, 2><<<grid, 64 * KS, 0, st>>>(WT16, dg16_next, dout, ldd, dh_ext, acts, lda, c_prev, c_t,
                                                         dc, dg_out, ldg, dg16_out, B, H, KS);
  else if (NB == 2)
    lstm_bwd_step_kernel<2, 1><<<grid, 64 * KS, 0, st>>>(WT16, dg16_next, dout, ldd, dh_ext, acts, lda, c_prev, c_t,
                                                         dc, dg_out, ldg, dg16_out, B, H, KS);
  else
    lstm_bwd_step_kernel<1, 1><<<grid, 64 * KS, 0, st>>>(WT16, dg16_next, dout, ldd, dh_ext, acts, lda, c_prev, c_t,
                                                         dc, dg_out, ldg, dg16_out, B, H, KS);
  HIP_LAUNCH_CHECK();
  return 0;
}
