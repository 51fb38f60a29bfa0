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

// acc += sum over K (multiple of 32) of A-row x B-row fragments. K is consumed in groups of 8 k-steps whose 16
// loads are all issued before the group's 8 MFMAs, so a wave pays about one memory round trip per group; the
// step kernels split K over many waves so that each wave has one or two groups (a long per-wave chain of
// L2/MALL round trips was the measured bottleneck, tools/lstm_micro.py).
__device__ __forceinline__ v4f mfma_rows(const bf16_t* __restrict__ pa, const bf16_t* __restrict__ pb, int K, v4f acc) {
  constexpr int CH = 8;
  const int steps = K / 32, full = steps / CH * CH;
  for (int s = 0; s < full; s += CH) {
    v8s a[CH], b[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) { a[i] = ld8(pa + (s + i) * 32); b[i] = ld8(pb + (s + i) * 32); }
#pragma unroll
    for (int i = 0; i < CH; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[i], acc, 0, 0, 0);
  }
  for (int s = full; s < steps; ++s)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ld8(pa + s * 32), ld8(pb + s * 32), acc, 0, 0, 0);
  return acc;
}

// K-split factor: chunks of >= 256 (8 k-steps), at most `cap` waves per output tile.
__host__ __device__ inline int ksplit(int K, int cap) {
  int ks = K / 256;
  if (ks < 1) ks = 1;
  if (ks > cap) ks = cap;
  while (ks > 1 && (K % (ks * 32)) != 0) --ks;
  return ks;
}

// Forward step. Workgroup = 16 hidden units x 16 batch rows, 4*KS waves: wave w owns units j0+4(w&3)..+3 as
// one 16-row MFMA tile (row = unit*4 + gate) over K chunk w>>2; all waves of a chunk share the batch tile's
// h_{t-1} fragments (L1). The 64 gate rows a workgroup reads are the same every step (L2-resident on its
// XCD). Gates are summed over the K chunks in LDS, then the cell update and all its loads / stores run
// coalesced along the hidden dimension (16 consecutive units per batch row).
__global__ void __launch_bounds__(1024) lstm_fwd_step_kernel(
    const bf16_t* __restrict__ W16, const bf16_t* __restrict__ h16_prev, const float* __restrict__ xg, long ldx,
    const float* __restrict__ c_prev, float* __restrict__ c_out, float* __restrict__ h_out, long ldh,
    bf16_t* __restrict__ h16_out, float* __restrict__ acts, long lda, int B, int H, int KS) {
  __shared__ float gl[4][16][16][5];                         // [K chunk][batch][unit][gate] (+1 pad)
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kh = lane >> 4;
  const int mt = wave & 3, kc = wave >> 2;
  const int j0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  const bool cell = threadIdx.x < 256;
  // cell element of threads 0..255: (batch b0 + m, unit j0 + n); operands loaded before the GEMM
  const int m = (threadIdx.x >> 4) & 15, n = threadIdx.x & 15;
  const int b = b0 + m, j = j0 + n;
  const bool live = cell && b < B;
  const int bs = b < B ? b : 0;
  float x0 = 0.f, x1 = 0.f, x2 = 0.f, x3 = 0.f, cp = 0.f;
  if (cell) {
    const float* x = xg + (long)bs * ldx + j;
    x0 = x[0]; x1 = x[H]; x2 = x[2 * H]; x3 = x[3 * H];
    cp = c_prev != nullptr ? c_prev[(long)bs * H + j] : 0.f;
  }
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  if (h16_prev != nullptr) {
    const int kl = H / KS;
    const int grow = (r & 3) * H + j0 + mt * 4 + (r >> 2);          // A row r = unit*4 + gate
    const int bl = b0 + r;
    // batch rows past B read row 0: a batch column only feeds its own output column, never stored
    acc = mfma_rows(W16 + (long)grow * H + kc * kl + kh * 8,
                    h16_prev + (long)(bl < B ? bl : 0) * H + kc * kl + kh * 8, kl, acc);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) gl[kc][r][mt * 4 + kh][i] = acc[i];  // D[row = unit*4+gate][col = batch]
  __syncthreads();
  if (!live) return;
  float g[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float v = 0.f;
    for (int k = 0; k < KS; ++k) v += gl[k][m][n][i];
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
__global__ void __launch_bounds__(1024) lstm_bwd_step_kernel(
    const bf16_t* __restrict__ WT16, const bf16_t* __restrict__ dg16_next, const float* __restrict__ dout, long ldd,
    const float* __restrict__ dh_ext, const float* __restrict__ acts, long lda, const float* __restrict__ c_prev,
    const float* __restrict__ c_t, float* __restrict__ dc, float* __restrict__ dg_out, long ldg,
    bf16_t* __restrict__ dg16_out, int B, int H, int KS) {
  __shared__ float red[16][16][17];                          // [K chunk][batch][unit]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kh = lane >> 4;
  const int j0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  const bool cell = threadIdx.x < 256;
  const int m = (threadIdx.x >> 4) & 15, n = threadIdx.x & 15;
  const int b = b0 + m, j = j0 + n;
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
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  if (dg16_next != nullptr) {
    const int ba = b0 + r;
    const long G = 4L * H;
    const int kl = (int)(G / KS);
    // batch rows past B read row 0: an A row only feeds its own output row, whose thread never stores
    acc = mfma_rows(dg16_next + (long)(ba < B ? ba : 0) * G + (long)wave * kl + kh * 8,
                    WT16 + (long)(j0 + r) * G + (long)wave * kl + kh * 8, kl, acc);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) red[wave][kh * 4 + i][r] = acc[i];      // D[row = batch][col = unit]
  __syncthreads();
  if (!live) return;
  for (int k = 0; k < KS; ++k) dh += red[k][m][n];
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

}  // namespace

int bigdl_lstm_fwd_step(const uint16_t* W16, const uint16_t* h16_prev, const float* xg, long ldx, const float* c_prev,
                        float* c_out, float* h_out, long ldh, uint16_t* h16_out, float* acts, long lda, int B, int H,
                        hipStream_t st) {
  if (H % 32 != 0 || B <= 0) return -1;
  const int KS = ksplit(H, 4);
  dim3 grid(H / 16, (B + 15) / 16);
  lstm_fwd_step_kernel<<<grid, 256 * KS, 0, st>>>(W16, h16_prev, xg, ldx, c_prev, c_out, h_out, ldh, h16_out, acts,
                                                  lda, B, H, KS);
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_lstm_bwd_step(const uint16_t* WT16, const uint16_t* dg16_next, const float* dout, long ldd,
                        const float* dh_ext, const float* acts, long lda, const float* c_prev, const float* c_t,
                        float* dc, float* dg_out, long ldg, uint16_t* dg16_out, int B, int H, hipStream_t st) {
  if (H % 32 != 0 || B <= 0) return -1;
  const int KS = ksplit(4 * H, 16) < 4 ? 4 : ksplit(4 * H, 16);     // >= 4 waves so all 256 cell threads exist
  dim3 grid(H / 16, (B + 15) / 16);
  lstm_bwd_step_kernel<<<grid, 64 * KS, 0, st>>>(WT16, dg16_next, dout, ldd, dh_ext, acts, lda, c_prev, c_t, dc,
                                                 dg_out, ldg, dg16_out, B, H, KS);
  HIP_LAUNCH_CHECK();
  return 0;
}
