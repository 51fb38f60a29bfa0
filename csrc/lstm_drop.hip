// LSTM with dropout (p != 0) on the GPU: the reference's per-gate Dropout + Linear branches (S/nn/LSTM.scala:68-96:
// preTopology = null; four independent Dropout(p) -> Linear(inputSize, hiddenSize) for the input and four
// Dropout(p) -> Linear(hiddenSize, hiddenSize) for the hidden state, joined and summed every step).
//
// Gate g of step t sees x_t * m_x(g, t) and h_{t-1} * m_h(g, t) with independent Bernoulli masks. Nothing here stores a
// mask: every mask bit is a counter-based Philox-4x32-10 draw keyed by (seed, element id), so the backward pass
// regenerates exactly the forward's masks. The host side (nn/recurrent.py, _LSTMDropSeq) composes:
//   * lstm_drop_rep: x -> four masked bf16 copies [4][T*B][Kp] (time-major rows, optional ones column at k = K that
//     carries the folded biases through the GEMM), the operand of ONE batched gate GEMM over the whole sequence;
//     per step the same kernel masks h_{t-1} for the four recurrent GEMMs;
//   * bmm_nt (bmm.hip) for the gate GEMMs, lstm_cell_fwd / bwd (lstm.hip) for the cell;
//   * lstm_drop_rep_bwd: the gradient of the four masked copies summed back through the masks (+ an optional
//     addend, the step's output gradient), written in the input's [B][T][K] order;
//   * lstm_pack_gate_w: gate-blocked bf16 weights [4][H][Kp] (+ the bias column) and their per-gate transposes.
#include "common.h"
#include "kernels.h"

namespace {

struct P4 { unsigned x, y, z, w; };
__device__ __forceinline__ P4 philox4(unsigned long long seed, unsigned long long ctr) {
  unsigned c0 = (unsigned)ctr, c1 = (unsigned)(ctr >> 32), c2 = 0, c3 = 0;
  unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    const unsigned n0 = (unsigned)(p1 >> 32) ^ c1 ^ k0, n2 = (unsigned)(p0 >> 32) ^ c3 ^ k1;
    c1 = (unsigned)p1; c3 = (unsigned)p0; c0 = n0; c2 = n2;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return {c0, c1, c2, c3};
}
__device__ __forceinline__ bool keep_bit(unsigned v, float p) { return (v >> 8) * (1.0f / 16777216.0f) >= p; }

// 4 consecutive mask bits of gate g, row (t, b), columns k .. k + 3 (k % 4 == 0): element id
// ((g * T + t) * B + b) * K + k + off, one Philox draw per 4 elements
__device__ __forceinline__ P4 mask4(unsigned long long seed, long long off, int g, int t, int b, int k, int T, int B,
                                    int K) {
  const unsigned long long e = (unsigned long long)(((long long)(g * T + t) * B + b) * K + k + off);
  return philox4(seed, e >> 2);
}

// y[g][(t * B + b) * Kp + k] = x[b][t][k] * mask * mul (k < K); 1 at k == K when ones; 0 up to Kp
template <typename T_IN>
__global__ __launch_bounds__(256) void drop_rep_kernel(const T_IN* __restrict__ x, long xs_b, long xs_t,
                                                       bf16_t* __restrict__ y, long ys_g, int B, int T, int K, int Kp,
                                                       int ones, float p, float mul, unsigned long long seed,
                                                       long long off) {
  const int kq = Kp >> 2;
  const long total = 4L * T * B * kq;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int q = (int)(i % kq);
    long rest = i / kq;
    const int b = (int)(rest % B);
    rest /= B;
    const int t = (int)(rest % T);
    const int g = (int)(rest / T);
    const int k = 4 * q;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (k < K) {
      const P4 r = mask4(seed, off, g, t, b, k, T, B, K);
      const unsigned rr[4] = {r.x, r.y, r.z, r.w};
      const T_IN* xp = x + b * xs_b + t * xs_t + k;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (k + e < K) {
          float xv;
          if constexpr (sizeof(T_IN) == 4) xv = xp[e];
          else xv = bf2f(xp[e]);
          v[e] = keep_bit(rr[e], p) ? xv * mul : 0.f;
        } else if (ones && k + e == K) {
          v[e] = 1.f;
        }
      }
    } else if (ones && k <= K && K < k + 4) {
      v[K - k] = 1.f;
    }
    bf16_t* yp = y + g * ys_g + ((long)t * B + b) * Kp + k;
    *reinterpret_cast<v2u*>(yp) = v2u{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
  }
}

// dx[b][t][k] = add[b][t][k] + sum_g dy[g][(t * B + b) * ldy + k] * mask * mul
__global__ __launch_bounds__(256) void drop_rep_bwd_kernel(const float* __restrict__ dy, long dys_g, int ldy,
                                                           float* __restrict__ dx, long dxs_b, long dxs_t,
                                                           const float* __restrict__ add, long as_b, long as_t, int B,
                                                           int T, int K, float p, float mul, unsigned long long seed,
                                                           long long off) {
  const int kq = (K + 3) >> 2;
  const long total = (long)T * B * kq;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int q = (int)(i % kq);
    long rest = i / kq;
    const int b = (int)(rest % B);
    const int t = (int)(rest / B);
    const int k = 4 * q;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    if (add != nullptr) {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (k + e < K) s[e] = add[b * as_b + t * as_t + k + e];
    }
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const P4 r = mask4(seed, off, g, t, b, k, T, B, K);
      const unsigned rr[4] = {r.x, r.y, r.z, r.w};
      const float* dp = dy + g * dys_g + ((long)t * B + b) * ldy + k;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (k + e < K && keep_bit(rr[e], p)) s[e] += dp[e] * mul;
    }
    float* o = dx + b * dxs_b + t * dxs_t + k;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (k + e < K) o[e] = s[e];
  }
}

// out[g][h][k] = W[g * H + h][k] (k < Kin), b1 + b2 at k == Kin when bias, 0 up to Kp; outT[g][k][h] = W[g * H + h][k]
__global__ __launch_bounds__(256) void pack_gate_w_kernel(const float* __restrict__ W, const float* __restrict__ b1,
                                                          const float* __restrict__ b2, int H, int Kin, int Kp,
                                                          bf16_t* __restrict__ out, bf16_t* __restrict__ outT) {
  const long n1 = out ? 4L * H * Kp : 0, n2 = outT ? 4L * H * Kin : 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n1 + n2; i += (long)gridDim.x * blockDim.x) {
    if (i < n1) {
      const int k = (int)(i % Kp);
      const long gh = i / Kp;
      float v = 0.f;
      if (k < Kin) v = W[gh * Kin + k];
      else if (k == Kin && (b1 || b2)) v = (b1 ? b1[gh] : 0.f) + (b2 ? b2[gh] : 0.f);
      out[i] = f2bf(v);
    } else {
      const long j = i - n1;
      const int h = (int)(j % H);
      const long gk = j / H;
      const int k = (int)(gk % Kin);
      const int g = (int)(gk / Kin);
      outT[j] = f2bf(W[((long)g * H + h) * Kin + k]);
    }
  }
}

int blocks_for(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 16384 ? 16384 : (b < 1 ? 1 : b));
}

}  // namespace

extern "C" {

int bigdl_lstm_drop_rep(const void* x, int x_bf16, long xs_b, long xs_t, uint16_t* y, long ys_g, int B, int T, int K,
                        int Kp, int ones, float p, float mul, unsigned long long seed, long long off,
                        hipStream_t st) {
  // mask draws are 4-aligned per row: K % 4 == 0 keeps every row on whole draws
  if (K % 4 != 0 || Kp % 4 != 0 || Kp < K + (ones ? 1 : 0) || (off & 3)) return -1;
  const long total = 4L * T * B * (Kp / 4);
  if (x_bf16)
    drop_rep_kernel<bf16_t><<<blocks_for(total), 256, 0, st>>>((const bf16_t*)x, xs_b, xs_t, y, ys_g, B, T, K, Kp,
                                                               ones, p, mul, seed, off);
  else
    drop_rep_kernel<float><<<blocks_for(total), 256, 0, st>>>((const float*)x, xs_b, xs_t, y, ys_g, B, T, K, Kp, ones,
                                                              p, mul, seed, off);
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_lstm_drop_rep_bwd(const float* dy, long dys_g, int ldy, float* dx, long dxs_b, long dxs_t, const float* add,
                            long as_b, long as_t, int B, int T, int K, float p, float mul, unsigned long long seed,
                            long long off, hipStream_t st) {
  if (K % 4 != 0 || (off & 3)) return -1;
  const long total = (long)T * B * (K / 4);
  drop_rep_bwd_kernel<<<blocks_for(total), 256, 0, st>>>(dy, dys_g, ldy, dx, dxs_b, dxs_t, add, as_b, as_t, B, T, K,
                                                         p, mul, seed, off);
  HIP_LAUNCH_CHECK();
  return 0;
}

void bigdl_lstm_pack_gate_w(const float* W, const float* b1, const float* b2, int H, int Kin, int Kp, uint16_t* out,
                            uint16_t* outT, hipStream_t st) {
  const long n = (out ? 4L * H * Kp : 0) + (outT ? 4L * H * Kin : 0);
  pack_gate_w_kernel<<<blocks_for(n), 256, 0, st>>>(W, b1, b2, H, Kin, Kp, out, outT);
  HIP_LAUNCH_CHECK();
}

}  // extern "C"
