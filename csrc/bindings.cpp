// Torch binding layer for the bigdl_amd HIP kernel library.
//
// Thin by design: Python (bigdl_amd/ops) owns allocation and buffer reuse (so whole training steps can be
// captured into one HIP graph); this file only validates tensors, extracts raw pointers and launches the
// C-ABI kernels of csrc/*.hip on the current HIP stream.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <vector>
#include <algorithm>
#include "kernels.h"

namespace {

using at::Tensor;
using OptT = c10::optional<Tensor>;

hipStream_t stream() { return at::hip::getCurrentHIPStream().stream(); }

void check(const Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}
const uint16_t* cbf(const Tensor& t, const char* n) { check(t, at::kBFloat16, n); return (const uint16_t*)t.data_ptr(); }
uint16_t* mbf(const Tensor& t, const char* n) { check(t, at::kBFloat16, n); return (uint16_t*)t.data_ptr(); }
const float* cf(const Tensor& t, const char* n) { check(t, at::kFloat, n); return (const float*)t.data_ptr(); }
float* mf(const Tensor& t, const char* n) { check(t, at::kFloat, n); return (float*)t.data_ptr(); }
const uint16_t* ocbf(const OptT& t, const char* n) { return (t && t->defined()) ? cbf(*t, n) : nullptr; }
uint16_t* ombf(const OptT& t, const char* n) { return (t && t->defined()) ? mbf(*t, n) : nullptr; }
const float* ocf(const OptT& t, const char* n) { return (t && t->defined()) ? cf(*t, n) : nullptr; }
float* omf(const OptT& t, const char* n) { return (t && t->defined()) ? mf(*t, n) : nullptr; }
// optional [P][C / 8] uint8 ReLU sign mask (bigdl_bn_apply zm)
uint8_t* omzm(const OptT& t, int64_t P, int64_t C, const char* n) {
  if (!(t && t->defined())) return nullptr;
  check(*t, at::kByte, n);
  TORCH_CHECK(t->is_contiguous() && t->numel() == P * (C / 8), n, ": sign mask must be a contiguous [P][C/8] uint8 tensor");
  return (uint8_t*)t->data_ptr();
}

// geo = [Nb, Hs, Ws, Cs, OH, OW, mul_h, mul_w, ldw, Ncol, ldo, OHo, OWo, omul_h, omul_w, ooff_h, ooff_w]
// taps = flat [tap_h0, tap_w0, tap_k0, tap_h1, ...]
// pre: optional [2 Cs] fp32 scale | shift of a training BN + ReLU whose input `src` is (ConvArgs::pre). When no kernel
// applies it on load, the BN output is materialised here (bigdl_bn_apply) and returned so the caller can reuse it (the
// weight gradient reads it); otherwise returns None.
OptT conv_nt(const Tensor& src, const Tensor& wt, const Tensor& out, const OptT& bias, const OptT& stats,
             std::vector<int64_t> geo, std::vector<int64_t> taps, bool relu, const OptT& addend, const OptT& bn_x,
             const OptT& bn_z, const OptT& bn_mean, const OptT& bn_aff, const OptT& bn_red, bool accumulate,
             const OptT& bn_zm, const OptT& addend_zm, const OptT& pre) {
  TORCH_CHECK(geo.size() == 17 || geo.size() == 18, "conv_nt: bad geometry");
  if (stats && stats->defined())
    TORCH_CHECK(stats->numel() >= BIGDL_STAT_SLOTS * 2 * geo[9], "conv_nt: stats must hold STAT_SLOTS x 2Ncol");
  TORCH_CHECK(taps.size() % 3 == 0 && !taps.empty() && taps.size() / 3 <= CONV_MAX_TAPS, "conv_nt: bad taps");
  // the epilogue statistics / BN reductions land through multi-writer float atomics: not in deterministic mode
  // (callers take bn_stats / bn_bwd_reduce there instead)
  TORCH_CHECK(!bigdl_deterministic() || (!(stats && stats->defined()) && !(bn_red && bn_red->defined())),
              "conv_nt: epilogue statistics are not deterministic; use bn_stats in deterministic mode");
  ConvArgs a;
  a.src = cbf(src, "src"); a.wt = cbf(wt, "wt");
  a.out = nullptr; a.out32 = nullptr; a.accum32 = accumulate ? 1 : 0;
  if (out.scalar_type() == at::kFloat) a.out32 = mf(out, "out");   // fp32 GEMM output (weight gradients)
  else a.out = mbf(out, "out");
  a.bias = ocf(bias, "bias"); a.stats = omf(stats, "stats");
  a.addend = ocbf(addend, "addend");
  if (a.addend) TORCH_CHECK(addend->numel() == out.numel(), "conv_nt: addend must match out");
  a.bnx = ocbf(bn_x, "bn_x"); a.bnz = ocbf(bn_z, "bn_z"); a.bnmean = ocf(bn_mean, "bn_mean");
  a.bnaff = ocf(bn_aff, "bn_aff"); a.bnred = omf(bn_red, "bn_red");
  a.addzm = nullptr;
  if (addend_zm && addend_zm->defined()) {
    TORCH_CHECK(a.addend && geo[10] == geo[9] && geo[9] % 8 == 0, "conv_nt: a masked addend needs ldo == Ncol");
    a.addzm = omzm(addend_zm, out.numel() / geo[9], geo[9], "addend_zm");
  }
  a.bnzm = nullptr;
  if (bn_zm && bn_zm->defined()) {
    TORCH_CHECK(geo[10] == geo[9] && geo[9] % 8 == 0, "conv_nt: a sign-mask z needs a dense output (ldo == Ncol)");
    a.bnzm = omzm(bn_zm, out.numel() / geo[9], geo[9], "bn_zm");
  }
  if (a.bnred) {
    TORCH_CHECK(a.bnx && a.bnmean && bn_x->numel() == out.numel(), "conv_nt: bn_x must match out, bn_mean required");
    TORCH_CHECK(!a.bnz || bn_z->numel() == out.numel(), "conv_nt: bn_z must match out");
    TORCH_CHECK(bn_mean->numel() >= geo[9] && (!a.bnaff || bn_aff->numel() >= 2 * geo[9]), "conv_nt: bn vectors");
    TORCH_CHECK(bn_red->numel() >= BIGDL_STAT_SLOTS * 2 * geo[9], "conv_nt: bn_red must hold STAT_SLOTS x 2Ncol");
  }
  a.Nb = geo[0]; a.Hs = geo[1]; a.Ws = geo[2]; a.Cs = geo[3]; a.OH = geo[4]; a.OW = geo[5];
  a.mul_h = geo[6]; a.mul_w = geo[7]; a.ldw = geo[8]; a.Ncol = geo[9]; a.ldo = geo[10];
  a.OHo = geo[11]; a.OWo = geo[12]; a.omul_h = geo[13]; a.omul_w = geo[14]; a.ooff_h = geo[15]; a.ooff_w = geo[16];
  a.pstride = geo.size() == 18 ? (int)geo[17] : 0;
  TORCH_CHECK(a.pstride >= 0 && a.pstride % 8 == 0, "conv_nt: pixel stride must be a multiple of 8");
  a.pre = ocf(pre, "pre");
  if (a.pre)
    TORCH_CHECK(pre->numel() >= 2 * geo[3] && a.pstride == 0 && src.numel() % geo[3] == 0 &&
                    (src.is_contiguous() || src.is_contiguous(at::MemoryFormat::ChannelsLast)),
                "conv_nt: pre must hold 2 x Cs floats for a dense source");
  a.ntaps = (int)(taps.size() / 3);
  a.Kdim = a.ntaps * a.Cs;
  a.M = a.Nb * a.OH * a.OW;
  a.ident_out = (a.OHo == a.OH && a.OWo == a.OW && a.omul_h == 1 && a.omul_w == 1 && a.ooff_h == 0 && a.ooff_w == 0);
  a.relu = relu ? 1 : 0;
  int max_tk = 0;
  for (int t = 0; t < a.ntaps; ++t) {
    a.tap_h[t] = (short)taps[3 * t]; a.tap_w[t] = (short)taps[3 * t + 1]; a.tap_k[t] = (short)taps[3 * t + 2];
    max_tk = std::max(max_tk, (int)a.tap_k[t]);
  }
  if (a.pstride > 0) {   // overlapping windows: every window must end inside its source row
    int max_tw = 0;
    for (int t = 0; t < a.ntaps; ++t) max_tw = std::max(max_tw, (int)a.tap_w[t]);
    TORCH_CHECK(((int64_t)(a.OW - 1) * a.mul_w + max_tw) * a.pstride + a.Cs <= (int64_t)a.Ws * a.pstride,
                "conv_nt: a window crosses its source row");
    TORCH_CHECK(src.numel() >= (int64_t)a.Nb * a.Hs * a.Ws * a.pstride, "conv_nt: src too small");
  } else {
    TORCH_CHECK(src.numel() >= (int64_t)a.Nb * a.Hs * a.Ws * a.Cs, "conv_nt: src too small");
  }
  TORCH_CHECK(wt.numel() >= (int64_t)(a.Ncol - 1) * a.ldw + (int64_t)(max_tk + 1) * a.Cs, "conv_nt: weight too small");
  // `out` may be a channel-slice view of a wider NHWC buffer (concat written in place): bound by its storage
  const int64_t out_avail = (int64_t)(out.storage().nbytes() / out.element_size()) - out.storage_offset();
  TORCH_CHECK(a.ldo >= a.Ncol && out_avail >= ((int64_t)a.Nb * a.OHo * a.OWo - 1) * a.ldo + a.Ncol,
              "conv_nt: out too small");
  if (a.addend) TORCH_CHECK(a.ldo == a.Ncol, "conv_nt: an addend needs a dense output (ldo == Ncol)");
  TORCH_CHECK((a.OH - 1) * a.omul_h + a.ooff_h < a.OHo && (a.OW - 1) * a.omul_w + a.ooff_w < a.OWo,
              "conv_nt: output placement out of range");
  OptT materialised;
  if (a.pre && !bigdl_conv_pre_applies(&a)) {
    Tensor y = at::empty_like(src);
    const int64_t P = src.numel() / a.Cs;
    bigdl_bn_apply(a.src, a.pre, a.pre + a.Cs, nullptr, (uint16_t*)y.data_ptr(), P, a.Cs, 1, stream(), nullptr);
    a.src = (const uint16_t*)y.data_ptr();
    a.pre = nullptr;
    materialised = y;
  }
  a.ws = nullptr;
  Tensor ws;
  const long wsn = bigdl_conv_nt_plan(&a);
  if (wsn > 0) {     // split-K partials in a caching-allocator workspace (graph-capture safe)
    ws = at::empty({wsn}, out.options().dtype(at::kFloat));
    a.ws = ws.data_ptr<float>();
  }
  const int rc = bigdl_conv_nt(&a, stream());
  TORCH_CHECK(rc == 0, "conv_nt: unsupported shape (channels must be a multiple of 8; fp32 output needs Ncol % 8 "
              "== 0 and no fused stats / BN / ReLU / addend)");
  return materialised;
}

// geo = [Nb, Hs, Ws, Cs, OH, OW, R, S, sh, sw, ph, pw, dh, dw, M, Ncol, Kdim, ldy]
// pre: optional [2 Cs] scale | shift of the training BN + ReLU whose input `src` is (WgradArgs::pre): applied on load
// by the halo 3x3 weight gradient, else the BN output is materialised here first (bigdl_bn_apply)
void conv_wgrad(const Tensor& dy, const Tensor& src, const Tensor& dw, const OptT& dbias, std::vector<int64_t> geo,
                const OptT& pre) {
  TORCH_CHECK(geo.size() == 18, "conv_wgrad: bad geometry");
  WgradArgs a;
  a.dy = cbf(dy, "dy"); a.src = cbf(src, "src"); a.dw = mf(dw, "dw"); a.dbias = omf(dbias, "dbias");
  int* f = &a.Nb;
  for (int i = 0; i < 18; ++i) f[i] = (int)geo[i];
  a.m_per_split = 0;
  a.ws = nullptr;
  a.splits = 0;
  a.pre = ocf(pre, "pre");
  Tensor det_ws;
  a.det_ws = nullptr;
  if (bigdl_deterministic() && a.dbias) {
    det_ws = at::empty({(int64_t)BIGDL_DET_SLOTS * a.Ncol}, dw.options().dtype(at::kFloat));
    a.det_ws = det_ws.data_ptr<float>();
  }
  Tensor mat;
  if (a.pre) {
    TORCH_CHECK(pre->numel() >= 2 * a.Cs && src.numel() % a.Cs == 0, "conv_wgrad: pre must hold 2 x Cs floats");
    if (!bigdl_wgrad_pre_applies(&a)) {
      mat = at::empty_like(src);
      bigdl_bn_apply(a.src, a.pre, a.pre + a.Cs, nullptr, (uint16_t*)mat.data_ptr(), src.numel() / a.Cs, a.Cs, 1,
                     stream(), nullptr);
      a.src = (const uint16_t*)mat.data_ptr();
      a.pre = nullptr;
    }
  }
  TORCH_CHECK(dw.numel() >= (int64_t)a.Ncol * a.Kdim, "conv_wgrad: dw too small");
  TORCH_CHECK(a.M == a.Nb * a.OH * a.OW, "conv_wgrad: M mismatch");
  TORCH_CHECK(dy.numel() >= (int64_t)(a.M - 1) * a.ldy + a.Ncol, "conv_wgrad: dy too small");
  TORCH_CHECK(src.numel() >= (int64_t)a.Nb * a.Hs * a.Ws * a.Cs, "conv_wgrad: src too small");
  Tensor ws;
  const long wsn = bigdl_conv_wgrad_plan(&a);
  if (wsn > 0) {     // split-K partials in a caching-allocator workspace (graph-capture safe)
    ws = at::empty({wsn}, dw.options().dtype(at::kFloat));
    a.ws = ws.data_ptr<float>();
  }
  const int rc = bigdl_conv_wgrad(&a, stream());
  TORCH_CHECK(rc == 0, "conv_wgrad: unsupported shape (channels must be a multiple of 8)");
}

// true when conv_wgrad would run the phase-interleaved 256 x 256 kernel on this geometry (callers skip the
// transpose-based NT GEMM route then)
bool conv_wgrad_uses_p8(std::vector<int64_t> geo, bool bias) {
  TORCH_CHECK(geo.size() == 18, "conv_wgrad_uses_p8: bad geometry");
  WgradArgs a{};
  int* f = &a.Nb;
  for (int i = 0; i < 18; ++i) f[i] = (int)geo[i];
  static float dummy;
  a.dbias = bias ? &dummy : nullptr;
  return bigdl_conv_wgrad_uses_p8(&a) != 0;
}

void transpose_krsc(const Tensor& w, const Tensor& wt, int64_t K, int64_t RS, int64_t C) {
  TORCH_CHECK(w.numel() == K * RS * C && wt.numel() == K * RS * C, "transpose_krsc: size mismatch");
  bigdl_transpose_krsc(cbf(w, "w"), mbf(wt, "wt"), (int)K, (int)RS, (int)C, stream());
}

void bn_stats(const Tensor& x, const Tensor& stats, int64_t P, int64_t C) {
  TORCH_CHECK(C % 8 == 0 && x.numel() == P * C, "bn_stats: shape");
  TORCH_CHECK(stats.numel() >= BIGDL_STAT_SLOTS * 2 * C, "bn_stats: stats must hold STAT_SLOTS x 2C");
  bigdl_bn_stats(cbf(x, "x"), mf(stats, "stats"), P, (int)C, stream());
}
void bn_finalize(const Tensor& stats, int64_t nslots, const OptT& gamma, const OptT& beta, const OptT& rmean,
                 const OptT& rvar, const OptT& smean, const OptT& sinv, const Tensor& scale, const Tensor& shift,
                 int64_t P, int64_t C, double eps, double momentum, bool training) {
  TORCH_CHECK(stats.numel() >= nslots * 2 * C, "bn_finalize: stats size");
  bigdl_bn_finalize(cf(stats, "stats"), (int)nslots, ocf(gamma, "gamma"), ocf(beta, "beta"), omf(rmean, "rmean"),
                    omf(rvar, "rvar"), omf(smean, "smean"), omf(sinv, "sinv"), mf(scale, "scale"),
                    mf(shift, "shift"), P, (int)C, (float)eps, (float)momentum, training ? 1 : 0, stream());
}
void bn_slot_reduce(const Tensor& in, int64_t nslots, int64_t C, const Tensor& out) {
  TORCH_CHECK(in.numel() >= nslots * 2 * C && out.numel() >= 2 * C, "bn_slot_reduce: size");
  bigdl_bn_slot_reduce(cf(in, "in"), (int)nslots, (int)C, mf(out, "out"), stream());
}
void bn_apply(const Tensor& x, const Tensor& scale, const Tensor& shift, const OptT& res, const Tensor& y, int64_t P,
              int64_t C, bool relu, const OptT& zm) {
  TORCH_CHECK(C % 8 == 0 && x.numel() == P * C && y.numel() == P * C, "bn_apply: shape");
  bigdl_bn_apply(cbf(x, "x"), cf(scale, "scale"), cf(shift, "shift"), ocbf(res, "res"), mbf(y, "y"), P, (int)C,
                 relu ? 1 : 0, stream(), omzm(zm, P, C, "zm"));
}
void bn_bwd_reduce(const Tensor& dz, const OptT& z, const Tensor& x, const Tensor& mean, const Tensor& red, int64_t P,
                   int64_t C, const OptT& aff, const OptT& zm) {
  TORCH_CHECK(C % 8 == 0 && x.numel() == P * C && dz.numel() == P * C, "bn_bwd_reduce: shape");
  TORCH_CHECK(red.numel() >= BIGDL_STAT_SLOTS * 2 * C, "bn_bwd_reduce: red must hold STAT_SLOTS x 2C");
  if (aff && aff->defined()) TORCH_CHECK(aff->numel() >= 2 * C && aff->is_contiguous(), "bn_bwd_reduce: aff is [2C]");
  bigdl_bn_bwd_reduce(cbf(dz, "dz"), ocbf(z, "z"), cbf(x, "x"), cf(mean, "mean"), mf(red, "red"), P, (int)C,
                      ocf(aff, "aff"), stream(), omzm(zm, P, C, "zm"));
}
void bn_bwd_apply(const Tensor& dz, const OptT& z, const Tensor& x, const Tensor& mean, const Tensor& invstd,
                  const OptT& gamma, const OptT& red, int64_t nslots, const Tensor& coef, const OptT& dx,
                  const OptT& dres, const OptT& dgamma, const OptT& dbeta, int64_t P, int64_t C, const OptT& aff,
                  const OptT& zm, const OptT& x2, const OptT& mean2, const OptT& red2) {
  TORCH_CHECK(coef.numel() >= 3 * C, "bn_bwd_apply: coef size");
  const bool r2 = red2 && red2->defined();
  if (r2) {
    TORCH_CHECK(dres && dres->defined() && x2 && x2->defined() && mean2 && mean2->defined(),
                "bn_bwd_apply: red2 needs dres, x2 and mean2");
    TORCH_CHECK(x2->numel() == x.numel() && x2->strides() == x.strides(), "bn_bwd_apply: x2 must match x's layout");
    TORCH_CHECK(mean2->numel() >= C && red2->numel() >= (int64_t)BIGDL_STAT_SLOTS * 2 * C, "bn_bwd_apply: mean2 / red2 size");
  }
  if (aff && aff->defined()) TORCH_CHECK(aff->numel() >= 2 * C && aff->is_contiguous(), "bn_bwd_apply: aff is [2C]");
  const bool training = red && red->defined();
  bigdl_bn_bwd_apply(cbf(dz, "dz"), ocbf(z, "z"), cbf(x, "x"), cf(mean, "mean"), cf(invstd, "invstd"),
                     ocf(gamma, "gamma"), ocf(red, "red"), (int)nslots, mf(coef, "coef"), ombf(dx, "dx"),
                     ombf(dres, "dres"), omf(dgamma, "dgamma"), omf(dbeta, "dbeta"), P, (int)C, training ? 1 : 0,
                     ocf(aff, "aff"), stream(), omzm(zm, P, C, "zm"), r2 ? cbf(*x2, "x2") : nullptr,
                     r2 ? cf(*mean2, "mean2") : nullptr, r2 ? omf(red2, "red2") : nullptr);
}

void dgrad_fill(const Tensor& out, const OptT& addend, int64_t sh, int64_t sw, int64_t mask) {
  TORCH_CHECK(out.dim() == 4 && out.is_contiguous(at::MemoryFormat::ChannelsLast) && out.size(1) % 8 == 0,
              "dgrad_fill: out must be NHWC bf16 with C % 8 == 0");
  TORCH_CHECK(sh * sw <= 32, "dgrad_fill: at most 32 stride phases");
  if (addend && addend->defined())
    TORCH_CHECK(addend->sizes() == out.sizes() && addend->is_contiguous(at::MemoryFormat::ChannelsLast),
                "dgrad_fill: addend must match out (NHWC)");
  bigdl_dgrad_fill(mbf(out, "out"), ocbf(addend, "addend"), out.size(0) * out.size(2) * out.size(3), out.size(2),
                   out.size(3), out.size(1), (int)sh, (int)sw, (unsigned)mask, stream());
}
void hog_cus(int64_t n, double us, const Tensor& done) {
  TORCH_CHECK(done.is_cuda() && done.scalar_type() == at::kInt && done.numel() >= n, "hog_cus: done must be int32 cuda [n]");
  bigdl_hog_cus((int)n, us, done.data_ptr<int>(), stream());
}
void spin_us(double us, const Tensor& done) {
  TORCH_CHECK(done.is_cuda() && done.scalar_type() == at::kInt && done.numel() >= 1, "spin_us: done must be int32 cuda");
  bigdl_spin_us(us, done.data_ptr<int>(), stream());
}
void relu_fwd(const Tensor& x, const Tensor& y) {
  TORCH_CHECK(x.numel() == y.numel(), "relu: size");
  bigdl_relu_fwd(cbf(x, "x"), mbf(y, "y"), x.numel(), stream());
}
void relu_bwd(const Tensor& dy, const Tensor& y, const Tensor& dx) {
  TORCH_CHECK(dy.numel() == y.numel() && dx.numel() == y.numel(), "relu_bwd: size");
  bigdl_relu_bwd(cbf(dy, "dy"), cbf(y, "y"), mbf(dx, "dx"), y.numel(), stream());
}
void add_bf16(const Tensor& a, const Tensor& b, const Tensor& y) {
  TORCH_CHECK(a.numel() == b.numel() && a.numel() == y.numel(), "add: size");
  bigdl_add_bf16(cbf(a, "a"), cbf(b, "b"), mbf(y, "y"), a.numel(), stream());
}
void nchw_to_nhwc(const Tensor& x, const Tensor& y, int64_t Cp) {
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous(), "nchw_to_nhwc: x must be contiguous NCHW");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(y.numel() == (int64_t)N * H * W * Cp && Cp >= C && Cp % 8 == 0, "nchw_to_nhwc: y size / Cp % 8");
  bigdl_nchw_f32_to_nhwc_bf16(cf(x, "x"), mbf(y, "y"), N, C, H, W, (int)Cp, stream());
}
void nchw_to_pairs(const Tensor& x, const Tensor& y, int64_t ph, int64_t pw) {
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && x.size(1) <= 4, "nchw_to_pairs: x must be contiguous NCHW, C <= 4");
  TORCH_CHECK(y.dim() == 4 && y.is_contiguous() && y.size(3) == 8 && y.size(0) == x.size(0), "nchw_to_pairs: y shape");
  const int Hp = y.size(1), Wp = 2 * y.size(2);
  TORCH_CHECK(Hp >= x.size(2) + ph && Wp >= x.size(3) + pw, "nchw_to_pairs: padded image too small");
  bigdl_nchw_to_pairs(cf(x, "x"), mbf(y, "y"), x.size(0), x.size(1), x.size(2), x.size(3), Hp, Wp, (int)ph, (int)pw,
                      stream());
}
void pair_weight(const Tensor& w, const Tensor& wp) {
  TORCH_CHECK(w.dim() == 4 && w.size(1) <= 4, "pair_weight: w must be (K, C<=4, R, S)");
  const int K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3), S2 = (S + 1) / 2;
  TORCH_CHECK(wp.numel() == (int64_t)K * R * S2 * 8 && wp.is_contiguous(), "pair_weight: wp size");
  const long st[4] = {(long)w.stride(0), (long)w.stride(1), (long)w.stride(2), (long)w.stride(3)};
  bigdl_pair_weight(cbf(w, "w"), mbf(wp, "wp"), K, C, R, S, st, stream());
}
void pair_wgrad_add(const Tensor& dwp, const Tensor& gw, double scale) {
  TORCH_CHECK(gw.dim() == 4 && gw.size(1) <= 4, "pair_wgrad_add: gw must be (K, C<=4, R, S)");
  const int K = gw.size(0), C = gw.size(1), R = gw.size(2), S = gw.size(3), S2 = (S + 1) / 2;
  TORCH_CHECK(dwp.numel() == (int64_t)K * R * S2 * 8 && dwp.is_contiguous(), "pair_wgrad_add: dwp size");
  const long st[4] = {(long)gw.stride(0), (long)gw.stride(1), (long)gw.stride(2), (long)gw.stride(3)};
  bigdl_pair_wgrad_add(cf(dwp, "dwp"), mf(gw, "gw"), K, C, R, S, st, (float)scale, stream());
}
// Strided views are accepted as long as each row is contiguous (stride(2) == 1): batch / row strides are passed
// through (the LSTM dropout path writes gate GEMMs straight into a [T][B][4H] buffer viewed as [4][B][H]).
static void bmm_operand(const Tensor& t, const char* n, at::ScalarType ty) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == ty, "bmm_nt: ", n, " has the wrong dtype / device");
  TORCH_CHECK(t.stride(2) == 1 && t.stride(1) >= t.size(2) && t.stride(0) >= 0, "bmm_nt: ", n, " rows must be dense");
  const int64_t last = (t.size(0) - 1) * t.stride(0) + (t.size(1) - 1) * t.stride(1) + t.size(2);
  TORCH_CHECK((int64_t)(t.storage().nbytes() / t.element_size()) - t.storage_offset() >= last, "bmm_nt: ", n,
              " view exceeds its storage");
}
void bmm_nt(const Tensor& a, const Tensor& b, const Tensor& c, double alpha, bool accum) {
  TORCH_CHECK(a.dim() == 3 && b.dim() == 3 && c.dim() == 3, "bmm_nt: [batch, rows, K] operands, [batch, M, N] out");
  bmm_operand(a, "a", at::kBFloat16); bmm_operand(b, "b", at::kBFloat16); bmm_operand(c, "c", at::kFloat);
  TORCH_CHECK(a.size(0) == b.size(0) && a.size(0) == c.size(0) && a.size(2) == b.size(2) && c.size(1) == a.size(1) &&
              c.size(2) == b.size(1), "bmm_nt: shapes");
  TORCH_CHECK(a.size(2) % 32 == 0, "bmm_nt: K must be padded to a multiple of 32");
  const int rc = bigdl_bmm_nt(reinterpret_cast<const uint16_t*>(a.data_ptr()),
                              reinterpret_cast<const uint16_t*>(b.data_ptr()), c.data_ptr<float>(), a.size(0),
                              a.size(1), b.size(1), a.size(2), a.stride(0), b.stride(0), c.stride(0), a.stride(1),
                              b.stride(1), c.stride(1), (float)alpha, accum ? 1 : 0, stream());
  TORCH_CHECK(rc == 0, "bmm_nt: unsupported shape");
}
// ---- TensorMath backend (tensor_math.hip): operands are fp32 GPU tensors already broadcast to the output's
// sizes; the Python side collapses dimensions and passes per-operand strides (elements)
void tensor_apply(const Tensor& out, const OptT& a, const OptT& b, const OptT& c, std::vector<int64_t> size,
                  std::vector<int64_t> so, std::vector<int64_t> sa, std::vector<int64_t> sb, std::vector<int64_t> sc,
                  int64_t op, double s0, double s1, bool contiguous) {
  const int nd = (int)size.size();
  TORCH_CHECK(nd <= 6 && so.size() == size.size() && (sa.empty() || sa.size() == size.size()) &&
                  (sb.empty() || sb.size() == size.size()) && (sc.empty() || sc.size() == size.size()),
              "tensor_apply: at most 6 collapsed dims, one stride per dim and operand");
  int64_t n = 1;
  for (auto v : size) n *= v;
  TORCH_CHECK(n <= out.numel() || nd == 0, "tensor_apply: sizes exceed the output");
  const int rc = bigdl_tensor_apply(mf(out, "out"), ocf(a, "a"), ocf(b, "b"), ocf(c, "c"), nd, size.data(), so.data(),
                                    sa.empty() ? nullptr : sa.data(), sb.empty() ? nullptr : sb.data(),
                                    sc.empty() ? nullptr : sc.data(), (int)op, (float)s0, (float)s1, contiguous ? 1 : 0,
                                    stream());
  TORCH_CHECK(rc == 0, "tensor_apply failed");
}
void tensor_reduce(const Tensor& x, int64_t outer, int64_t R, int64_t inner, int64_t op, double p, const Tensor& out,
                   const OptT& outi, bool mean, const OptT& ws, int64_t chunks) {
  TORCH_CHECK(x.is_contiguous() && x.numel() == outer * R * inner, "tensor_reduce: contiguous [outer, R, inner] input");
  TORCH_CHECK(out.numel() == outer * inner && out.is_contiguous(), "tensor_reduce: out [outer * inner]");
  if (outi && outi->defined()) TORCH_CHECK(outi->numel() == outer * inner, "tensor_reduce: indices [outer * inner]");
  if (chunks > 1) TORCH_CHECK(ws && ws->defined() && ws->numel() >= chunks * outer * inner * 3 + 1, "tensor_reduce: workspace");
  const int rc = bigdl_tensor_reduce(cf(x, "x"), outer, R, inner, (int)op, (float)p, mf(out, "out"), omf(outi, "outi"),
                                     mean ? 1 : 0, omf(ws, "ws"), chunks, stream());
  TORCH_CHECK(rc == 0, "tensor_reduce: unsupported size");
}
// index ops over [outer, R, inner] (csrc/index_ops.hip): op 0 index_select(b -> out), 1 index_add(b into a),
// 2 gather(b -> out, idx shaped like out), 3 scatter(b into a, idx shaped like b's [outer, n, inner])
void index_op(int64_t op, const OptT& a, const Tensor& idx, const OptT& b, const OptT& out, int64_t outer, int64_t R,
              int64_t n, int64_t inner, int64_t Rsrc, const OptT& err) {
  TORCH_CHECK(idx.is_cuda() && idx.is_contiguous() && (idx.scalar_type() == at::kFloat || idx.scalar_type() == at::kLong),
              "index_op: idx must be a contiguous fp32 or int64 cuda tensor");
  // err: an int32 cuda word, or None = the process's host-mapped index-error word (read back by host_word(1))
  int* ep = reinterpret_cast<int*>(bigdl_host_word_dev(1));
  if (err && err->defined()) {
    TORCH_CHECK(err->scalar_type() == at::kInt && err->is_cuda(), "index_op: err int32");
    ep = err->data_ptr<int>();
  }
  TORCH_CHECK(ep != nullptr, "index_op: no error word");
  for (const OptT* t : {&a, &b, &out})
    if (*t && (*t)->defined()) TORCH_CHECK((*t)->is_contiguous(), "index_op: operands must be contiguous");
  const int rc = bigdl_index_op((int)op, omf(a, "a"), idx.data_ptr(), idx.scalar_type() == at::kLong ? 1 : 0,
                                ocf(b, "b"), omf(out, "out"), outer, R, n, inner, Rsrc, ep, stream());
  TORCH_CHECK(rc == 0, "index_op: unsupported op");
}
void masked_fill(const Tensor& x, const Tensor& mask, double v) {
  TORCH_CHECK(x.is_contiguous() && mask.is_contiguous() && x.numel() == mask.numel(), "masked_fill: contiguous, same size");
  bigdl_masked_fill(mf(x, "x"), cf(mask, "mask"), (float)v, x.numel(), stream());
}
int64_t mask_blocks(int64_t n) { return bigdl_mask_blocks(n); }
void mask_scan(const Tensor& mask, const Tensor& counts) {
  TORCH_CHECK(mask.is_contiguous() && counts.scalar_type() == at::kInt &&
                  counts.numel() >= bigdl_mask_blocks(mask.numel()) + 1, "mask_scan: counts int32[blocks + 1]");
  bigdl_mask_scan(cf(mask, "mask"), mask.numel(), counts.data_ptr<int>(), stream());
}
void mask_write(bool copy, const Tensor& x, const Tensor& mask, const OptT& src, const OptT& out, const Tensor& counts) {
  TORCH_CHECK(x.is_contiguous() && mask.is_contiguous() && x.numel() == mask.numel(), "mask_write: contiguous, same size");
  const long nsrc = (src && src->defined()) ? src->numel() : 0;
  bigdl_mask_write(copy ? 1 : 0, mf(x, "x"), cf(mask, "mask"), ocf(src, "src"), omf(out, "out"), x.numel(),
                   counts.data_ptr<int>(), nsrc, stream());
}
bool topk_f32(const Tensor& x, int64_t outer, int64_t R, int64_t inner, int64_t k, bool largest, const Tensor& vals,
              const Tensor& inds) {
  TORCH_CHECK(x.is_contiguous() && x.numel() == outer * R * inner, "topk: contiguous [outer, R, inner]");
  TORCH_CHECK(vals.numel() == outer * k * inner && inds.numel() == vals.numel(), "topk: outputs [outer, k, inner]");
  return bigdl_topk(cf(x, "x"), outer, R, inner, (int)k, largest ? 1 : 0, mf(vals, "vals"), mf(inds, "inds"),
                    stream()) == 0;
}
// strides s = [sam, sak, sbk, sbn, scm, scn, smm, smn, bsa, bsb, bsc, bsm]
void gemm_f32(const Tensor& A, const Tensor& B, const OptT& Min, const Tensor& C, int64_t batch, int64_t M, int64_t N,
              int64_t K, std::vector<int64_t> s, double alpha, double beta) {
  TORCH_CHECK(s.size() == 12, "gemm_f32: 12 strides");
  TORCH_CHECK(M < (1L << 31) && N < (1L << 31) && K < (1L << 31), "gemm_f32: sizes");
  const int rc = bigdl_gemm_f32(cf(A, "A"), cf(B, "B"), ocf(Min, "M"), mf(C, "C"), (int)batch, (int)M, (int)N, (int)K,
                                s.data(), (float)alpha, (float)beta, stream());
  TORCH_CHECK(rc == 0, "gemm_f32: unsupported shape");
}
void gemv_f32(const Tensor& A, const Tensor& x, const OptT& Min, const Tensor& y, int64_t M, int64_t K,
              std::vector<int64_t> s, double alpha, double beta) {
  TORCH_CHECK(s.size() == 5, "gemv_f32: strides [sam, sak, sx, smin, sy]");
  const int rc = bigdl_gemv_f32(cf(A, "A"), cf(x, "x"), ocf(Min, "M"), mf(y, "y"), (int)M, (int)K, s[0], s[1], s[2],
                                s[3], s[4], (float)alpha, (float)beta, stream());
  TORCH_CHECK(rc == 0, "gemv_f32 failed");
}
// byte fill of a whole GPU tensor (hipMemsetAsync: a runtime fill, no aten kernel) — int8 buffers' padding channels
void fill_bytes(const Tensor& t, int64_t value) {
  TORCH_CHECK(t.is_cuda() && t.is_non_overlapping_and_dense(), "fill_bytes: dense GPU tensor (any memory format)");
  if (t.numel() == 0) return;
  bigdl_fill_bytes(t.data_ptr(), (int)value, (long)(t.numel() * t.element_size()), stream());   // a kernel, not a memset node
}
void copy_rows_i8(const Tensor& src, const Tensor& dst, int64_t rows, int64_t C, int64_t lds, int64_t ldd) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.scalar_type() == at::kChar && dst.scalar_type() == at::kChar,
              "copy_rows_i8: int8 GPU tensors");
  TORCH_CHECK(rows >= 0 && C >= 0 && lds >= C && ldd >= C, "copy_rows_i8: geometry");
  const int64_t span_s = rows ? (rows - 1) * lds + C : 0, span_d = rows ? (rows - 1) * ldd + C : 0;
  TORCH_CHECK(span_s <= (int64_t)src.storage().nbytes() - src.storage_offset() &&
                  span_d <= (int64_t)dst.storage().nbytes() - dst.storage_offset(),
              "copy_rows_i8: rows exceed the tensors' storage");
  bigdl_copy_rows_i8((const int8_t*)src.data_ptr(), (int8_t*)dst.data_ptr(), rows, (int)C, lds, ldd, stream());
}
void cast_f32_bf16(const Tensor& x, const Tensor& y) {
  TORCH_CHECK(x.numel() == y.numel() && x.is_contiguous() && y.is_contiguous(), "cast: size");
  bigdl_cast_f32_bf16(cf(x, "x"), mbf(y, "y"), x.numel(), stream());
}
void cast_bf16_f32(const Tensor& x, const Tensor& y) {
  TORCH_CHECK(x.numel() == y.numel() && x.is_contiguous() && y.is_contiguous(), "cast: size");
  bigdl_cast_bf16_f32(cbf(x, "x"), mf(y, "y"), x.numel(), stream());
}

// pg = [N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw]
// pre: optional [2 C] scale | shift of the training BN + ReLU whose input x is (applied on load by the fixed 3x3/2
// kernel, else materialised first)
void maxpool_fwd(const Tensor& x, const Tensor& y, const Tensor& idx, std::vector<int64_t> g, const OptT& pre) {
  TORCH_CHECK(g.size() == 12 && g[3] % 8 == 0 && g[6] * g[7] <= 256, "maxpool: geometry");
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.numel() == y.numel(), "maxpool: idx");
  const float* pr = ocf(pre, "pre");
  const uint16_t* xs = cbf(x, "x");
  Tensor tmp;
  if (pr) {
    TORCH_CHECK(pre->numel() >= 2 * g[3] && x.numel() == g[0] * g[1] * g[2] * g[3], "maxpool: pre / x");
    if (!bigdl_maxpool_pre_applies(g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9])) {
      tmp = at::empty_like(x);
      bigdl_bn_apply(xs, pr, pr + g[3], nullptr, (uint16_t*)tmp.data_ptr(), x.numel() / g[3], g[3], 1, stream(), nullptr);
      xs = (const uint16_t*)tmp.data_ptr();
      pr = nullptr;
    }
  }
  bigdl_maxpool_fwd(xs, mbf(y, "y"), (uint8_t*)idx.data_ptr(), g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7],
                    g[8], g[9], g[10], g[11], stream(), pr);
}
void maxpool_bwd(const Tensor& dy, const Tensor& idx, const Tensor& dx, std::vector<int64_t> g) {
  TORCH_CHECK(g.size() == 12 && g[3] % 8 == 0, "maxpool_bwd: geometry");
  bigdl_maxpool_bwd(cbf(dy, "dy"), (const uint8_t*)idx.data_ptr(), mbf(dx, "dx"), g[0], g[1], g[2], g[3], g[4], g[5],
                    g[6], g[7], g[8], g[9], g[10], g[11], stream());
}
// maxpool backward that also accumulates the backward reduction of the BN whose output is the pool's input;
// returns false (nothing launched) when the fused kernel does not apply
bool maxpool_bwd_bnred(const Tensor& dy, const Tensor& idx, const Tensor& dx, std::vector<int64_t> g, const Tensor& bx,
                       const Tensor& mean, const c10::optional<Tensor>& aff, const c10::optional<Tensor>& zm,
                       const Tensor& red) {
  TORCH_CHECK(g.size() == 12 && g[3] % 8 == 0, "maxpool_bwd_bnred: geometry");
  if (!bigdl_maxpool_bwd_bnred_applies(g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11]))
    return false;
  TORCH_CHECK(bx.numel() == dx.numel() && bx.scalar_type() == at::kBFloat16 && bx.is_contiguous(at::MemoryFormat::ChannelsLast),
              "maxpool_bwd_bnred: BN input must be bf16 NHWC of the pool input's shape");
  TORCH_CHECK(mean.scalar_type() == at::kFloat && mean.numel() >= g[3], "maxpool_bwd_bnred: mean");
  TORCH_CHECK(red.scalar_type() == at::kFloat && red.numel() >= (int64_t)BIGDL_STAT_SLOTS * 2 * g[3], "maxpool_bwd_bnred: red");
  TORCH_CHECK(aff.has_value() != zm.has_value(), "maxpool_bwd_bnred: exactly one of aff / zm");
  if (aff) TORCH_CHECK(aff->scalar_type() == at::kFloat && aff->numel() >= 2 * g[3], "maxpool_bwd_bnred: aff");
  if (zm) TORCH_CHECK(zm->scalar_type() == at::kByte && zm->numel() * 8 >= dx.numel(), "maxpool_bwd_bnred: zm");
  bigdl_maxpool_bwd_bnred(cbf(dy, "dy"), (const uint8_t*)idx.data_ptr(), mbf(dx, "dx"), g[0], g[3], g[4], g[5],
                          cbf(bx, "bx"), mean.data_ptr<float>(), aff ? aff->data_ptr<float>() : nullptr,
                          zm ? (const uint8_t*)zm->data_ptr() : nullptr, red.data_ptr<float>(), stream());
  return true;
}
void avgpool_fwd(const Tensor& x, const Tensor& y, std::vector<int64_t> g, bool count_pad) {
  TORCH_CHECK(g.size() == 12 && g[3] % 8 == 0, "avgpool: geometry");
  bigdl_avgpool_fwd(cbf(x, "x"), mbf(y, "y"), g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11],
                    count_pad ? 1 : 0, stream());
}
void avgpool_bwd(const Tensor& dy, const Tensor& dx, std::vector<int64_t> g, bool count_pad) {
  TORCH_CHECK(g.size() == 12 && g[3] % 8 == 0, "avgpool_bwd: geometry");
  bigdl_avgpool_bwd(cbf(dy, "dy"), mbf(dx, "dx"), g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10],
                    g[11], count_pad ? 1 : 0, stream());
}

void softmax_xent(const Tensor& logits, const Tensor& labels, const OptT& loss, const OptT& dlogits, double label_base,
                  double grad_scale) {
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "softmax_xent: logits must be contiguous [B, K]");
  const int B = logits.size(0), K = logits.size(1);
  TORCH_CHECK(labels.numel() == B, "softmax_xent: labels");
  const bool bf = logits.scalar_type() == at::kBFloat16;
  const uint16_t* lb = bf ? cbf(logits, "logits") : nullptr;
  const float* lf = bf ? nullptr : cf(logits, "logits");
  uint16_t* db = nullptr; float* df = nullptr;
  if (dlogits && dlogits->defined()) {
    TORCH_CHECK(dlogits->numel() == logits.numel(), "softmax_xent: dlogits");
    if (dlogits->scalar_type() == at::kBFloat16) db = mbf(*dlogits, "dlogits"); else df = mf(*dlogits, "dlogits");
  }
  bigdl_softmax_xent(lb, lf, cf(labels, "labels"), omf(loss, "loss"), db, df, B, K, (float)label_base,
                     (float)grad_scale, stream());
}

void sgd_step(const Tensor& w, const Tensor& g, const OptT& mom, const OptT& w16, double lr, double wd,
              double momentum, double dampening, bool nesterov, bool first, const OptT& lr_dev,
              const OptT& seg_off, const OptT& seg_wd, int64_t base) {
  TORCH_CHECK(w.numel() == g.numel(), "sgd: size");
  TORCH_CHECK(!(mom && mom->defined()) || mom->numel() == w.numel(), "sgd: mom has ", mom ? mom->numel() : 0,
              " elements, w has ", w.numel());
  TORCH_CHECK(!(w16 && w16->defined()) || w16->numel() == w.numel(), "sgd: w16 size");
  const long* so = nullptr;
  int nseg = 0;
  if (seg_off && seg_off->defined()) {
    TORCH_CHECK(seg_off->scalar_type() == at::kLong && seg_off->is_cuda(), "sgd: seg_off must be int64 GPU");
    so = (const long*)seg_off->data_ptr();
    nseg = (int)seg_off->numel();
    TORCH_CHECK(seg_wd && seg_wd->numel() == nseg, "sgd: seg_wd size");
  }
  bigdl_sgd_step(mf(w, "w"), cf(g, "g"), omf(mom, "mom"), ombf(w16, "w16"), w.numel(), ocf(lr_dev, "lr_dev"),
                 (float)lr, (float)wd, (float)momentum, (float)dampening, nesterov ? 1 : 0, first ? 1 : 0, so,
                 ocf(seg_wd, "seg_wd"), nseg, (long)base, stream());
}
void adam_step(const Tensor& w, const Tensor& g, const Tensor& m, const Tensor& v, const OptT& w16, double lr,
               double b1, double b2, double eps, double wd, double bc1, double bc2) {
  TORCH_CHECK(w.numel() == g.numel() && m.numel() == w.numel() && v.numel() == w.numel(), "adam: state size");
  bigdl_adam_step(mf(w, "w"), cf(g, "g"), mf(m, "m"), mf(v, "v"), ombf(w16, "w16"), w.numel(), (float)lr, (float)b1,
                  (float)b2, (float)eps, (float)wd, (float)bc1, (float)bc2, stream());
}
void optim_step(int64_t method, const Tensor& x, const Tensor& g, const Tensor& s1, const OptT& s2, const OptT& w16,
                double a, double b, double c, double d, double e) {
  TORCH_CHECK(g.numel() == x.numel() && s1.numel() == x.numel() && (!s2 || !s2->defined() || s2->numel() == x.numel())
                  && (!w16 || !w16->defined() || w16->numel() >= x.numel()), "optim_step: buffer sizes");
  for (const Tensor* t : {&x, &g, &s1}) TORCH_CHECK(t->is_contiguous(), "optim_step: contiguous buffers");
  const OptimHP hp{(float)a, (float)b, (float)c, (float)d, (float)e};
  TORCH_CHECK(bigdl_optim_step((int)method, &hp, mf(x, "x"), cf(g, "g"), mf(s1, "s1"), omf(s2, "s2"),
                               ombf(w16, "w16"), x.numel(), stream()) == 0, "optim_step: unknown method");
}
void sumsq(const Tensor& x, const Tensor& out) {
  Tensor ws;      // deterministic mode: per-call slot workspace (re-entrant across streams)
  if (bigdl_deterministic()) ws = at::empty({BIGDL_DET_SLOTS}, out.options().dtype(at::kFloat));
  bigdl_sumsq(cf(x, "x"), mf(out, "out"), x.numel(), stream(), ws.defined() ? ws.data_ptr<float>() : nullptr);
}
void scale_f32(const Tensor& x, const OptT& sdev, double s) {
  bigdl_scale_f32(mf(x, "x"), x.numel(), ocf(sdev, "scale"), (float)s, stream());
}
void lstm_cell_fwd(const Tensor& gates, const OptT& c_prev, const Tensor& c, const Tensor& h, const Tensor& act) {
  const int B = gates.size(0), H = gates.size(1) / 4;
  bigdl_lstm_cell_fwd(cf(gates, "gates"), ocf(c_prev, "c_prev"), mf(c, "c"), mf(h, "h"), mf(act, "act"), B, H,
                      stream());
}
void lstm_cell_bwd(const Tensor& act, const OptT& c_prev, const Tensor& c, const OptT& dh, const OptT& dc_next,
                   const Tensor& dgates, const OptT& dc_prev) {
  const int B = act.size(0), H = act.size(1) / 4;
  bigdl_lstm_cell_bwd(cf(act, "act"), ocf(c_prev, "c_prev"), cf(c, "c"), ocf(dh, "dh"), ocf(dc_next, "dc_next"),
                      mf(dgates, "dgates"), omf(dc_prev, "dc_prev"), B, H, stream());
}

// int8 path (csrc/quant.hip)
void quantize_act(const Tensor& x, const Tensor& q, const Tensor& amax, const Tensor& scale, int64_t N, int64_t P,
                  int64_t C, int64_t Cp, bool static_amax) {
  TORCH_CHECK(x.is_cuda() && x.is_contiguous(), "quantize_act: x must be a contiguous device tensor");
  const bool bf = x.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || x.scalar_type() == at::kFloat, "quantize_act: x must be bf16 or fp32");
  TORCH_CHECK(x.numel() == N * P * C, "quantize_act: x size");
  TORCH_CHECK(q.scalar_type() == at::kChar && q.is_contiguous() && q.numel() == N * P * Cp && Cp % 16 == 0 && Cp >= C,
              "quantize_act: q must be int8 [N][P][Cp], Cp % 16 == 0");
  TORCH_CHECK(amax.numel() >= N && scale.numel() >= N && amax.scalar_type() == at::kFloat, "quantize_act: amax/scale");
  bigdl_quantize_act(x.data_ptr(), bf ? 1 : 0, q.data_ptr<int8_t>(), amax.data_ptr<float>(), scale.data_ptr<float>(),
                     (int)N, P, (int)C, (int)Cp, static_amax ? 1 : 0, stream());
}

// xscale: [N] per-sample scales, or None with xs_const (a static per-tensor scale); out bf16 / fp32 / int8 (int8:
// requantized with out_scale). `out` may be a channel slice of a wider NHWC buffer (rows geo[10] = ldo apart).
void conv_i8(const Tensor& src, const Tensor& wt, const Tensor& out, const OptT& bias, const OptT& xscale,
             const Tensor& wscale, std::vector<int64_t> geo, std::vector<int64_t> taps, bool relu, double xs_const,
             double out_scale, const OptT& addend, double add_scale) {
  TORCH_CHECK(geo.size() == 17, "conv_i8: bad geometry");
  TORCH_CHECK(src.scalar_type() == at::kChar && wt.scalar_type() == at::kChar && src.is_cuda() && wt.is_cuda() &&
                  src.is_contiguous() && wt.is_contiguous(), "conv_i8: src/wt must be contiguous int8 device tensors");
  const int mode = out.scalar_type() == at::kFloat ? 1 : out.scalar_type() == at::kChar ? 2 : 0;
  TORCH_CHECK(mode != 0 || out.scalar_type() == at::kBFloat16, "conv_i8: out bf16, fp32 or int8");
  TORCH_CHECK(mode != 2 || out_scale > 0, "conv_i8: int8 output needs out_scale > 0");
  TORCH_CHECK(out.is_cuda(), "conv_i8: out must be a device tensor");
  TORCH_CHECK(taps.size() % 3 == 0 && !taps.empty() && taps.size() / 3 <= CONV_MAX_TAPS, "conv_i8: bad taps");
  ConvArgs a;
  a.src = reinterpret_cast<const uint16_t*>(src.data_ptr<int8_t>());
  a.wt = reinterpret_cast<const uint16_t*>(wt.data_ptr<int8_t>());
  a.out = reinterpret_cast<uint16_t*>(out.data_ptr());
  a.bias = ocf(bias, "bias"); a.stats = nullptr; a.addend = nullptr; a.out32 = nullptr; a.accum32 = 0;
  a.ws = nullptr; a.ksplit = 0; a.pstride = 0; a.pre = nullptr;
  a.bnx = nullptr; a.bnz = nullptr; a.bnzm = nullptr; a.addzm = nullptr; a.bnmean = nullptr; a.bnaff = nullptr;
  a.bnred = nullptr;
  a.Nb = geo[0]; a.Hs = geo[1]; a.Ws = geo[2]; a.Cs = geo[3]; a.OH = geo[4]; a.OW = geo[5];
  a.mul_h = geo[6]; a.mul_w = geo[7]; a.ldw = geo[8]; a.Ncol = geo[9]; a.ldo = geo[10];
  a.OHo = geo[11]; a.OWo = geo[12]; a.omul_h = geo[13]; a.omul_w = geo[14]; a.ooff_h = geo[15]; a.ooff_w = geo[16];
  a.ntaps = (int)(taps.size() / 3);
  a.Kdim = a.ntaps * a.Cs;
  a.M = a.Nb * a.OH * a.OW;
  a.ident_out = 1;
  a.relu = relu ? 1 : 0;
  int max_tk = 0;
  for (int t = 0; t < a.ntaps; ++t) {
    a.tap_h[t] = (short)taps[3 * t]; a.tap_w[t] = (short)taps[3 * t + 1]; a.tap_k[t] = (short)taps[3 * t + 2];
    max_tk = std::max(max_tk, (int)a.tap_k[t]);
  }
  TORCH_CHECK(src.numel() >= (int64_t)a.Nb * a.Hs * a.Ws * a.Cs, "conv_i8: src too small");
  TORCH_CHECK(wt.numel() >= (int64_t)(a.Ncol - 1) * a.ldw + (int64_t)(max_tk + 1) * a.Cs, "conv_i8: weight too small");
  const int64_t out_avail = (int64_t)(out.storage().nbytes() / out.element_size()) - out.storage_offset();
  TORCH_CHECK(a.ldo >= a.Ncol && out_avail >= (int64_t)(a.M - 1) * a.ldo + a.Ncol, "conv_i8: out too small");
  const bool has_xs = xscale && xscale->defined();
  TORCH_CHECK(!has_xs || (xscale->numel() >= a.Nb && xscale->scalar_type() == at::kFloat && xscale->is_cuda()),
              "conv_i8: xscale must hold N fp32 scales");
  TORCH_CHECK(wscale.numel() >= a.Ncol && wscale.scalar_type() == at::kFloat, "conv_i8: wscale");
  const int8_t* add8 = nullptr;
  long add_ld = 0;
  if (addend && addend->defined()) {
    TORCH_CHECK(addend->scalar_type() == at::kChar && addend->is_cuda() && addend->dim() == 4 &&
                    addend->size(0) * addend->size(1) * addend->size(2) == (int64_t)a.M && addend->size(3) >= a.Ncol &&
                    addend->stride(3) == 1 && addend->stride(1) == addend->size(2) * addend->stride(2) &&
                    addend->stride(0) == addend->size(1) * addend->stride(1),
                "conv_i8: addend must be int8 [N][OH][OW][>= Ncol] rows of one stride");
    add8 = addend->data_ptr<int8_t>();
    add_ld = addend->stride(2);
  }
  const int rc = bigdl_conv_i8(&a, has_xs ? xscale->data_ptr<float>() : nullptr, (float)xs_const,
                               wscale.data_ptr<float>(), mode, mode == 2 ? (float)(1.0 / out_scale) : 0.f, add8,
                               (float)add_scale, add_ld, stream());
  TORCH_CHECK(rc == 0, "conv_i8: unsupported shape (channels must be a multiple of 16)");
}

// int8 7x7/2 image stem straight from the fp32 NCHW image (conv_halo.hip stem_i8f_kernel): geo / taps are the width-
// im2col geometry conv_i8 would get for quantize_wim2col_f32's output (Hs = image rows), `scale` the input
// quantization scale (quantize with 1 / scale, dequantize with scale). Returns false when the kernel does not apply
// (the caller then quantizes into the im2col and calls conv_i8).
bool conv_i8_stem_f32(const Tensor& x, const Tensor& wt, const Tensor& out, const OptT& bias, const Tensor& wscale,
                      std::vector<int64_t> geo, std::vector<int64_t> taps, bool relu, double scale, double out_scale) {
  TORCH_CHECK(geo.size() == 17 && taps.size() % 3 == 0 && !taps.empty() && taps.size() / 3 <= CONV_MAX_TAPS,
              "conv_i8_stem_f32: bad geometry");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && x.scalar_type() == at::kFloat && x.is_cuda() && x.size(0) == geo[0] &&
                  x.size(2) == geo[1], "conv_i8_stem_f32: x must be the fp32 NCHW image of the geometry");
  TORCH_CHECK(wt.scalar_type() == at::kChar && wt.is_cuda() && wt.is_contiguous(), "conv_i8_stem_f32: int8 weight");
  const int mode = out.scalar_type() == at::kFloat ? 1 : out.scalar_type() == at::kChar ? 2 : 0;
  TORCH_CHECK(mode != 0 || out.scalar_type() == at::kBFloat16, "conv_i8_stem_f32: out bf16, fp32 or int8");
  TORCH_CHECK(mode != 2 || out_scale > 0, "conv_i8_stem_f32: int8 output needs out_scale > 0");
  TORCH_CHECK(scale > 0 && wscale.numel() >= geo[9] && wscale.scalar_type() == at::kFloat, "conv_i8_stem_f32: scales");
  ConvArgs a{};
  a.src = nullptr;
  a.wt = reinterpret_cast<const uint16_t*>(wt.data_ptr<int8_t>());
  a.out = reinterpret_cast<uint16_t*>(out.data_ptr());
  a.bias = ocf(bias, "bias");
  a.Nb = geo[0]; a.Hs = geo[1]; a.Ws = geo[2]; a.Cs = geo[3]; a.OH = geo[4]; a.OW = geo[5];
  a.mul_h = geo[6]; a.mul_w = geo[7]; a.ldw = geo[8]; a.Ncol = geo[9]; a.ldo = geo[10];
  a.OHo = geo[11]; a.OWo = geo[12]; a.omul_h = geo[13]; a.omul_w = geo[14]; a.ooff_h = geo[15]; a.ooff_w = geo[16];
  a.ntaps = (int)(taps.size() / 3);
  a.Kdim = a.ntaps * a.Cs;
  a.M = a.Nb * a.OH * a.OW;
  a.ident_out = 1;
  a.relu = relu ? 1 : 0;
  for (int t = 0; t < a.ntaps; ++t) {
    a.tap_h[t] = (short)taps[3 * t]; a.tap_w[t] = (short)taps[3 * t + 1]; a.tap_k[t] = (short)taps[3 * t + 2];
  }
  TORCH_CHECK(wt.numel() >= (int64_t)a.Ncol * a.ldw, "conv_i8_stem_f32: weight too small");
  const int64_t out_avail = (int64_t)(out.storage().nbytes() / out.element_size()) - out.storage_offset();
  TORCH_CHECK(a.ldo >= a.Ncol && out_avail >= (int64_t)(a.M - 1) * a.ldo + a.Ncol, "conv_i8_stem_f32: out too small");
  const I8Epi ep{nullptr, (float)scale, wscale.data_ptr<float>(), mode, mode == 2 ? (float)(1.0 / out_scale) : 0.f,
                 nullptr, 0.f, 0};
  return bigdl_stem_i8_f32(&a, &ep, x.data_ptr<float>(), (int)x.size(1), (int)x.size(3), (float)(1.0 / scale),
                           stream()) == 0;
}

void pool_i8(const Tensor& x, const Tensor& y, std::vector<int64_t> g, bool avg, bool count_pad) {
  // g = [N, H, W, Cp, OH, OW, kh, kw, sh, sw, ph, pw, ldo]
  TORCH_CHECK(g.size() == 13 && x.scalar_type() == at::kChar && y.scalar_type() == at::kChar && x.is_cuda() &&
                  y.is_cuda() && x.is_contiguous(), "pool_i8: int8 device tensors, 13 geometry values");
  TORCH_CHECK(g[3] % 16 == 0 && x.numel() >= g[0] * g[1] * g[2] * g[3], "pool_i8: x is [N][H][W][Cp], Cp % 16 == 0");
  const int64_t y_avail = (int64_t)y.storage().nbytes() - y.storage_offset();
  TORCH_CHECK(g[12] >= g[3] && y_avail >= (g[0] * g[4] * g[5] - 1) * g[12] + g[3] && (y.storage_offset() % 16) == 0,
              "pool_i8: y too small or misaligned");
  bigdl_pool_i8(x.data_ptr<int8_t>(), y.data_ptr<int8_t>(), g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9],
                g[10], g[11], avg ? 1 : 0, count_pad ? 1 : 0, g[12], stream());
}

// int8 stem input: fp32 NCHW (C <= 4) -> int8 width im2col [N][H][OW][32] (quant.hip)
void quantize_wim2col_f32(const Tensor& x, const Tensor& y, int64_t OW, int64_t S, int64_t sw, int64_t pw,
                          double scale) {
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && x.scalar_type() == at::kFloat && x.is_cuda() && x.size(1) <= 4,
              "quantize_wim2col_f32: x fp32 contiguous NCHW with <= 4 channels");
  TORCH_CHECK(S >= 1 && S <= 8 && sw >= 1 && OW >= 1, "quantize_wim2col_f32: 1 <= S <= 8 width taps");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(y.scalar_type() == at::kChar && y.is_cuda() && y.is_contiguous() && y.numel() >= N * H * OW * 32,
              "quantize_wim2col_f32: y is int8 [N][H][OW][32]");
  bigdl_quantize_wim2col_f32(x.data_ptr<float>(), y.data_ptr<int8_t>(), (int)N, (int)C, (int)H, (int)W, (int)OW,
                             (int)S, (int)sw, (int)pw, (float)(1.0 / scale), stream());
}

void quantize_nchw_f32(const Tensor& x, const Tensor& q, int64_t Cp, double scale) {
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && x.scalar_type() == at::kFloat && x.is_cuda(),
              "quantize_nchw_f32: x fp32 contiguous NCHW");
  const int64_t N = x.size(0), C = x.size(1), HW = x.size(2) * x.size(3);
  TORCH_CHECK(Cp % 16 == 0 && Cp >= C && q.scalar_type() == at::kChar && q.numel() >= N * HW * Cp && q.is_contiguous(),
              "quantize_nchw_f32: q is int8 [N][H][W][Cp]");
  bigdl_quantize_nchw_f32(x.data_ptr<float>(), q.data_ptr<int8_t>(), N, C, HW, Cp, (float)(1.0 / scale), stream());
}

void quantize_rows_bf16(const Tensor& x, const Tensor& q, int64_t P, int64_t C, int64_t ldq, double scale) {
  TORCH_CHECK(C % 8 == 0 && x.numel() == P * C && x.scalar_type() == at::kBFloat16 && q.scalar_type() == at::kChar,
              "quantize_rows_bf16: x bf16 [P][C], C % 8 == 0");
  const int64_t q_avail = (int64_t)q.storage().nbytes() - q.storage_offset();
  TORCH_CHECK(ldq >= C && q_avail >= (P - 1) * ldq + C && (q.storage_offset() % 8) == 0, "quantize_rows_bf16: q");
  bigdl_quantize_rows_bf16((const uint16_t*)x.data_ptr(), q.data_ptr<int8_t>(), P, C, ldq, (float)(1.0 / scale),
                           stream());
}

void dequantize_rows(const Tensor& q, const Tensor& y, int64_t P, int64_t C, int64_t ld, double scale) {
  TORCH_CHECK(q.scalar_type() == at::kChar && y.scalar_type() == at::kBFloat16 && y.numel() == P * C &&
                  q.numel() >= (P - 1) * ld + C, "dequantize_rows: shapes");
  bigdl_dequantize_rows(q.data_ptr<int8_t>(), (uint16_t*)y.data_ptr(), P, C, ld, (float)scale, stream());
}

// point-wise activations (csrc/activation.hip)
static bool act_dense(const Tensor& t) {
  return t.is_contiguous() || (t.dim() == 4 && t.is_contiguous(at::MemoryFormat::ChannelsLast));
}
void act_fwd(const Tensor& x, const Tensor& y, int64_t kind, double a, double b) {
  const bool bf = x.scalar_type() == at::kBFloat16;
  TORCH_CHECK(x.is_cuda() && (bf || x.scalar_type() == at::kFloat) && y.scalar_type() == x.scalar_type() &&
                  y.numel() == x.numel() && act_dense(x) && x.strides() == y.strides(),
              "act_fwd: x / y dense bf16 or fp32 device tensors of one layout");
  TORCH_CHECK(bigdl_act_fwd(x.data_ptr(), y.data_ptr(), x.numel(), bf ? 1 : 0, (int)kind, (float)a, (float)b,
                            stream()) == 0, "act_fwd: unknown kind");
}
void act_bwd(const Tensor& x, const Tensor& y, const Tensor& dy, const Tensor& dx, int64_t kind, double a, double b) {
  const bool bf = x.scalar_type() == at::kBFloat16;
  TORCH_CHECK(x.is_cuda() && (bf || x.scalar_type() == at::kFloat) && act_dense(x), "act_bwd: x");
  for (const Tensor* t : {&y, &dy, &dx})
    TORCH_CHECK(t->scalar_type() == x.scalar_type() && t->numel() == x.numel() && t->strides() == x.strides(),
                "act_bwd: y / dy / dx must match x (dtype, size, layout)");
  TORCH_CHECK(bigdl_act_bwd(x.data_ptr(), y.data_ptr(), dy.data_ptr(), dx.data_ptr(), x.numel(), bf ? 1 : 0,
                            (int)kind, (float)a, (float)b, stream()) == 0, "act_bwd: unknown kind");
}


// N-d pooling / nearest up-sampling (csrc/pool_nd.hip): dense [B][D][H][W][C] views, geo = the 17 PoolNdGeo ints
static PoolNdGeo nd_geo(const std::vector<int64_t>& v) {
  TORCH_CHECK(v.size() == 17, "pool_nd geo: 17 ints (B D H W C OD OH OW kd kh kw sd sh sw pd ph pw)");
  PoolNdGeo g;
  int* f = &g.B;
  for (int i = 0; i < 17; ++i) {
    TORCH_CHECK(v[i] >= 0 && v[i] < (1ll << 31), "pool_nd geo out of range");
    f[i] = (int)v[i];
  }
  return g;
}
static bool nd_dtype(const Tensor& a, const Tensor& b, const char* what) {
  const bool bf = a.scalar_type() == at::kBFloat16;
  TORCH_CHECK(a.is_cuda() && (bf || a.scalar_type() == at::kFloat) && b.scalar_type() == a.scalar_type() &&
                  a.is_contiguous() && b.is_contiguous(), what, ": contiguous bf16 or fp32 device tensors of one dtype");
  return bf;
}
void poolnd_fwd(const Tensor& x, const Tensor& y, const c10::optional<Tensor>& idx, std::vector<int64_t> geo,
                bool max_mode, bool count_pad) {
  const PoolNdGeo g = nd_geo(geo);
  const bool bf = nd_dtype(x, y, "poolnd_fwd");
  TORCH_CHECK(x.numel() == (int64_t)g.B * g.D * g.H * g.W * g.C && y.numel() == (int64_t)g.B * g.OD * g.OH * g.OW * g.C,
              "poolnd_fwd: sizes do not match the geometry");
  int* ip = nullptr;
  if (idx && idx->defined()) {
    TORCH_CHECK(idx->scalar_type() == at::kInt && idx->is_contiguous() && idx->numel() == y.numel(), "poolnd_fwd: idx");
    ip = idx->data_ptr<int>();
  }
  TORCH_CHECK(bigdl_poolnd_fwd(x.data_ptr(), y.data_ptr(), ip, &g, max_mode, count_pad, bf, stream()) == 0,
              "poolnd_fwd: unsupported geometry");
}
void poolnd_bwd(const Tensor& dy, const c10::optional<Tensor>& idx, const Tensor& dx, std::vector<int64_t> geo,
                bool max_mode, bool count_pad) {
  const PoolNdGeo g = nd_geo(geo);
  const bool bf = nd_dtype(dy, dx, "poolnd_bwd");
  TORCH_CHECK(dx.numel() == (int64_t)g.B * g.D * g.H * g.W * g.C && dy.numel() == (int64_t)g.B * g.OD * g.OH * g.OW * g.C,
              "poolnd_bwd: sizes do not match the geometry");
  const int* ip = nullptr;
  if (max_mode) {
    TORCH_CHECK(idx && idx->defined() && idx->scalar_type() == at::kInt && idx->is_contiguous() &&
                    idx->numel() == dy.numel(), "poolnd_bwd: max pooling needs the int32 index tensor");
    ip = idx->data_ptr<int>();
  }
  TORCH_CHECK(bigdl_poolnd_bwd(dy.data_ptr(), ip, dx.data_ptr(), &g, max_mode, count_pad, bf, stream()) == 0,
              "poolnd_bwd: unsupported geometry");
}
void upsample_nearest(const Tensor& src, const Tensor& dst, std::vector<int64_t> geo, bool backward) {
  const PoolNdGeo g = nd_geo(geo);
  const bool bf = nd_dtype(src, dst, "upsample_nearest");
  const int64_t small = (int64_t)g.B * g.D * g.H * g.W * g.C, big = (int64_t)g.B * g.OD * g.OH * g.OW * g.C;
  TORCH_CHECK(src.numel() == (backward ? big : small) && dst.numel() == (backward ? small : big),
              "upsample_nearest: sizes do not match the geometry");
  TORCH_CHECK(bigdl_upsample_nearest(src.data_ptr(), dst.data_ptr(), &g, backward, bf, stream()) == 0,
              "upsample_nearest: output extent must be input x factor");
}

// batched KRSC -> CRSK weight transposes (one launch for all conv layers): desc built by ops/conv.py
void transpose_krsc_batched(const Tensor& desc, int64_t n, int64_t total_tiles) {
  TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == at::kLong && desc.is_contiguous() && desc.numel() == 6 * n,
              "transpose_krsc_batched: desc must be a device int64 [n, 6] tensor");
  TORCH_CHECK(n >= 0 && n < (1 << 16) && total_tiles >= 0 && total_tiles < (1ll << 31), "transpose_krsc_batched: size");
  bigdl_transpose_krsc_batched(reinterpret_cast<const long*>(desc.data_ptr<int64_t>()), (int)n, (int)total_tiles,
                               stream());
}

// detection (csrc/detection.hip)
static void check_f32(const Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.scalar_type() == at::kFloat, n, ": contiguous fp32 device tensor");
}

int64_t nms(const Tensor& boxes_sorted, double thresh, bool normalized, int64_t max_keep, const Tensor& keep,
            const Tensor& count) {
  check_f32(boxes_sorted, "nms boxes");
  const int64_t n = boxes_sorted.numel() / 4;
  TORCH_CHECK(boxes_sorted.dim() == 2 && boxes_sorted.size(1) == 4, "nms: boxes must be [n, 4]");
  TORCH_CHECK(keep.scalar_type() == at::kInt && keep.numel() >= n && count.scalar_type() == at::kInt &&
                  count.numel() >= 1, "nms: keep / count int32 buffers");
  const int64_t words = (n + 63) / 64;
  TORCH_CHECK(words <= 256, "nms: at most 16384 boxes");
  auto ws = at::empty({std::max<int64_t>(n * words, 1)}, boxes_sorted.options().dtype(at::kLong));
  const int rc = bigdl_nms(boxes_sorted.data_ptr<float>(), (int)n, (float)thresh, normalized ? 1 : 0, (int)max_keep,
                           reinterpret_cast<unsigned long long*>(ws.data_ptr<int64_t>()), keep.data_ptr<int>(),
                           count.data_ptr<int>(), stream());
  TORCH_CHECK(rc == 0, "nms failed");
  return n;
}

void roi_align_fwd(const Tensor& x, const Tensor& rois, const Tensor& out, double scale, int64_t sampling) {
  check_f32(x, "roi_align x"); check_f32(rois, "roi_align rois"); check_f32(out, "roi_align out");
  TORCH_CHECK(x.dim() == 4 && rois.dim() == 2 && (rois.size(1) == 4 || rois.size(1) == 5) && out.dim() == 4 &&
                  out.size(0) == rois.size(0) && out.size(1) == x.size(1), "roi_align: shapes");
  bigdl_roi_align_fwd(x.data_ptr<float>(), rois.data_ptr<float>(), out.data_ptr<float>(), (int)rois.size(0),
                      (int)rois.size(1), (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)out.size(2),
                      (int)out.size(3), (float)scale, (int)sampling, stream());
}

void roi_pool_fwd(const Tensor& x, const Tensor& rois, const Tensor& out, const Tensor& argmax, double scale) {
  check_f32(x, "roi_pool x"); check_f32(rois, "roi_pool rois"); check_f32(out, "roi_pool out");
  TORCH_CHECK(x.dim() == 4 && rois.dim() == 2 && rois.size(1) == 5 && out.dim() == 4 && out.size(0) == rois.size(0) &&
                  out.size(1) == x.size(1) && argmax.scalar_type() == at::kInt && argmax.numel() == out.numel(),
              "roi_pool: shapes");
  bigdl_roi_pool_fwd(x.data_ptr<float>(), rois.data_ptr<float>(), out.data_ptr<float>(), argmax.data_ptr<int>(),
                     (int)rois.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3), (int)out.size(2),
                     (int)out.size(3), (float)scale, stream());
}

void roi_pool_bwd(const Tensor& gy, const Tensor& argmax, const Tensor& rois, const Tensor& gx) {
  check_f32(gy, "roi_pool gy"); check_f32(rois, "roi_pool rois"); check_f32(gx, "roi_pool gx");
  TORCH_CHECK(gy.dim() == 4 && gx.dim() == 4 && argmax.numel() == gy.numel() && rois.size(0) == gy.size(0),
              "roi_pool_bwd: shapes");
  bigdl_roi_pool_bwd(gy.data_ptr<float>(), argmax.data_ptr<int>(), rois.data_ptr<float>(), gx.data_ptr<float>(),
                     (int)gy.size(0), (int)gx.size(1), (int)gx.size(2), (int)gx.size(3), (int)gy.size(2),
                     (int)gy.size(3), stream());
}

// packed variable-size batch (csrc/image.hip image_pipeline_kernel): src uint8 flat, offs int64 [N], prm fp32 [N, 16]
void image_pipeline(const Tensor& src, const Tensor& offs, const Tensor& prm, const Tensor& out, std::vector<double> mean,
                    std::vector<double> std, bool rgb) {
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kByte && src.is_contiguous(), "image_pipeline: src uint8 device");
  TORCH_CHECK(offs.is_cuda() && offs.scalar_type() == at::kLong && offs.is_contiguous() && offs.dim() == 1,
              "image_pipeline: offs int64 [N] device");
  const int N = (int)offs.size(0);
  TORCH_CHECK(prm.is_cuda() && prm.scalar_type() == at::kFloat && prm.is_contiguous() && prm.dim() == 2 &&
                  prm.size(0) == N && prm.size(1) == 16, "image_pipeline: prm fp32 [N, 16] device");
  TORCH_CHECK(mean.size() == 3 && std.size() == 3, "image_pipeline: mean/std need 3 entries");
  const bool bf = out.scalar_type() == at::kBFloat16;
  int OH, OW;
  if (bf) {
    TORCH_CHECK(out.dim() == 4 && out.size(3) == 3 && out.is_contiguous() && out.size(0) == N, "image_pipeline: bf16 out is [N, OH, OW, 3]");
    OH = (int)out.size(1); OW = (int)out.size(2);
  } else {
    TORCH_CHECK(out.scalar_type() == at::kFloat && out.dim() == 4 && out.size(1) == 3 && out.is_contiguous() &&
                    out.size(0) == N, "image_pipeline: fp32 out is [N, 3, OH, OW]");
    OH = (int)out.size(2); OW = (int)out.size(3);
  }
  // bounds are validated on the host copy of the parameters (the kernel trusts them)
  auto pc = prm.cpu(), oc = offs.cpu();
  const float* p = pc.data_ptr<float>();
  const int64_t* o = oc.data_ptr<int64_t>();
  for (int n = 0; n < N; ++n) {
    const float* q = p + 16 * n;
    const int64_t H = (int64_t)q[0], W = (int64_t)q[1], y0 = (int64_t)q[2], x0 = (int64_t)q[3], ch = (int64_t)q[4],
                  cw = (int64_t)q[5];
    TORCH_CHECK(H > 0 && W > 0 && ch > 0 && cw > 0 && y0 >= 0 && x0 >= 0 && y0 + ch <= H && x0 + cw <= W,
                "image_pipeline: crop box out of bounds for image ", n);
    TORCH_CHECK(o[n] >= 0 && o[n] + H * W * 3 <= src.numel(), "image_pipeline: image ", n, " exceeds the buffer");
    TORCH_CHECK(q[7] >= 0 && q[7] <= 4, "image_pipeline: at most 4 colour ops");
  }
  const float m[3] = {(float)mean[0], (float)mean[1], (float)mean[2]};
  const float inv[3] = {(float)(1.0 / std[0]), (float)(1.0 / std[1]), (float)(1.0 / std[2])};
  bigdl_image_pipeline(src.data_ptr<uint8_t>(), reinterpret_cast<const long*>(offs.data_ptr<int64_t>()),
                       prm.data_ptr<float>(), out.data_ptr(), N, OH, OW, m, inv, rgb ? 1 : 0, bf ? 1 : 0, stream());
}
void image_augment(const Tensor& src, const Tensor& params, const Tensor& out, std::vector<double> mean,
                   std::vector<double> std, bool rgb) {
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kByte && src.dim() == 4 && src.size(3) == 3 &&
                  src.is_contiguous(), "image_augment: src must be a contiguous uint8 [N, H, W, 3] device tensor");
  TORCH_CHECK(params.scalar_type() == at::kInt && params.is_contiguous() && params.numel() == 3 * src.size(0),
              "image_augment: params must be int32 [N, 3]");
  TORCH_CHECK(mean.size() == 3 && std.size() == 3, "image_augment: mean/std need 3 entries");
  const int N = src.size(0), H = src.size(1), W = src.size(2);
  const bool bf = out.scalar_type() == at::kBFloat16;
  int OH, OW;
  if (bf) {
    TORCH_CHECK(out.dim() == 4 && out.size(3) == 3 && out.is_contiguous(), "image_augment: bf16 out is [N, OH, OW, 3]");
    OH = out.size(1), OW = out.size(2);
  } else {
    TORCH_CHECK(out.scalar_type() == at::kFloat && out.dim() == 4 && out.size(1) == 3 && out.is_contiguous(),
                "image_augment: fp32 out is [N, 3, OH, OW]");
    OH = out.size(2), OW = out.size(3);
  }
  TORCH_CHECK(out.size(0) == N && OH <= H && OW <= W, "image_augment: crop larger than the image");
  auto pc = params.cpu();
  const int* p = pc.data_ptr<int>();
  for (int n = 0; n < N; ++n)
    TORCH_CHECK(p[3 * n] >= 0 && p[3 * n] + OH <= H && p[3 * n + 1] >= 0 && p[3 * n + 1] + OW <= W,
                "image_augment: crop window out of bounds for sample ", n);
  float m[3], inv[3];
  for (int c = 0; c < 3; ++c) m[c] = (float)mean[c], inv[c] = (float)(1.0 / std[c]);
  auto pd = params.is_cuda() ? params : params.to(src.device());
  bigdl_image_augment(src.data_ptr<uint8_t>(), pd.data_ptr<int>(), out.data_ptr(), N, H, W, OH, OW, m, inv,
                      rgb ? 1 : 0, bf ? 1 : 0, stream());
}

// ------------------------------------------------------------------------------------------ misc NN (nn_misc.hip)
void contig(const Tensor& t, const char* n) { TORCH_CHECK(t.is_contiguous(), n, " must be contiguous"); }

void lrn_fwd(const Tensor& x, const Tensor& y, const Tensor& scale, int64_t size, double alpha, double beta, double k) {
  contig(x, "x");
  TORCH_CHECK(x.dim() == 4 && y.numel() == x.numel() && scale.numel() == x.numel(), "lrn_fwd: bad shapes");
  bigdl_lrn_fwd(cf(x, "x"), mf(y, "y"), mf(scale, "scale"), x.size(0), x.size(1), x.size(2) * x.size(3), size, alpha,
                beta, k, stream());
}
void lrn_bwd(const Tensor& x, const Tensor& y, const Tensor& scale, const Tensor& gy, const Tensor& gx, int64_t size,
             double alpha, double beta) {
  contig(x, "x"); contig(gy, "gy");
  TORCH_CHECK(x.dim() == 4 && gy.numel() == x.numel() && gx.numel() == x.numel(), "lrn_bwd: bad shapes");
  bigdl_lrn_bwd(cf(x, "x"), cf(y, "y"), cf(scale, "scale"), cf(gy, "gy"), mf(gx, "gx"), x.size(0), x.size(1),
                x.size(2) * x.size(3), size, alpha, beta, stream());
}
static int64_t view_room(const Tensor& t) {
  return (int64_t)(t.storage().nbytes() / t.element_size()) - t.storage_offset();
}
// y[g][(t*B + b)*Kp + k] = x[b*xs_b + t*xs_t + k] * mask * mul (+ a ones column at k == K): lstm_drop.hip
void lstm_drop_rep(const Tensor& x, int64_t xs_b, int64_t xs_t, const Tensor& y, int64_t ys_g, int64_t B, int64_t T,
                   int64_t K, int64_t Kp, bool ones, double p, double mul, int64_t seed, int64_t off) {
  TORCH_CHECK(x.is_cuda() && y.is_cuda() && y.scalar_type() == at::kBFloat16, "lstm_drop_rep: bf16 y on the GPU");
  const bool bf = x.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || x.scalar_type() == at::kFloat, "lstm_drop_rep: x fp32 or bf16");
  TORCH_CHECK(view_room(x) >= (B - 1) * xs_b + (T - 1) * xs_t + K, "lstm_drop_rep: x view too small");
  TORCH_CHECK(view_room(y) >= 3 * ys_g + T * B * Kp && ys_g >= T * B * Kp, "lstm_drop_rep: y view too small");
  const int rc = bigdl_lstm_drop_rep(x.data_ptr(), bf ? 1 : 0, xs_b, xs_t, reinterpret_cast<uint16_t*>(y.data_ptr()),
                                     ys_g, (int)B, (int)T, (int)K, (int)Kp, ones ? 1 : 0, (float)p, (float)mul,
                                     (unsigned long long)seed, (long long)off, stream());
  TORCH_CHECK(rc == 0, "lstm_drop_rep: K and Kp must be multiples of 4 (Kp > K with the ones column)");
}
// dx[b*dxs_b + t*dxs_t + k] = add[...] + sum_g dy[g*dys_g + (t*B + b)*ldy + k] * mask * mul
void lstm_drop_rep_bwd(const Tensor& dy, int64_t dys_g, int64_t ldy, const Tensor& dx, int64_t dxs_b, int64_t dxs_t,
                       const OptT& add, int64_t as_b, int64_t as_t, int64_t B, int64_t T, int64_t K, double p,
                       double mul, int64_t seed, int64_t off) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kFloat && dx.scalar_type() == at::kFloat, "lstm_drop_rep_bwd: fp32");
  TORCH_CHECK(view_room(dy) >= 3 * dys_g + (T * B - 1) * ldy + K, "lstm_drop_rep_bwd: dy view too small");
  TORCH_CHECK(view_room(dx) >= (B - 1) * dxs_b + (T - 1) * dxs_t + K, "lstm_drop_rep_bwd: dx view too small");
  const float* ap = nullptr;
  if (add && add->defined()) {
    TORCH_CHECK(add->scalar_type() == at::kFloat && view_room(*add) >= (B - 1) * as_b + (T - 1) * as_t + K,
                "lstm_drop_rep_bwd: addend");
    ap = add->data_ptr<float>();
  }
  const int rc = bigdl_lstm_drop_rep_bwd(dy.data_ptr<float>(), dys_g, (int)ldy, dx.data_ptr<float>(), dxs_b, dxs_t,
                                         ap, as_b, as_t, (int)B, (int)T, (int)K, (float)p, (float)mul,
                                         (unsigned long long)seed, (long long)off, stream());
  TORCH_CHECK(rc == 0, "lstm_drop_rep_bwd: K must be a multiple of 4");
}
// gate-blocked bf16 weights: out [4][H][Kp] (bias column b1 + b2 at k == Kin), outT [4][Kin][H]
void lstm_pack_gate_w(const Tensor& W, const OptT& b1, const OptT& b2, int64_t H, int64_t Kin, int64_t Kp,
                      const OptT& out, const OptT& outT) {
  contig(W, "W");
  TORCH_CHECK(W.scalar_type() == at::kFloat && W.numel() == 4 * H * Kin, "lstm_pack_gate_w: W [4H, Kin] fp32");
  if (b1 && b1->defined()) TORCH_CHECK(b1->numel() == 4 * H && b1->is_contiguous(), "lstm_pack_gate_w: b1");
  if (b2 && b2->defined()) TORCH_CHECK(b2->numel() == 4 * H && b2->is_contiguous(), "lstm_pack_gate_w: b2");
  if (out && out->defined()) TORCH_CHECK(out->numel() == 4 * H * Kp && out->is_contiguous(), "lstm_pack_gate_w: out");
  if (outT && outT->defined())
    TORCH_CHECK(outT->numel() == 4 * H * Kin && outT->is_contiguous(), "lstm_pack_gate_w: outT");
  bigdl_lstm_pack_gate_w(cf(W, "W"), ocf(b1, "b1"), ocf(b2, "b2"), (int)H, (int)Kin, (int)Kp,
                         (out && out->defined()) ? reinterpret_cast<uint16_t*>(out->data_ptr()) : nullptr,
                         (outT && outT->defined()) ? reinterpret_cast<uint16_t*>(outT->data_ptr()) : nullptr,
                         stream());
}
void dropout(const Tensor& x, const Tensor& y, double p, double mul, int64_t seed) {
  contig(x, "x"); contig(y, "y");
  TORCH_CHECK(x.numel() == y.numel() && x.scalar_type() == y.scalar_type(), "dropout: x/y mismatch");
  const bool bf = x.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bf || x.scalar_type() == at::kFloat, "dropout: fp32 or bf16 only");
  TORCH_CHECK(x.is_cuda() && y.is_cuda(), "dropout: GPU tensors");
  bigdl_dropout(x.data_ptr(), y.data_ptr(), bf ? 1 : 0, x.numel(), p, mul, (unsigned long long)seed, stream());
}
void embedding_fwd(const Tensor& W, const Tensor& idx, const Tensor& out) {
  contig(W, "W"); contig(idx, "idx"); contig(out, "out");
  TORCH_CHECK(W.dim() == 2 && idx.scalar_type() == at::kLong && idx.is_cuda(), "embedding_fwd: W 2-D, idx int64");
  TORCH_CHECK(out.numel() == idx.numel() * W.size(1), "embedding_fwd: out size");
  bigdl_embedding_fwd(cf(W, "W"), (const long*)idx.data_ptr(), mf(out, "out"), idx.numel(), W.size(1), W.size(0),
                      stream());
}
void embedding_bwd(const Tensor& gout, const Tensor& idx, const Tensor& gW, double scale) {
  contig(gout, "gout"); contig(idx, "idx"); contig(gW, "gW");
  TORCH_CHECK(gW.dim() == 2 && idx.scalar_type() == at::kLong && idx.is_cuda(), "embedding_bwd: gW 2-D, idx int64");
  TORCH_CHECK(gout.numel() == idx.numel() * gW.size(1), "embedding_bwd: gout size");
  bigdl_embedding_bwd(cf(gout, "gout"), (const long*)idx.data_ptr(), mf(gW, "gW"), idx.numel(), gW.size(1), gW.size(0),
                      scale, stream());
}
// LookupTable on its raw 1-based ids (float32 or int64 input tensor): no index tensor, bf16 or f32 output gradient
void embedding_fwd_ids(const Tensor& W, const Tensor& ids, const Tensor& out, bool mask_zero) {
  contig(W, "W"); contig(ids, "ids"); contig(out, "out");
  const bool il = ids.scalar_type() == at::kLong;
  TORCH_CHECK(W.dim() == 2 && ids.is_cuda() && (il || ids.scalar_type() == at::kFloat), "embedding_fwd_ids: ids f32/i64");
  TORCH_CHECK(out.numel() == ids.numel() * W.size(1), "embedding_fwd_ids: out size");
  bigdl_embedding_fwd_ids(cf(W, "W"), ids.data_ptr(), il ? 1 : 0, mf(out, "out"), ids.numel(), W.size(1), W.size(0),
                          mask_zero ? 1 : 0, stream());
}
void embedding_bwd_ids(const Tensor& gout, const Tensor& ids, const Tensor& gW, int64_t pad, double scale) {
  contig(gout, "gout"); contig(ids, "ids"); contig(gW, "gW");
  const bool il = ids.scalar_type() == at::kLong, gb = gout.scalar_type() == at::kBFloat16;
  TORCH_CHECK(gW.dim() == 2 && ids.is_cuda() && (il || ids.scalar_type() == at::kFloat), "embedding_bwd_ids: ids f32/i64");
  TORCH_CHECK(gb || gout.scalar_type() == at::kFloat, "embedding_bwd_ids: gout f32 or bf16");
  TORCH_CHECK(gout.numel() == ids.numel() * gW.size(1), "embedding_bwd_ids: gout size");
  bigdl_embedding_bwd_ids(gout.data_ptr(), gb ? 1 : 0, ids.data_ptr(), il ? 1 : 0, mf(gW, "gW"), ids.numel(), gW.size(1),
                          gW.size(0), pad, (float)scale, stream());
}
void resize_bilinear_fwd(const Tensor& x, const Tensor& y, double sh, double sw) {
  contig(x, "x"); contig(y, "y");
  TORCH_CHECK(x.dim() == 4 && y.dim() == 4 && x.size(0) * x.size(1) == y.size(0) * y.size(1), "resize: shapes");
  bigdl_resize_bilinear_fwd(cf(x, "x"), mf(y, "y"), x.size(0) * x.size(1), x.size(2), x.size(3), y.size(2), y.size(3),
                            sh, sw, stream());
}
void resize_bilinear_bwd(const Tensor& gy, const Tensor& gx, double sh, double sw) {
  contig(gy, "gy"); contig(gx, "gx");
  TORCH_CHECK(gy.dim() == 4 && gx.dim() == 4 && gx.size(0) * gx.size(1) == gy.size(0) * gy.size(1), "resize: shapes");
  bigdl_resize_bilinear_bwd(cf(gy, "gy"), mf(gx, "gx"), gy.size(0) * gy.size(1), gx.size(2), gx.size(3), gy.size(2),
                            gy.size(3), sh, sw, stream());
}
void log_softmax_fwd(const Tensor& x, const Tensor& y) {
  contig(x, "x"); contig(y, "y");
  TORCH_CHECK(x.numel() == y.numel() && x.dim() >= 1, "log_softmax_fwd: shapes");
  const int64_t cols = x.size(-1);
  bigdl_log_softmax_fwd(cf(x, "x"), mf(y, "y"), x.numel() / cols, cols, stream());
}
void log_softmax_bwd(const Tensor& y, const Tensor& gy, const Tensor& gx) {
  contig(y, "y"); contig(gy, "gy"); contig(gx, "gx");
  TORCH_CHECK(y.numel() == gy.numel() && gx.numel() == y.numel(), "log_softmax_bwd: shapes");
  const int64_t cols = y.size(-1);
  bigdl_log_softmax_bwd(cf(y, "y"), cf(gy, "gy"), mf(gx, "gx"), y.numel() / cols, cols, stream());
}
void f32_to_bf16_rtz(const Tensor& x, const Tensor& y) {
  contig(x, "x"); contig(y, "y");
  TORCH_CHECK(x.numel() == y.numel(), "f32_to_bf16_rtz: sizes");
  bigdl_f32_to_bf16_rtz(cf(x, "x"), mbf(y, "y"), x.numel(), stream());
}

// ------------------------------------------------------------------------------------------ fused LSTM steps
// Row-strided views (e.g. xg[:, t] of a [B, T, 4H] tensor) are passed with their batch-row stride.
int64_t rowstride(const Tensor& t, int64_t inner, const char* n) {
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1 && t.size(1) == inner, n, ": expected [B, ", inner, "] with unit inner stride");
  return t.stride(0);
}
void lstm_fwd_step(const Tensor& W16, const OptT& h16_prev, const Tensor& xg, const OptT& c_prev, const Tensor& c_out,
                   const Tensor& h_out, const Tensor& h16_out, const Tensor& acts) {
  const int64_t B = xg.size(0), H = W16.size(1);
  TORCH_CHECK(W16.size(0) == 4 * H && W16.is_contiguous(), "lstm_fwd_step: W16 must be [4H, H] contiguous");
  TORCH_CHECK(H % 32 == 0, "lstm_fwd_step: H must be a multiple of 32");
  const int64_t ldx = rowstride(xg, 4 * H, "xg"), ldh = rowstride(h_out, H, "h_out"), lda = rowstride(acts, 4 * H, "acts");
  TORCH_CHECK(h_out.size(0) == B && acts.size(0) == B && c_out.numel() == B * H && h16_out.numel() == B * H,
              "lstm_fwd_step: batch mismatch");
  TORCH_CHECK(c_out.is_contiguous() && h16_out.is_contiguous(), "lstm_fwd_step: c_out/h16_out contiguous");
  if (h16_prev && h16_prev->defined()) TORCH_CHECK(h16_prev->numel() == B * H && h16_prev->is_contiguous(), "h16_prev");
  if (c_prev && c_prev->defined()) TORCH_CHECK(c_prev->numel() == B * H && c_prev->is_contiguous(), "c_prev");
  bigdl_lstm_fwd_step(cbf(W16, "W16"), ocbf(h16_prev, "h16_prev"), cf(xg, "xg"), ldx, ocf(c_prev, "c_prev"),
                      mf(c_out, "c_out"), mf(h_out, "h_out"), ldh, mbf(h16_out, "h16_out"), mf(acts, "acts"), lda, B, H,
                      stream());
}
void lstm_bwd_step(const Tensor& WT16, const OptT& dg16_next, const OptT& dout, const OptT& dh_ext, const Tensor& acts,
                   const OptT& c_prev, const Tensor& c_t, const Tensor& dc, const Tensor& dg_out, const Tensor& dg16_out) {
  const int64_t H = WT16.size(0), B = acts.size(0);
  TORCH_CHECK(WT16.size(1) == 4 * H && WT16.is_contiguous(), "lstm_bwd_step: WT16 must be [H, 4H] contiguous");
  TORCH_CHECK(H % 32 == 0, "lstm_bwd_step: H must be a multiple of 32");
  const int64_t lda = rowstride(acts, 4 * H, "acts"), ldg = rowstride(dg_out, 4 * H, "dg_out");
  int64_t ldd = 0;
  if (dout && dout->defined()) { ldd = rowstride(*dout, H, "dout"); TORCH_CHECK(dout->size(0) == B, "dout batch"); }
  TORCH_CHECK(dg_out.size(0) == B && c_t.numel() == B * H && dc.numel() == B * H && dg16_out.numel() == B * 4 * H,
              "lstm_bwd_step: batch mismatch");
  TORCH_CHECK(c_t.is_contiguous() && dc.is_contiguous() && dg16_out.is_contiguous(), "lstm_bwd_step: contiguity");
  if (dg16_next && dg16_next->defined()) TORCH_CHECK(dg16_next->numel() == B * 4 * H && dg16_next->is_contiguous(), "dg16_next");
  if (dh_ext && dh_ext->defined()) TORCH_CHECK(dh_ext->numel() == B * H && dh_ext->is_contiguous(), "dh_ext");
  if (c_prev && c_prev->defined()) TORCH_CHECK(c_prev->numel() == B * H && c_prev->is_contiguous(), "c_prev");
  bigdl_lstm_bwd_step(cbf(WT16, "WT16"), ocbf(dg16_next, "dg16_next"), ocf(dout, "dout"), ldd, ocf(dh_ext, "dh_ext"),
                      cf(acts, "acts"), lda, ocf(c_prev, "c_prev"), cf(c_t, "c_t"), mf(dc, "dc"), mf(dg_out, "dg_out"),
                      ldg, mbf(dg16_out, "dg16_out"), B, H, stream());
}

// Whole-sequence persistent GRU (csrc/lstm_seq.hip): Wrz16 [2H, H], Wn16 [H, H] bf16; xg [B, T, 3H] f32 (r|z|n),
// h16 [T + 1, B, H] bf16 (h16[0] = h0), rh16 [T, B, H] bf16, gates [3, T, B, H] f32, out [B, T, H] f32.
bool gru_seq_supported(int64_t B, int64_t H) { return bigdl_gru_seq_supported((int)B, (int)H) != 0; }
void gru_seq_fwd(const Tensor& Wrz16, const Tensor& Wn16, const Tensor& xg, const OptT& h0, const Tensor& h16,
                 const Tensor& rh16, const Tensor& gates, const Tensor& out, const Tensor& sync) {
  TORCH_CHECK(xg.dim() == 3 && xg.is_contiguous() && xg.scalar_type() == at::kFloat, "gru_seq_fwd: xg [B, T, 3H] f32");
  const int64_t B = xg.size(0), T = xg.size(1), H = Wn16.size(0);
  TORCH_CHECK(Wrz16.is_contiguous() && Wrz16.size(0) == 2 * H && Wrz16.size(1) == H && Wn16.is_contiguous() &&
              Wn16.size(1) == H && xg.size(2) == 3 * H, "gru_seq_fwd: weights");
  TORCH_CHECK(h16.is_contiguous() && h16.numel() == (T + 1) * B * H && rh16.is_contiguous() && rh16.numel() == T * B * H &&
              gates.is_contiguous() && gates.numel() == 3 * T * B * H && out.is_contiguous() && out.numel() == B * T * H,
              "gru_seq_fwd: buffers");
  TORCH_CHECK(sync.scalar_type() == at::kInt && sync.numel() >= bigdl_lstm_seq_sync_words(), "gru_seq_fwd: sync");
  if (h0 && h0->defined()) TORCH_CHECK(h0->is_contiguous() && h0->numel() == B * H, "gru_seq_fwd: h0");
  TORCH_CHECK(bigdl_gru_seq(0, cbf(Wrz16, "Wrz16"), cbf(Wn16, "Wn16"), cf(xg, "xg"), ocf(h0, "h0"), mbf(h16, "h16"),
                            mbf(rh16, "rh16"), mf(gates, "gates"), mf(out, "out"), nullptr, nullptr, nullptr, nullptr,
                            nullptr, nullptr, reinterpret_cast<unsigned*>(sync.data_ptr<int>()), (int)B, (int)H, (int)T,
                            stream()) == 0, "gru_seq_fwd: unsupported shape");
}
void gru_seq_bwd(const Tensor& Wrz16, const Tensor& Wn16, const OptT& h0, const Tensor& gates, const Tensor& out,
                 const OptT& dout, const OptT& dhT, const Tensor& dx, const Tensor& dn16, const Tensor& drz16,
                 const Tensor& dh0, const Tensor& sync) {
  TORCH_CHECK(dx.dim() == 3 && dx.is_contiguous() && dx.scalar_type() == at::kFloat, "gru_seq_bwd: dx [B, T, 3H] f32");
  const int64_t B = dx.size(0), T = dx.size(1), H = Wn16.size(0);
  TORCH_CHECK(Wrz16.is_contiguous() && Wrz16.size(0) == 2 * H && Wn16.is_contiguous() && dx.size(2) == 3 * H,
              "gru_seq_bwd: weights");
  TORCH_CHECK(gates.numel() == 3 * T * B * H && out.numel() == B * T * H && dn16.numel() == T * B * H &&
              drz16.numel() == T * B * 2 * H && dh0.numel() == B * H && gates.is_contiguous() && out.is_contiguous() &&
              dn16.is_contiguous() && drz16.is_contiguous() && dh0.is_contiguous(), "gru_seq_bwd: buffers");
  TORCH_CHECK(sync.scalar_type() == at::kInt && sync.numel() >= bigdl_lstm_seq_sync_words(), "gru_seq_bwd: sync");
  if (dout && dout->defined()) TORCH_CHECK(dout->is_contiguous() && dout->numel() == B * T * H, "gru_seq_bwd: dout");
  if (dhT && dhT->defined()) TORCH_CHECK(dhT->is_contiguous() && dhT->numel() == B * H, "gru_seq_bwd: dhT");
  if (h0 && h0->defined()) TORCH_CHECK(h0->is_contiguous() && h0->numel() == B * H, "gru_seq_bwd: h0");
  TORCH_CHECK(bigdl_gru_seq(1, cbf(Wrz16, "Wrz16"), cbf(Wn16, "Wn16"), nullptr, ocf(h0, "h0"), nullptr, nullptr,
                            mf(gates, "gates"), mf(out, "out"), ocf(dout, "dout"), ocf(dhT, "dhT"), mf(dx, "dx"),
                            mbf(dn16, "dn16"), mbf(drz16, "drz16"), mf(dh0, "dh0"),
                            reinterpret_cast<unsigned*>(sync.data_ptr<int>()), (int)B, (int)H, (int)T, stream()) == 0,
              "gru_seq_bwd: unsupported shape");
}

// Whole-sequence persistent LSTM: xg [B, T, 4H] f32, h16 [T + 1, B, H] bf16 (h16[0] = h0), out [B, T, H],
// cs [T, B, H], acts [T, B, 4H]; sync = int32 workspace of lstm_seq_sync_words() words (zeroed by the launch).
bool lstm_seq_supported(int64_t B, int64_t H) { return bigdl_lstm_seq_supported((int)B, (int)H) != 0; }
int64_t lstm_seq_sync_words() { return bigdl_lstm_seq_sync_words(); }

// A HIP stream restricted to the CUs whose bits are set in `mask` (32 CUs per word; hipExtStreamCreateWithCUMask).
// Returned as an integer handle for torch.cuda.ExternalStream; the stream lives for the process.
int64_t cu_masked_stream(int64_t device, std::vector<int64_t> mask) {
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice((int)device);
  std::vector<uint32_t> m(mask.begin(), mask.end());
  hipStream_t st = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&st, (uint32_t)m.size(), m.data());
  (void)hipSetDevice(prev);
  TORCH_CHECK(e == hipSuccess, "hipExtStreamCreateWithCUMask failed: ", hipGetErrorString(e));
  return (int64_t)(uintptr_t)st;
}
void lstm_seq_fwd(const Tensor& W16, const Tensor& xg, const OptT& c0, const Tensor& h16, const Tensor& out,
                  const OptT& hT, const Tensor& cs, const Tensor& acts, const Tensor& sync) {
  TORCH_CHECK(xg.dim() == 3 && xg.is_contiguous(), "lstm_seq_fwd: xg must be [B, T, 4H] contiguous");
  const bool bio = xg.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bio || xg.scalar_type() == at::kFloat, "lstm_seq_fwd: xg must be float32 or bfloat16");
  TORCH_CHECK(out.scalar_type() == xg.scalar_type(), "lstm_seq_fwd: out must have xg's dtype");
  const int64_t B = xg.size(0), T = xg.size(1), H = W16.size(1);
  TORCH_CHECK(W16.size(0) == 4 * H && W16.is_contiguous() && xg.size(2) == 4 * H, "lstm_seq_fwd: W16 [4H, H]");
  TORCH_CHECK(h16.is_contiguous() && h16.numel() == (T + 1) * B * H, "lstm_seq_fwd: h16 [T + 1, B, H]");
  TORCH_CHECK(out.is_contiguous() && out.numel() == B * T * H && cs.is_contiguous() && cs.numel() == T * B * H &&
              acts.is_contiguous() && acts.numel() == T * B * 4 * H, "lstm_seq_fwd: out / cs / acts");
  TORCH_CHECK(sync.scalar_type() == at::kInt && sync.numel() >= bigdl_lstm_seq_sync_words(), "lstm_seq_fwd: sync");
  if (c0 && c0->defined()) TORCH_CHECK(c0->is_contiguous() && c0->numel() == B * H, "lstm_seq_fwd: c0");
  if (hT && hT->defined()) TORCH_CHECK(hT->is_contiguous() && hT->numel() == B * H, "lstm_seq_fwd: hT");
  TORCH_CHECK(bigdl_lstm_seq_fwd(cbf(W16, "W16"), xg.data_ptr(), ocf(c0, "c0"), mbf(h16, "h16"), out.data_ptr(),
                                 (hT && hT->defined()) ? mf(*hT, "hT") : nullptr, mf(cs, "cs"), mf(acts, "acts"),
                                 reinterpret_cast<unsigned*>(sync.data_ptr<int>()), (int)B, (int)H, (int)T, bio ? 1 : 0,
                                 stream()) == 0, "lstm_seq_fwd: unsupported shape");
}
void lstm_seq_bwd(const Tensor& W16, const OptT& dout, const OptT& dhT, const OptT& dcT, const Tensor& acts,
                  const Tensor& cs, const OptT& c0, const Tensor& dg16, const Tensor& dxg, const Tensor& dc0,
                  const Tensor& dh0, const Tensor& sync) {
  TORCH_CHECK(dxg.dim() == 3 && dxg.is_contiguous(), "lstm_seq_bwd: dxg must be [B, T, 4H] contiguous");
  const bool bio = dxg.scalar_type() == at::kBFloat16;
  TORCH_CHECK(bio || dxg.scalar_type() == at::kFloat, "lstm_seq_bwd: dxg must be float32 or bfloat16");
  const int64_t B = dxg.size(0), T = dxg.size(1), H = W16.size(1);
  TORCH_CHECK(W16.size(0) == 4 * H && W16.is_contiguous() && dxg.size(2) == 4 * H, "lstm_seq_bwd: W16 [4H, H]");
  TORCH_CHECK(acts.is_contiguous() && acts.numel() == T * B * 4 * H && cs.is_contiguous() && cs.numel() == T * B * H,
              "lstm_seq_bwd: acts / cs");
  TORCH_CHECK(dg16.is_contiguous() && dg16.numel() == T * B * 4 * H && dc0.is_contiguous() && dc0.numel() == B * H &&
              dh0.is_contiguous() && dh0.numel() == B * H, "lstm_seq_bwd: dg16 / dc0 / dh0");
  TORCH_CHECK(sync.scalar_type() == at::kInt && sync.numel() >= bigdl_lstm_seq_sync_words(), "lstm_seq_bwd: sync");
  const void* dp = nullptr;
  if (dout && dout->defined()) {
    TORCH_CHECK(dout->is_contiguous() && dout->numel() == B * T * H && dout->scalar_type() == dxg.scalar_type(),
                "lstm_seq_bwd: dout must be [B, T, H] contiguous with dxg's dtype");
    dp = dout->data_ptr();
  }
  if (dhT && dhT->defined()) TORCH_CHECK(dhT->is_contiguous() && dhT->numel() == B * H, "lstm_seq_bwd: dhT");
  if (dcT && dcT->defined()) TORCH_CHECK(dcT->is_contiguous() && dcT->numel() == B * H, "lstm_seq_bwd: dcT");
  if (c0 && c0->defined()) TORCH_CHECK(c0->is_contiguous() && c0->numel() == B * H, "lstm_seq_bwd: c0");
  TORCH_CHECK(bigdl_lstm_seq_bwd(cbf(W16, "W16"), dp, ocf(dhT, "dhT"), ocf(dcT, "dcT"), cf(acts, "acts"), cf(cs, "cs"),
                                 ocf(c0, "c0"), mbf(dg16, "dg16"), dxg.data_ptr(), mf(dc0, "dc0"), mf(dh0, "dh0"),
                                 reinterpret_cast<unsigned*>(sync.data_ptr<int>()), (int)B, (int)H, (int)T, bio ? 1 : 0,
                                 stream()) == 0, "lstm_seq_bwd: unsupported shape");
}

void layernorm_fwd(const Tensor& x, const OptT& g, const OptT& b, const Tensor& y, const Tensor& mean,
                   const Tensor& rstd, double eps) {
  TORCH_CHECK(x.is_contiguous() && y.is_contiguous() && x.numel() == y.numel() && x.dim() >= 1, "layernorm_fwd: x/y");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(mean.numel() == rows && rstd.numel() == rows, "layernorm_fwd: mean/rstd must hold one value per row");
  if (g && g->defined()) TORCH_CHECK(g->numel() == D && g->is_contiguous(), "layernorm_fwd: gamma");
  if (b && b->defined()) TORCH_CHECK(b->numel() == D && b->is_contiguous(), "layernorm_fwd: beta");
  TORCH_CHECK(bigdl_layernorm_fwd(cf(x, "x"), ocf(g, "g"), ocf(b, "b"), mf(y, "y"), mf(mean, "mean"), mf(rstd, "rstd"),
                                  rows, (int)D, (float)eps, stream()) == 0, "layernorm_fwd: hidden size > 4096");
}
void layernorm_bwd(const Tensor& dy, const Tensor& x, const OptT& g, const Tensor& mean, const Tensor& rstd,
                   const OptT& dx, const OptT& dg, const OptT& db) {
  TORCH_CHECK(dy.is_contiguous() && x.is_contiguous() && dy.numel() == x.numel(), "layernorm_bwd: dy/x");
  const int64_t D = x.size(-1), rows = x.numel() / D;
  TORCH_CHECK(mean.numel() == rows && rstd.numel() == rows, "layernorm_bwd: mean/rstd");
  if (dx && dx->defined()) TORCH_CHECK(dx->is_contiguous() && dx->numel() == x.numel(), "layernorm_bwd: dx");
  if (g && g->defined()) TORCH_CHECK(g->numel() == D, "layernorm_bwd: gamma");
  if (dg && dg->defined()) TORCH_CHECK(dg->numel() == D && dg->is_contiguous(), "layernorm_bwd: dgamma");
  if (db && db->defined()) TORCH_CHECK(db->numel() == D && db->is_contiguous(), "layernorm_bwd: dbeta");
  TORCH_CHECK(bigdl_layernorm_bwd(cf(dy, "dy"), cf(x, "x"), ocf(g, "g"), cf(mean, "mean"), cf(rstd, "rstd"),
                                  omf(dx, "dx"), omf(dg, "dg"), omf(db, "db"), rows, (int)D, stream()) == 0,
              "layernorm_bwd: hidden size > 4096");
}
AttnCall attn_call(const Tensor& q, const Tensor& k, const Tensor& v, const OptT& bias, int64_t H, bool causal) {
  TORCH_CHECK(q.dim() == 3 && k.dim() == 3 && v.dim() == 3, "attention: q/k/v must be [B*H, L, D]");
  TORCH_CHECK(q.is_contiguous() && k.is_contiguous() && v.is_contiguous(), "attention: contiguous q/k/v");
  TORCH_CHECK(k.sizes() == v.sizes() && q.size(0) == k.size(0) && q.size(2) == k.size(2), "attention: shapes");
  AttnCall c{};
  c.q = cbf(q, "q"); c.k = cbf(k, "k"); c.v = cbf(v, "v");
  c.BH = (int)q.size(0); c.H = (int)H; c.Lq = (int)q.size(1); c.Lk = (int)k.size(1); c.D = (int)q.size(2);
  TORCH_CHECK(c.D == 32 || c.D == 64 || c.D == 96 || c.D == 128, "attention: head dim must be 32, 64, 96 or 128");
  TORCH_CHECK(H > 0 && c.BH % H == 0, "attention: heads");
  c.causal = causal ? 1 : 0;
  if (bias && bias->defined()) {
    TORCH_CHECK(bias->dim() == 4, "attention: bias must be 4-D (broadcast over batch, head, query, key)");
    const int64_t B = c.BH / H;
    TORCH_CHECK((bias->size(0) == B || bias->size(0) == 1) && (bias->size(1) == H || bias->size(1) == 1) &&
                (bias->size(2) == c.Lq || bias->size(2) == 1) && (bias->size(3) == c.Lk || bias->size(3) == 1),
                "attention: bias not broadcastable to [B, H, Lq, Lk]");
    c.bias = cf(*bias, "bias");
    c.sb = bias->size(0) == 1 ? 0 : bias->stride(0); c.sh = bias->size(1) == 1 ? 0 : bias->stride(1);
    c.sq = bias->size(2) == 1 ? 0 : bias->stride(2); c.sk = bias->size(3) == 1 ? 0 : bias->stride(3);
  }
  return c;
}
void attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, const OptT& bias, int64_t H, bool causal,
              const Tensor& o, const Tensor& lse, double drop_p, int64_t seed) {
  AttnCall c = attn_call(q, k, v, bias, H, causal);
  TORCH_CHECK(drop_p >= 0.0 && drop_p < 1.0, "attention: dropout probability in [0, 1)");
  c.drop_p = (float)drop_p; c.seed = (unsigned long long)seed;
  TORCH_CHECK(o.is_contiguous() && o.numel() == q.numel() && lse.numel() == (int64_t)c.BH * c.Lq, "attn_fwd: o/lse");
  c.o = mf(o, "o"); c.lse = mf(lse, "lse");
  TORCH_CHECK(bigdl_attn_fwd(&c, stream()) == 0, "attn_fwd: unsupported shape");
}
void attn_bwd(const Tensor& q, const Tensor& k, const Tensor& v, const OptT& bias, int64_t H, bool causal,
              const Tensor& o, const Tensor& lse, const Tensor& dout, const Tensor& dq, const Tensor& dk,
              const Tensor& dv, const Tensor& delta_ws, double drop_p, int64_t seed) {
  AttnCall c = attn_call(q, k, v, bias, H, causal);
  TORCH_CHECK(drop_p >= 0.0 && drop_p < 1.0, "attention: dropout probability in [0, 1)");
  c.drop_p = (float)drop_p; c.seed = (unsigned long long)seed;
  TORCH_CHECK(o.is_contiguous() && dout.is_contiguous() && o.numel() == q.numel() && dout.numel() == q.numel(),
              "attn_bwd: o/dout");
  TORCH_CHECK(dq.is_contiguous() && dq.numel() == q.numel() && dk.numel() == k.numel() && dv.numel() == v.numel() &&
              dk.is_contiguous() && dv.is_contiguous(), "attn_bwd: gradient buffers");
  TORCH_CHECK(lse.numel() == (int64_t)c.BH * c.Lq && delta_ws.numel() == (int64_t)c.BH * c.Lq, "attn_bwd: lse/delta");
  c.o = mf(o, "o"); c.lse = mf(lse, "lse"); c.dout = cf(dout, "dout");
  c.dq = mf(dq, "dq"); c.dk = mf(dk, "dk"); c.dv = mf(dv, "dv");
  TORCH_CHECK(bigdl_attn_bwd(&c, mf(delta_ws, "delta"), stream()) == 0, "attn_bwd: unsupported shape");
}
// geo = [stride_h, stride_w, pad_h, pad_w, dil_h, dil_w, groups]
void gconv(int64_t pass, const Tensor& x_or_dx, const Tensor& w_or_dw, const OptT& b_or_db, const Tensor& y_or_dy,
           std::vector<int64_t> geo) {
  TORCH_CHECK(geo.size() == 7, "gconv: geo = [sh, sw, ph, pw, dh, dw, groups]");
  const Tensor& x = x_or_dx;
  const Tensor& w = w_or_dw;
  const Tensor& y = y_or_dy;
  TORCH_CHECK(x.dim() == 4 && w.dim() == 4 && y.dim() == 4 && x.is_contiguous() && w.is_contiguous() &&
              y.is_contiguous(), "gconv: contiguous NCHW x / y and KCRS weight");
  GConvCall c{};
  c.N = (int)x.size(0); c.C = (int)x.size(1); c.H = (int)x.size(2); c.W = (int)x.size(3);
  c.K = (int)y.size(1); c.OH = (int)y.size(2); c.OW = (int)y.size(3); c.R = (int)w.size(2); c.S = (int)w.size(3);
  c.sh = (int)geo[0]; c.sw = (int)geo[1]; c.ph = (int)geo[2]; c.pw = (int)geo[3]; c.dh = (int)geo[4]; c.dw = (int)geo[5];
  c.G = (int)geo[6];
  TORCH_CHECK(y.size(0) == c.N && w.size(0) == c.K && c.G > 0 && c.C % c.G == 0 && c.K % c.G == 0 &&
              w.size(1) == c.C / c.G, "gconv: shapes (weight [K, C/groups, R, S])");
  TORCH_CHECK((c.OH - 1) * c.sh - c.ph + (c.R - 1) * c.dh < c.H + c.ph + c.sh &&
              (c.OW - 1) * c.sw - c.pw + (c.S - 1) * c.dw < c.W + c.pw + c.sw, "gconv: output size inconsistent");
  if (b_or_db && b_or_db->defined()) TORCH_CHECK(b_or_db->numel() == c.K && b_or_db->is_contiguous(), "gconv: bias");
  if (pass == 0) { c.x = cf(x, "x"); c.w = cf(w, "w"); c.b = ocf(b_or_db, "b"); c.y = mf(y, "y"); }
  else if (pass == 1) { c.dx = mf(x, "dx"); c.w = cf(w, "w"); c.dy = cf(y, "dy"); }
  else { c.x = cf(x, "x"); c.dwt = mf(w, "dw"); c.db = omf(b_or_db, "db"); c.dy = cf(y, "dy"); }
  TORCH_CHECK(bigdl_gconv(&c, (int)pass, stream()) == 0, "gconv: bad geometry");
}
void ones_col_pack(const Tensor& x, const Tensor& xe) {
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(1) % 8 == 0, "ones_col_pack: x must be [M, K] contiguous, K % 8 == 0");
  TORCH_CHECK(xe.dim() == 2 && xe.is_contiguous() && xe.size(0) == x.size(0) && xe.size(1) == x.size(1) + 8,
              "ones_col_pack: xe must be [M, K + 8] contiguous");
  bigdl_ones_col_pack(cbf(x, "x"), mbf(xe, "xe"), x.size(0), (int)x.size(1), stream());
}
void ones_col_acc(const Tensor& gw, const Tensor& gW, const OptT& gB, double sW, double sB) {
  TORCH_CHECK(gW.dim() == 2 && gW.is_contiguous() && gW.size(1) % 4 == 0, "ones_col_acc: gW must be [N, K] contiguous");
  TORCH_CHECK(gw.is_contiguous() && gw.dim() == 2 && gw.size(0) == gW.size(0) && gw.size(1) == gW.size(1) + 8,
              "ones_col_acc: gw must be [N, K + 8] contiguous");
  if (gB && gB->defined()) TORCH_CHECK(gB->numel() == gW.size(0) && gB->is_contiguous(), "ones_col_acc: gB is [N]");
  bigdl_ones_col_acc(cf(gw, "gw"), mf(gW, "gW"), omf(gB, "gB"), gW.size(0), (int)gW.size(1), (float)sW, (float)sB,
                     stream());
}
void colsum_bf16(const Tensor& x, const Tensor& out) {
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(1) % 8 == 0, "colsum_bf16: x must be [P, K] contiguous, K % 8 == 0");
  TORCH_CHECK(out.is_contiguous() && out.numel() == x.size(1), "colsum_bf16: out must hold K floats");
  Tensor ws;
  if (bigdl_deterministic()) ws = at::empty({(int64_t)BIGDL_DET_SLOTS * x.size(1)}, out.options().dtype(at::kFloat));
  bigdl_colsum_bf16(cbf(x, "x"), mf(out, "out"), x.size(0), (int)x.size(1), stream(),
                    ws.defined() ? ws.data_ptr<float>() : nullptr);
}
int64_t rows_of(const OptT& t, int64_t B, int64_t cols, const char* name) {
  if (!(t && t->defined())) return 0;
  TORCH_CHECK(t->dim() == 2 && t->size(0) == B && t->size(1) >= cols && t->stride(1) == 1, name,
              ": expected [B, >=", cols, "] rows with unit inner stride");
  return t->stride(0);
}
void need_flat(const OptT& t, int64_t n, const char* name) {
  if (t && t->defined()) TORCH_CHECK(t->is_contiguous() && t->numel() == n, name, ": expected ", n, " contiguous elements");
}
void gru_step(int64_t mode, const OptT& A, const Tensor& W, int64_t B, int64_t H, const OptT& xg, const OptT& hprev,
              const OptT& r, const OptT& z, const OptT& n, const OptT& rh16, const OptT& hout, const OptT& h16out,
              const OptT& dout, const OptT& dhp, const OptT& dx, const OptT& dn16, const OptT& drz16, const OptT& dh0) {
  TORCH_CHECK(W.dim() == 2 && W.is_contiguous(), "gru_step: W must be [N, K] contiguous");
  const int64_t N = W.size(0), K = W.size(1);
  TORCH_CHECK(H % 32 == 0 && K % 32 == 0 && N % 16 == 0 && B > 0, "gru_step: H, K multiples of 32, N of 16");
  TORCH_CHECK(mode >= 0 && mode <= 4, "gru_step: bad mode");
  TORCH_CHECK(N == (mode == 0 ? 2 * H : H) && K == (mode == 2 || mode == 4 ? 2 * H : H), "gru_step: W shape vs mode");
  GruStepArgs a{};
  a.mode = (int)mode; a.B = (int)B; a.H = (int)H; a.K = (int)K; a.N = (int)N;
  a.W = cbf(W, "W");
  if (A && A->defined()) { a.lda = rows_of(A, B, K, "A"); a.A = cbf(*A, "A"); }
  need_flat(r, B * H, "r"); need_flat(z, B * H, "z"); need_flat(n, B * H, "n"); need_flat(rh16, B * H, "rh16");
  need_flat(h16out, B * H, "h16out"); need_flat(dhp, B * H, "dhp"); need_flat(dn16, B * H, "dn16");
  need_flat(drz16, B * 2 * H, "drz16"); need_flat(dh0, B * H, "dh0");
  a.ldx = rows_of(xg, B, 3 * H, "xg"); a.ldhp = rows_of(hprev, B, H, "hprev"); a.ldho = rows_of(hout, B, H, "hout");
  a.ldd = rows_of(dout, B, H, "dout"); a.lddx = rows_of(dx, B, 3 * H, "dx");
  a.xg = ocf(xg, "xg"); a.hprev = ocf(hprev, "hprev"); a.r = omf(r, "r"); a.z = omf(z, "z"); a.n = omf(n, "n");
  a.rh16 = ombf(rh16, "rh16"); a.hout = omf(hout, "hout"); a.h16out = ombf(h16out, "h16out"); a.dout = ocf(dout, "dout");
  a.dhp = omf(dhp, "dhp"); a.dx = omf(dx, "dx"); a.dn16 = ombf(dn16, "dn16"); a.drz16 = ombf(drz16, "drz16");
  a.dh0 = omf(dh0, "dh0");
  switch (mode) {
    case 0: TORCH_CHECK(a.xg && a.r && a.z && a.rh16, "gru_step fwd r/z: xg, r, z, rh16 required"); break;
    case 1: TORCH_CHECK(a.A && a.xg && a.z && a.n && a.hout && a.h16out, "gru_step fwd n: A, xg, z, n, hout, h16out required"); break;
    case 2: TORCH_CHECK(a.z && a.n && a.dhp && a.dx && a.dn16 && a.drz16, "gru_step bwd h: z, n, dhp, dx, dn16, drz16 required"); break;
    case 3: TORCH_CHECK(a.A && a.r && a.dhp && a.dx && a.drz16, "gru_step bwd r: A, r, dhp, dx, drz16 required"); break;
    default: TORCH_CHECK(a.dhp && a.dh0, "gru_step bwd h0: dhp, dh0 required"); break;
  }
  TORCH_CHECK(bigdl_gru_step(&a, stream()) == 0, "gru_step: unsupported shape");
}

}  // namespace

void register_host_runtime(pybind11::module& m);   // csrc/host_runtime.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  register_host_runtime(m);
  m.doc() = "bigdl_amd native HIP kernels for gfx950 (MI355X)";
  m.def("conv_nt", &conv_nt, py::arg("src"), py::arg("wt"), py::arg("out"), py::arg("bias"), py::arg("stats"),
        py::arg("geo"), py::arg("taps"), py::arg("relu"), py::arg("addend") = py::none(), py::arg("bn_x") = py::none(),
        py::arg("bn_z") = py::none(), py::arg("bn_mean") = py::none(), py::arg("bn_aff") = py::none(),
        py::arg("bn_red") = py::none(), py::arg("accumulate") = false, py::arg("bn_zm") = py::none(),
        py::arg("addend_zm") = py::none(), py::arg("pre") = py::none());
  m.def("conv_wgrad", &conv_wgrad, py::arg("dy"), py::arg("src"), py::arg("dw"), py::arg("dbias"), py::arg("geo"),
        py::arg("pre") = py::none());
  m.def("transpose_krsc", &transpose_krsc);
  m.def("bn_stats", &bn_stats);
  m.def("bn_finalize", &bn_finalize);
  m.def("bn_apply", &bn_apply, py::arg("x"), py::arg("scale"), py::arg("shift"), py::arg("res"), py::arg("y"),
        py::arg("P"), py::arg("C"), py::arg("relu"), py::arg("zm") = py::none());
  m.def("bn_slot_reduce", &bn_slot_reduce);
  m.attr("STAT_SLOTS") = BIGDL_STAT_SLOTS;
  m.def("bn_bwd_reduce", &bn_bwd_reduce, py::arg("dz"), py::arg("z"), py::arg("x"), py::arg("mean"), py::arg("red"),
        py::arg("P"), py::arg("C"), py::arg("aff") = py::none(), py::arg("zm") = py::none());
  m.def("bn_bwd_apply", &bn_bwd_apply, py::arg("dz"), py::arg("z"), py::arg("x"), py::arg("mean"), py::arg("invstd"),
        py::arg("gamma"), py::arg("red"), py::arg("nslots"), py::arg("coef"), py::arg("dx"), py::arg("dres"),
        py::arg("dgamma"), py::arg("dbeta"), py::arg("P"), py::arg("C"), py::arg("aff") = py::none(),
        py::arg("zm") = py::none(), py::arg("x2") = py::none(), py::arg("mean2") = py::none(),
        py::arg("red2") = py::none());
  m.def("relu_fwd", &relu_fwd);
  m.def("dgrad_fill", &dgrad_fill);
  m.def("maxpool_bwd_bnred", &maxpool_bwd_bnred, "k3 s2 maxpool backward + the producing BN's backward reduction",
        py::arg("dy"), py::arg("idx"), py::arg("dx"), py::arg("g"), py::arg("bx"), py::arg("mean"), py::arg("aff"),
        py::arg("zm"), py::arg("red"));
  m.def("hog_cus", &hog_cus, "n one-wave workgroups holding a whole CU's LDS each, spinning `us` microseconds");
  m.def("spin_us", &spin_us, "device-side delay of `us` microseconds on the current stream (straggler injection)");
  m.def("relu_bwd", &relu_bwd);
  m.def("add_bf16", &add_bf16);
  m.def("nchw_to_nhwc", &nchw_to_nhwc);
  m.def("nchw_to_pairs", &nchw_to_pairs);
  m.def("bmm_nt", &bmm_nt, py::arg("a"), py::arg("b"), py::arg("c"), py::arg("alpha") = 1.0, py::arg("accum") = false);
  m.def("pair_weight", &pair_weight);
  m.def("pair_wgrad_add", &pair_wgrad_add);
  m.def("tensor_apply", &tensor_apply, py::arg("out"), py::arg("a"), py::arg("b"), py::arg("c"), py::arg("size"),
        py::arg("so"), py::arg("sa"), py::arg("sb"), py::arg("sc"), py::arg("op"), py::arg("s0") = 0.0,
        py::arg("s1") = 0.0, py::arg("contiguous") = false);
  m.def("tensor_reduce", &tensor_reduce, py::arg("x"), py::arg("outer"), py::arg("R"), py::arg("inner"), py::arg("op"),
        py::arg("p"), py::arg("out"), py::arg("outi"), py::arg("mean"), py::arg("ws"), py::arg("chunks"));
  m.def("gemm_f32", &gemm_f32);
  m.def("index_op", &index_op);
  m.def("masked_fill", &masked_fill);
  m.def("mask_blocks", &mask_blocks);
  m.def("mask_scan", &mask_scan);
  m.def("mask_write", &mask_write);
  m.def("topk_f32", &topk_f32);
  m.def("gemv_f32", &gemv_f32);
  m.def("fill_bytes", &fill_bytes);
  m.def("copy_rows_i8", &copy_rows_i8);
  m.def("cast_f32_bf16", &cast_f32_bf16);
  m.def("cast_bf16_f32", &cast_bf16_f32);
  m.def("maxpool_fwd", &maxpool_fwd, py::arg("x"), py::arg("y"), py::arg("idx"), py::arg("g"), py::arg("pre") = py::none());
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("softmax_xent", &softmax_xent);
  m.def("sgd_step", &sgd_step, py::arg("w"), py::arg("g"), py::arg("mom"), py::arg("w16"), py::arg("lr"), py::arg("wd"), py::arg("momentum"), py::arg("dampening"), py::arg("nesterov"), py::arg("first"), py::arg("lr_dev") = py::none(), py::arg("seg_off") = py::none(), py::arg("seg_wd") = py::none(), py::arg("base") = 0);
  m.def("adam_step", &adam_step);
  m.def("optim_step", &optim_step);
  m.def("sumsq", &sumsq);
  m.def("scale_f32", &scale_f32);
  m.def("lstm_cell_fwd", &lstm_cell_fwd);
  m.def("lstm_cell_bwd", &lstm_cell_bwd);
  m.def("image_augment", &image_augment);
  m.def("quantize_act", &quantize_act, py::arg("x"), py::arg("q"), py::arg("amax"), py::arg("scale"), py::arg("N"),
        py::arg("P"), py::arg("C"), py::arg("Cp"), py::arg("static_amax") = false);
  m.def("conv_i8", &conv_i8, py::arg("src"), py::arg("wt"), py::arg("out"), py::arg("bias"), py::arg("xscale"),
        py::arg("wscale"), py::arg("geo"), py::arg("taps"), py::arg("relu"), py::arg("xs_const") = 0.0,
        py::arg("out_scale") = 0.0, py::arg("addend") = py::none(), py::arg("add_scale") = 0.0);
  m.def("pool_i8", &pool_i8);
  m.def("act_fwd", &act_fwd);
  m.def("transpose_krsc_batched", &transpose_krsc_batched);
  m.def("image_pipeline", &image_pipeline);
  m.def("act_bwd", &act_bwd);
  m.def("poolnd_fwd", &poolnd_fwd);
  m.def("poolnd_bwd", &poolnd_bwd);
  m.def("upsample_nearest", &upsample_nearest);
  m.def("quantize_nchw_f32", &quantize_nchw_f32);
  m.def("quantize_wim2col_f32", &quantize_wim2col_f32);
  m.def("quantize_rows_bf16", &quantize_rows_bf16);
  m.def("dequantize_rows", &dequantize_rows);
  m.def("nms", &nms);
  m.def("roi_align_fwd", &roi_align_fwd);
  m.def("roi_pool_fwd", &roi_pool_fwd);
  m.def("roi_pool_bwd", &roi_pool_bwd);
  m.def("lrn_fwd", &lrn_fwd);
  m.def("lrn_bwd", &lrn_bwd);
  m.def("dropout", &dropout);
  m.def("lstm_drop_rep", &lstm_drop_rep);
  m.def("lstm_drop_rep_bwd", &lstm_drop_rep_bwd);
  m.def("lstm_pack_gate_w", &lstm_pack_gate_w);
  m.def("embedding_fwd", &embedding_fwd);
  m.def("embedding_bwd", &embedding_bwd);
  m.def("embedding_fwd_ids", &embedding_fwd_ids);
  m.def("embedding_bwd_ids", &embedding_bwd_ids);
  m.def("resize_bilinear_fwd", &resize_bilinear_fwd);
  m.def("resize_bilinear_bwd", &resize_bilinear_bwd);
  m.def("log_softmax_fwd", &log_softmax_fwd);
  m.def("log_softmax_bwd", &log_softmax_bwd);
  m.def("f32_to_bf16_rtz", &f32_to_bf16_rtz);
  m.def("lstm_fwd_step", &lstm_fwd_step);
  m.def("lstm_bwd_step", &lstm_bwd_step);
  m.def("lstm_seq_supported", &lstm_seq_supported);
  m.def("set_lstm_seq", &bigdl_set_lstm_seq);
  m.def("lstm_seq_sync_words", &lstm_seq_sync_words);
  m.def("host_word", [](int64_t slot, bool clear) { return (int64_t)bigdl_host_word((int)slot, clear ? 1 : 0); },
        "read (and optionally clear) a process-wide host-mapped device-error word: 0 persistent timeouts, 1 index range");
  m.def("persistent_error", [](bool clear) { return (int64_t)bigdl_persistent_error(clear ? 1 : 0); },
        "timeouts recorded by persistent (whole-sequence) kernels since the last clear; reads a host-mapped word, no sync");
  m.def("set_seq_timeout_us", &bigdl_set_seq_timeout_us, "bound of every persistent-kernel wait (<= 0: default 2 s)");
  m.def("lstm_seq_fwd", &lstm_seq_fwd);
  m.def("gru_seq_supported", &gru_seq_supported);
  m.def("gru_seq_fwd", &gru_seq_fwd);
  m.def("gru_seq_bwd", &gru_seq_bwd);
  m.def("lstm_seq_bwd", &lstm_seq_bwd);
  m.def("colsum_bf16", &colsum_bf16);
  m.def("ones_col_pack", &ones_col_pack);
  m.def("ones_col_acc", &ones_col_acc);
  m.def("layernorm_fwd", &layernorm_fwd);
  m.def("attn_fwd", &attn_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("bias"), py::arg("H"),
        py::arg("causal"), py::arg("o"), py::arg("lse"), py::arg("drop_p") = 0.0, py::arg("seed") = 0);
  m.def("gconv", &gconv);
  m.def("attn_bwd", &attn_bwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("bias"), py::arg("H"),
        py::arg("causal"), py::arg("o"), py::arg("lse"), py::arg("dout"), py::arg("dq"), py::arg("dk"), py::arg("dv"),
        py::arg("delta_ws"), py::arg("drop_p") = 0.0, py::arg("seed") = 0);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("gru_step", &gru_step, py::arg("mode"), py::arg("A"), py::arg("W"), py::arg("B"), py::arg("H"),
        py::arg("xg") = py::none(), py::arg("hprev") = py::none(), py::arg("r") = py::none(), py::arg("z") = py::none(),
        py::arg("n") = py::none(), py::arg("rh16") = py::none(), py::arg("hout") = py::none(),
        py::arg("h16out") = py::none(), py::arg("dout") = py::none(), py::arg("dhp") = py::none(),
        py::arg("dx") = py::none(), py::arg("dn16") = py::none(), py::arg("drz16") = py::none(),
        py::arg("dh0") = py::none());
  m.def("set_conv_impl", &bigdl_set_conv_impl);
  m.def("set_conv_s1", &bigdl_set_conv_s1);
  m.def("set_conv_halo", &bigdl_set_conv_halo);
  m.def("conv_i8_stem_f32", &conv_i8_stem_f32, "int8 7x7/2 stem straight from the fp32 image (false: not applicable)");
  m.def("set_stem_i8", &bigdl_set_stem_i8, "int8 image stem kernel on (1) / off (0)");
  m.def("set_stem_fwd", &bigdl_set_stem_fwd);
  m.def("set_stem_wgrad", &bigdl_set_stem_wgrad);
  m.def("cu_masked_stream", &cu_masked_stream, "HIP stream restricted to a CU mask (32 CUs per word)");
  m.def("set_conv_sk", &bigdl_set_conv_sk);
  m.def("set_wgrad_halo", &bigdl_set_wgrad_halo);
  m.def("set_deterministic", &bigdl_set_deterministic, "1: bitwise-reproducible reductions (no multi-writer float atomics)");
  m.def("deterministic", &bigdl_deterministic);
  m.def("get_conv_impl", &bigdl_get_conv_impl);
  m.def("set_conv_g4", &bigdl_set_conv_g4);
  m.def("set_conv_shortk", &bigdl_set_conv_shortk);
  m.def("set_conv_p8", &bigdl_set_conv_p8);
  m.def("set_wgrad_p8", &bigdl_set_wgrad_p8);
  m.def("conv_wgrad_uses_p8", &conv_wgrad_uses_p8);
  m.def("get_conv_g4", &bigdl_get_conv_g4);
  m.def("set_wgrad_g3", &bigdl_set_wgrad_g3);
  m.def("get_wgrad_g3", &bigdl_get_wgrad_g3);
  m.def("set_i8_g3", &bigdl_set_i8_g3);
  m.def("set_i8_p8", &bigdl_set_i8_p8);
  m.def("set_i8_s1", &bigdl_set_i8_s1);
  m.def("set_i8_epi", &bigdl_set_i8_epi);
  m.def("set_i8_shortk", &bigdl_set_i8_shortk);
  m.def("get_i8_g3", &bigdl_get_i8_g3);
  m.def("set_i8_cpl", &bigdl_set_i8_cpl);
  m.def("get_i8_cpl", &bigdl_get_i8_cpl);
  m.attr("arch") = "gfx950";
}
