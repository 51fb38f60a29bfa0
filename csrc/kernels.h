// C ABI of the bigdl_amd HIP kernel library (csrc/*.hip). The torch binding layer
// (csrc/bindings.cpp) is the only caller; the kernels themselves never include torch headers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CONV_MAX_TAPS 64
// Implicit-GEMM "NT" convolution launch (forward, or one stride phase of the data gradient):
//   out[orow(m)][n] = sum_{t < ntaps, c < Cs} src[pix(m) + (o_h*mul_h + tap_h[t], o_w*mul_w + tap_w[t])][c]
//                                             * wt[n*ldw + tap_k[t]*Cs + c]
// where m = (nb, o_h, o_w) over the Nb x OH x OW grid and orow(m) places the row in an OHo x OWo output grid
// at (o_h*omul_h + ooff_h, o_w*omul_w + ooff_w) (identity when ident_out).
struct ConvArgs {
  const uint16_t* src;
  const uint16_t* wt;
  uint16_t* out;
  const float* bias;
  float* stats;
  const uint16_t* addend;   // optional [rows][ldo] bf16 added in the epilogue (same placement as out)
  const uint8_t* addzm;     // optional sign mask of the addend ([rows][Ncol / 8] bytes, ldo == Ncol): the addend is
                            // added only where its bit is set (a ResNet block's residual gradient dz * (y > 0))
  // Optional BN-backward reduction of the consumer BatchNorm (data-gradient GEMMs only): with bnred set the
  // epilogue accumulates sum(dm) and sum(dm * (x - mean)) per channel into [STAT_SLOTS][2][Ncol] slots, where
  // dm = out masked by the fused ReLU (z > 0 when bnz is set, else x * aff[c] + aff[Ncol + c] > 0, else no mask)
  const uint16_t* bnx;      // BN input x, same placement / ldo as out
  const uint16_t* bnz;      // BN output (post residual + ReLU) or nullptr
  const uint8_t* bnzm;      // or its sign mask ([rows][Ncol / 8] bytes, bigdl_bn_apply zm), same placement / ldo
  const float* bnmean;      // [Ncol] batch mean
  const float* bnaff;       // [2 Ncol] scale | shift or nullptr
  float* bnred;
  int Nb, Hs, Ws, Cs;
  int OH, OW;
  int mul_h, mul_w;
  int ntaps, ldw;
  int M, Ncol, Kdim, ldo;
  int OHo, OWo, omul_h, omul_w, ooff_h, ooff_w, ident_out;
  int relu;
  short tap_h[CONV_MAX_TAPS], tap_w[CONV_MAX_TAPS], tap_k[CONV_MAX_TAPS];
  // fp32 output instead of bf16 (same placement / ldo), += into it when accum32: weight gradients of GEMM-shaped
  // layers computed as an NT GEMM over transposed operands (LDS-transposed epilogue only; no stats / bn / relu)
  float* out32;
  int accum32;
  // split-K (256 x 256 kernel on grids that do not fill the chip): fp32 partials [ksplit][M][Ncol] in ws, summed
  // by the split-K epilogue kernel, which applies everything the fused epilogue would (bigdl_conv_nt_plan sets them)
  float* ws;
  int ksplit;
  // elements between consecutive source pixels (0 = Cs). pstride < Cs views a row of small pixels as overlapping
  // windows of Cs elements: the bf16 stem's pixel pairs (stem.hip) read 4 consecutive pairs (all 7 width taps of
  // one output column) as one 32-element "pixel" (conv_nt_g4_kernel only)
  int pstride;
  // optional [2 Cs] fp32 scale | shift of a training BatchNorm + ReLU that produced the source: the kernel reads
  // relu(x * scale[c] + shift[c]) (rounded to bf16, bit-equal to bigdl_bn_apply's output) instead of x, and zero
  // padding stays zero — the BN output is never materialised (forward GEMMs of the streaming 1x1 and halo 3x3
  // kernels only: bigdl_conv_pre_applies)
  const float* pre;
};

// int8 convolution epilogue (quant.hip, conv_halo.hip): dequantize with the per-sample input scale and the per-channel
// weight scale, + bias, + an optional int8 residual addend, ReLU, then bf16 / fp32 / requantized int8 stores
struct I8Epi {
  const float* xscale;   // [N] per-sample scale, or nullptr -> xs_const
  float xs_const;
  const float* wscale;   // [Ncol]
  int out_mode;          // 0 bf16, 1 fp32, 2 int8
  float out_inv;         // int8 output: 1 / out_scale
  const int8_t* add8;    // optional int8 residual addend [M][add_ld] (dequantized with add_scale, before the ReLU)
  float add_scale;
  long add_ld;
};

struct WgradArgs {
  const uint16_t* dy;
  const uint16_t* src;
  float* dw;
  float* dbias;
  int Nb, Hs, Ws, Cs, OH, OW, R, S;
  int sh, sw, ph, pw, dh, dwl;
  int M, Ncol, Kdim, ldy;
  int m_per_split;
  float* ws;       // split-K partials [splits][Ncol][Kdim] (nullptr: fp32 atomics into dw)
  int splits;
  float* det_ws;    // deterministic mode with dbias: BIGDL_DET_SLOTS x Ncol floats for the bias column sum
  // optional [2 Cs] scale | shift: src is the input of a training BN + ReLU, read as relu(src * scale + shift)
  // (ConvArgs::pre semantics; the halo 3x3 weight gradient only: bigdl_wgrad_pre_applies)
  const float* pre;
};

extern "C" {
void bigdl_fill_bytes(void* ptr, int value, long bytes, hipStream_t st);
int bigdl_deterministic();
void bigdl_set_deterministic(int v);
// deterministic-mode partial slots (bigdl_colsum_bf16_ld / bigdl_sumsq workspaces: DET_SLOTS x K / DET_SLOTS floats)
#define BIGDL_DET_SLOTS 128
void bigdl_colsum_bf16_ld(const uint16_t* x, float* out, long P, int K, long ld, hipStream_t st,
                          float* det_ws = nullptr);
// 1 when bigdl_conv_nt can apply a->pre inside the kernel that takes the GEMM (else the caller materialises the source)
int bigdl_conv_pre_applies(const ConvArgs* a);
int bigdl_conv_nt(const ConvArgs* a, hipStream_t st);
// 3x3 / stride-1 / pad-1 forward or data-gradient GEMM from halo tiles (conv_halo.hip)
int bigdl_conv_halo_applies(const ConvArgs* a);
int bigdl_conv_halo(const ConvArgs* a, hipStream_t st);
void bigdl_set_conv_halo(int v);
// the same on the i8 matrix cores (int8 activations / weights, I8Epi epilogue; no residual addend)
int bigdl_conv_halo_i8_applies(const ConvArgs* a, const I8Epi* ep);
int bigdl_conv_halo_i8(const ConvArgs* a, const I8Epi* ep, hipStream_t st);
// 7x7 / stride-2 pair-view image stem forward (stem_fwd.hip)
int bigdl_stem_fwd_applies(const ConvArgs* a);
int bigdl_stem_fwd(const ConvArgs* a, hipStream_t st);
void bigdl_set_stem_fwd(int v);
long bigdl_stem_wgrad_plan(const WgradArgs* a);
int bigdl_stem_wgrad(const WgradArgs* a, hipStream_t st);
void bigdl_set_stem_wgrad(int v);
// Kernel choice for bigdl_conv_nt: sets a->ksplit and returns the fp32 workspace elements it needs (0: none).
long bigdl_conv_nt_plan(ConvArgs* a);
// Batched NT GEMM (bmm.hip): C[b][m][n] (=|+=) alpha * sum_k A[b][m][k] B[b][n][k]; A, B bf16 K-contiguous (K % 32
// == 0, row strides % 8 == 0), C fp32. Returns < 0 on unsupported shapes.
int bigdl_bmm_nt(const uint16_t* A, const uint16_t* B, float* C, int batch, int M, int N, int K, long sa, long sb,
                 long sc, int lda, int ldb, int ldc, float alpha, int accum, hipStream_t st);
// Pixel-pair packing for 3/4-channel width-stride-2 stems (stem.hip).
void bigdl_nchw_to_pairs(const float* x, uint16_t* y, int N, int C, int H, int W, int Hp, int Wp, int ph, int pw,
                         hipStream_t st);
void bigdl_pair_weight(const uint16_t* w, uint16_t* wp, int K, int C, int R, int S, const long* strides,
                       hipStream_t st);
void bigdl_pair_wgrad_add(const float* dwp, float* gw, int K, int C, int R, int S, const long* strides, float scale,
                          hipStream_t st);
int bigdl_conv_wgrad(const WgradArgs* a, hipStream_t st);
// Split-K plan for the weight gradient: fills m_per_split / splits; returns the workspace size in floats
// (0 when the single-split path accumulates straight into dw).
long bigdl_conv_wgrad_plan(WgradArgs* a);
void bigdl_transpose_krsc(const uint16_t* w, uint16_t* wt, int K, int RS, int C, hipStream_t st);
// batched form: desc = device int64 [n][6] {w ptr, wt ptr, K, RS, C, first tile}, tiles of 32 x 32 per (rs)
void bigdl_transpose_krsc_batched(const long* desc, int n, int total_tiles, hipStream_t st);

// batch norm (NHWC bf16, fp32 statistics). Statistics / backward-reduction buffers are
// [BIGDL_STAT_SLOTS][2][C] fp32, zeroed by the caller; producers add into slot (block id % slots).
#define BIGDL_STAT_SLOTS 128
void bigdl_bn_stats(const uint16_t* x, float* stats, long P, int C, hipStream_t st);
void bigdl_bn_finalize(const float* stats, int nslots, const float* gamma, const float* beta, float* run_mean,
                       float* run_var, float* save_mean, float* save_invstd, float* scale, float* shift,
                       long P, int C, float eps, float momentum, int training, hipStream_t st);
void bigdl_bn_slot_reduce(const float* in, int nslots, int C, float* out, hipStream_t st);
void bigdl_bn_apply(const uint16_t* x, const float* scale, const float* shift, const uint16_t* res,
                    uint16_t* y, long P, int C, int relu, hipStream_t st, uint8_t* zm = nullptr);
// aff (optional, [scale C | shift C] of the forward apply): with z == nullptr the ReLU mask is recomputed from x.
void bigdl_bn_bwd_reduce(const uint16_t* dz, const uint16_t* z, const uint16_t* x, const float* mean,
                         float* red, long P, int C, const float* aff, hipStream_t st, const uint8_t* zm = nullptr);
void bigdl_bn_bwd_apply(const uint16_t* dz, const uint16_t* z, const uint16_t* x, const float* mean,
                        const float* invstd, const float* gamma, const float* red, int nslots, float* coef,
                        uint16_t* dx, uint16_t* dres, float* dgamma, float* dbeta, long P, int C, int training,
                        const float* aff, hipStream_t st, const uint8_t* zm = nullptr,
                        const uint16_t* x2 = nullptr, const float* mean2 = nullptr, float* red2 = nullptr);
// x2 / mean2 / red2: also accumulate the backward reduction of a second (ReLU-less) BN whose output gradient is dres
// (input x2, same layout; mean2) into the slotted red2 (requires dres; csrc/batchnorm.hip bn_bwd_apply_kernel R2)
// zm: [P][C / 8] sign bytes of the post-ReLU output (bit e of byte (p, g) = channel 8g + e > 0), written by
// bigdl_bn_apply when non-null and read in place of z by the backward passes (1/16 of z's bytes)

// elementwise
void bigdl_relu_fwd(const uint16_t* x, uint16_t* y, long n, hipStream_t st);
void bigdl_spin_us(double us, int* done, hipStream_t st);
void bigdl_dgrad_fill(uint16_t* out, const uint16_t* add, long npix, int H, int W, int C, int sh, int sw, unsigned mask,
                      hipStream_t st);
void bigdl_relu_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dx, long n, hipStream_t st);
void bigdl_add_bf16(const uint16_t* a, const uint16_t* b, uint16_t* y, long n, hipStream_t st);
void bigdl_nchw_f32_to_nhwc_bf16(const float* x, uint16_t* y, int N, int C, int H, int W, int Cp,
                                 hipStream_t st);
void bigdl_cast_f32_bf16(const float* x, uint16_t* y, long n, hipStream_t st);
void bigdl_colsum_bf16(const uint16_t* x, float* out, long P, int K, hipStream_t st, float* det_ws = nullptr);
// [M][K] bf16 -> [M][K + 8] = [x | 1 | 0...]; gW += sW * gw[:, :K], gB += sB * gw[:, K] (gw [N][K + 8] fp32)
void bigdl_ones_col_pack(const uint16_t* x, uint16_t* xe, long M, int K, hipStream_t st);
void bigdl_ones_col_acc(const float* gw, float* gW, float* gB, long N, int K, float sW, float sB, hipStream_t st);
void bigdl_cast_bf16_f32(const uint16_t* x, float* y, long n, hipStream_t st);

// pooling (NHWC bf16)
void bigdl_maxpool_fwd(const uint16_t* x, uint16_t* y, uint8_t* idx, int N, int H, int W, int C, int OH,
                       int OW, int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t st, const float* pre = nullptr);
int bigdl_maxpool_pre_applies(int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh, int sw);
int bigdl_stem_i8_applies(const ConvArgs* a, const I8Epi* ep);
void bigdl_set_stem_i8(int v);
int bigdl_stem_i8_f32(const ConvArgs* a, const I8Epi* ep, const float* img, int C, int W, float inv, hipStream_t st);
int bigdl_stem_i8(const ConvArgs* a, const I8Epi* ep, hipStream_t st);
void bigdl_split_reduce_f32(const float* ws, float* dw, long n, int splits, hipStream_t st);
int bigdl_maxpool_bwd_bnred_applies(int N, int H, int W, int C, int OH, int OW, int kh, int kw, int sh, int sw, int ph,
                                    int pw);
void bigdl_maxpool_bwd_bnred(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int C, int OH, int OW,
                             const uint16_t* bx, const float* mean, const float* aff, const uint8_t* zm, float* red,
                             hipStream_t st);
void bigdl_maxpool_bwd(const uint16_t* dy, const uint8_t* idx, uint16_t* dx, int N, int H, int W, int C,
                       int OH, int OW, int kh, int kw, int sh, int sw, int ph, int pw, hipStream_t st);
void bigdl_avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int H, int W, int C, int OH, int OW, int kh,
                       int kw, int sh, int sw, int ph, int pw, int count_pad, hipStream_t st);
void bigdl_avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int H, int W, int C, int OH, int OW, int kh,
                       int kw, int sh, int sw, int ph, int pw, int count_pad, hipStream_t st);

// fused log-softmax + NLL (cross entropy) over rows of logits
void bigdl_softmax_xent(const uint16_t* logits_bf16, const float* logits_f32, const float* labels,
                        float* loss, uint16_t* dlogits_bf16, float* dlogits_f32, int B, int K,
                        float label_base, float grad_scale, hipStream_t st);

// optimizers over flat fp32 buffers (optional bf16 shadow written in the same pass)
void bigdl_sgd_step(float* w, const float* g, float* mom, uint16_t* w16, long n, const float* lr_dev, float lr,
                    float wd, float momentum, float dampening, int nesterov, int first, const long* seg_off,
                    const float* seg_wd, int nseg, long base, hipStream_t st);
void bigdl_adam_step(float* w, const float* g, float* m, float* v, uint16_t* w16, long n, float lr,
                     float beta1, float beta2, float eps, float wd, float bc1, float bc2, hipStream_t st);
void bigdl_sumsq(const float* x, float* out, long n, hipStream_t st, float* det_ws = nullptr);
void bigdl_scale_f32(float* x, long n, const float* scale_dev, float scale, hipStream_t st);

// LSTM cell pointwise (gates pre-activations -> c, h), fwd & bwd
void bigdl_lstm_cell_fwd(const float* gates, const float* c_prev, float* c, float* h, float* act, int B,
                         int H, hipStream_t st);
void bigdl_lstm_cell_bwd(const float* act, const float* c_prev, const float* c, const float* dh,
                         const float* dc_next, float* dgates, float* dc_prev, int B, int H, hipStream_t st);

// Int8 inference: per-sample activation quantization (x [N][P][C] bf16 or fp32 -> int8 [N][P][Cp]) and the
// dequantizing implicit-GEMM conv on the i8 MFMA (src/wt are int8 images; out bf16 or fp32).
int bigdl_quantize_act(const void* x, int is_bf16, int8_t* q, float* amax, float* scale, int N, long P, int C,
                       int Cp, int static_amax, hipStream_t st);
// xscale: [N] per-sample activation scales or nullptr (xs_const for the whole tensor); out_mode 0 bf16, 1 fp32,
// 2 int8 requantized with out_inv = 1 / out_scale. Output rows are a->ldo elements apart.
// add8 (optional): int8 residual addend [M][add_ld] with scale add_scale, summed before the ReLU.
int bigdl_conv_i8(const ConvArgs* a, const float* xscale, float xs_const, const float* wscale, int out_mode,
                  float out_inv, const int8_t* add8, float add_scale, long add_ld, hipStream_t st);
// int8 NHWC pooling (max or average, same scale in and out; output rows ldo apart), graph-input quantizer
// (fp32 NCHW -> int8 NHWC, static scale), bf16 rows -> int8 rows at a channel offset, int8 rows -> bf16.
void bigdl_pool_i8(const int8_t* x, int8_t* y, int N, int H, int W, int Cp, int OH, int OW, int kh, int kw, int sh,
                   int sw, int ph, int pw, int avg, int count_pad, long ldo, hipStream_t st);
void bigdl_quantize_nchw_f32(const float* x, int8_t* q, int N, int C, int HW, int Cp, float inv, hipStream_t st);
void bigdl_quantize_wim2col_f32(const float* x, int8_t* y, int N, int C, int H, int W, int OW, int S, int sw, int pw,
                                float inv, hipStream_t st);
void bigdl_quantize_rows_bf16(const uint16_t* x, int8_t* q, long P, int C, long ldq, float inv, hipStream_t st);
void bigdl_dequantize_rows(const int8_t* q, uint16_t* y, long P, int C, long ld, float scale, hipStream_t st);

// tensor_math.hip: native TensorMath backend (strided apply, reductions, fp32 MFMA GEMM / GEMV)
int bigdl_tensor_apply(float* out, const float* a, const float* b, const float* c, int nd, const long* size,
                       const long* so, const long* sa, const long* sb, const long* sc, int op, float s0, float s1,
                       int contiguous, hipStream_t st);
int bigdl_index_op(int op, float* a, const void* idx, int idx_i64, const float* b, float* out, long outer, long R,
                   long n, long inner, long Rsrc, int* err, hipStream_t st);
void bigdl_masked_fill(float* x, const float* mask, float v, long n, hipStream_t st);
long bigdl_mask_blocks(long n);
void bigdl_mask_scan(const float* mask, long n, int* counts, hipStream_t st);
void bigdl_mask_write(int copy, float* x, const float* mask, const float* src, float* out, long n, const int* counts,
                      long nsrc, hipStream_t st);
int bigdl_topk(const float* x, long outer, long R, long inner, int k, int largest, float* vals, float* inds,
               hipStream_t st);
int bigdl_tensor_reduce(const float* x, long outer, long R, long inner, int op, float p, float* out, float* outi,
                        int mean, float* ws, long chunks, hipStream_t st);
int bigdl_gemm_f32(const float* A, const float* B, const float* Min, float* C, int batch, int M, int N, int K,
                   const long* s, float alpha, float beta, hipStream_t st);
int bigdl_gemv_f32(const float* A, const float* x, const float* Min, float* y, int M, int K, long sam, long sak,
                   long sx, long smi, long sy, float alpha, float beta, hipStream_t st);
void bigdl_copy_rows_i8(const int8_t* src, int8_t* dst, long rows, int C, long lds, long ldd, hipStream_t st);
void bigdl_set_conv_impl(int impl);
void bigdl_set_conv_s1(int v);
void bigdl_set_conv_sk(int v);
// 3x3 / stride 1 / pad 1 weight gradient from halo tiles (wgrad_halo.hip): plan returns its splits (0 = n/a)
void bigdl_set_wgrad_halo(int v);
// LSTM with per-gate dropout masks (lstm_drop.hip)
int bigdl_lstm_drop_rep(const void* x, int x_bf16, long xs_b, long xs_t, uint16_t* y, long ys_g, int B, int T, int K,
                        int Kp, int ones, float p, float mul, unsigned long long seed, long long off, hipStream_t st);
int bigdl_lstm_drop_rep_bwd(const float* dy, long dys_g, int ldy, float* dx, long dxs_b, long dxs_t, const float* add,
                            long as_b, long as_t, int B, int T, int K, float p, float mul, unsigned long long seed,
                            long long off, hipStream_t st);
void bigdl_lstm_pack_gate_w(const float* W, const float* b1, const float* b2, int H, int Kin, int Kp, uint16_t* out,
                            uint16_t* outT, hipStream_t st);
int bigdl_wgrad_halo_plan(WgradArgs* a);
// 1 when bigdl_conv_wgrad applies a->pre on load (the halo kernel takes the GEMM), else the caller materialises src
int bigdl_wgrad_pre_applies(const WgradArgs* a);
int bigdl_wgrad_halo(const WgradArgs* a, hipStream_t st);
void bigdl_set_i8_s1(int v);
int bigdl_get_conv_impl();
void bigdl_set_conv_g4(int v);
void bigdl_set_conv_shortk(int v);
void bigdl_set_conv_p8(int v);
void bigdl_set_wgrad_p8(int v);
int bigdl_conv_wgrad_uses_p8(const WgradArgs* a);
int bigdl_get_conv_g4();
void bigdl_set_wgrad_g3(int v);
int bigdl_get_wgrad_g3();
void bigdl_set_i8_g3(int v);
void bigdl_set_i8_p8(int v);
void bigdl_set_i8_epi(int v);
void bigdl_set_i8_shortk(int v);
int bigdl_get_i8_g3();
void bigdl_set_i8_cpl(int v);
int bigdl_get_i8_cpl();

// Input pipeline: crop + flip + channel reorder + normalise of a uint8 [N, H, W, 3] BGR batch.
// params: int32 [N][3] = (y0, x0, flip). Output fp32 NCHW [N, 3, OH, OW] or bf16 NHWC [N, OH, OW, 3].
void bigdl_image_augment(const uint8_t* src, const int* params, void* out, int N, int H, int W, int OH, int OW,
                         const float* mean, const float* inv_std, int rgb, int nhwc_bf16, hipStream_t st);
// variable-size batch: resized crop + flip + colour jitter + normalise (csrc/image.hip image_pipeline_kernel);
// offs = int64 byte offset of each image, prm = 16 floats per image (layout in image.hip)
void bigdl_image_pipeline(const uint8_t* src, const long* offs, const float* prm, void* out, int N, int OH, int OW,
                          const float* mean, const float* inv_std, int rgb, int nhwc_bf16, hipStream_t st);

// Detection (csrc/detection.hip): greedy NMS over score-sorted boxes (mask_ws: n * ceil(n/64) uint64),
// RoiAlign forward, RoiPooling forward (argmax) / backward.
int bigdl_nms(const float* boxes_sorted, int n, float thresh, int normalized, int max_keep,
              unsigned long long* mask_ws, int* keep_out, int* count_out, hipStream_t st);
int bigdl_roi_align_fwd(const float* x, const float* rois, float* out, int R, int rcols, int C, int H, int W,
                        int PH, int PW, float scale, int sampling, hipStream_t st);
int bigdl_roi_pool_fwd(const float* x, const float* rois, float* out, int* argmax, int R, int C, int H, int W,
                       int PH, int PW, float scale, hipStream_t st);
int bigdl_roi_pool_bwd(const float* gy, const int* argmax, const float* rois, float* gx, int R, int C, int H, int W,
                       int PH, int PW, hipStream_t st);

// Misc NN kernels (csrc/nn_misc.hip): LRN across channels (NCHW fp32), Philox dropout (mask regenerated in
// backward), embedding gather / atomic scatter-add, TF-style bilinear resize (NCHW fp32), row log-softmax,
// fp32 -> bf16 round-toward-zero (FP16CompressedTensor parity).
void bigdl_lrn_fwd(const float* x, float* y, float* scale, int N, int C, long HW, int size, float alpha, float beta,
                   float k, hipStream_t st);
void bigdl_lrn_bwd(const float* x, const float* y, const float* scale, const float* gy, float* gx, int N, int C, long HW,
                   int size, float alpha, float beta, hipStream_t st);
void bigdl_dropout(const void* x, void* y, int is_bf16, long n, float p, float mul, unsigned long long seed,
                   hipStream_t st);
void bigdl_embedding_fwd(const float* W, const long* idx, float* out, long rows, int D, long nIndex, hipStream_t st);
void bigdl_embedding_fwd_ids(const float* W, const void* ids, int ids_long, float* out, long rows, int D, long nIndex,
                             int mask_zero, hipStream_t st);
void bigdl_embedding_bwd_ids(const void* gout, int gout_bf16, const void* ids, int ids_long, float* gW, long rows, int D,
                             long nIndex, long pad, float scale, hipStream_t st);
void bigdl_embedding_bwd(const float* gout, const long* idx, float* gW, long rows, int D, long nIndex, float scale,
                         hipStream_t st);
void bigdl_resize_bilinear_fwd(const float* x, float* y, long NC, int H, int W, int OH, int OW, float sh, float sw,
                               hipStream_t st);
void bigdl_resize_bilinear_bwd(const float* gy, float* gx, long NC, int H, int W, int OH, int OW, float sh, float sw,
                               hipStream_t st);
void bigdl_log_softmax_fwd(const float* x, float* y, long rows, int cols, hipStream_t st);
void bigdl_log_softmax_bwd(const float* y, const float* gy, float* gx, long rows, int cols, hipStream_t st);
void bigdl_f32_to_bf16_rtz(const float* x, uint16_t* y, long n, hipStream_t st);

// Fused LSTM steps (csrc/lstm.hip). W16 [4H][H] bf16 (gate blocks i, g, f, o), WT16 = W^T [H][4H] bf16.
// Row strides: xg/h_out/acts/dout/dg_out rows are batch rows (ldx, ldh, lda, ldd, ldg elements apart).
int bigdl_lstm_fwd_step(const uint16_t* W16, const uint16_t* h16_prev, const float* xg, long ldx, const float* c_prev,
                        float* c_out, float* h_out, long ldh, uint16_t* h16_out, float* acts, long lda, int B, int H,
                        hipStream_t st);
int bigdl_lstm_bwd_step(const uint16_t* WT16, const uint16_t* dg16_next, const float* dout, long ldd,
                        const float* dh_ext, const float* acts, long lda, const float* c_prev, const float* c_t,
                        float* dc, float* dg_out, long ldg, uint16_t* dg16_out, int B, int H, hipStream_t st);
// Whole-sequence persistent LSTM (csrc/lstm_seq.hip): one launch per direction, W resident in VGPRs.
int bigdl_lstm_seq_supported(int B, int H);
void bigdl_set_lstm_seq(int v);
int bigdl_lstm_seq_sync_words();
int bigdl_gru_seq_supported(int B, int H);
int bigdl_gru_seq(int bwd, const uint16_t* Wrz16, const uint16_t* Wn16, const float* xg, const float* h0,
                  uint16_t* h16, uint16_t* rh16, float* gates, float* out, const float* dout, const float* dhT,
                  float* dx, uint16_t* dn16, uint16_t* drz16, float* dh0, unsigned* sync, int B, int H, int T,
                  hipStream_t st);
int bigdl_persistent_error(int clear);
unsigned* bigdl_host_word_dev(int slot);
int bigdl_host_word(int slot, int clear);
void bigdl_set_seq_timeout_us(double us);
void bigdl_hog_cus(int n, double us, int* done, hipStream_t st);
unsigned* bigdl_persistent_err_dev();
unsigned long long bigdl_seq_spin_ticks();
int bigdl_lstm_seq_fwd(const uint16_t* W16, const void* xg, const float* c0, uint16_t* h16, void* out, float* hT,
                       float* cs, float* acts, unsigned* sync, int B, int H, int T, int bf16io, hipStream_t st);
int bigdl_lstm_seq_bwd(const uint16_t* W16, const void* dout, const float* dhT, const float* dcT, const float* acts,
                       const float* cs, const float* c0, uint16_t* dg16, void* dxg, float* dc0, float* dh0,
                       unsigned* sync, int B, int H, int T, int bf16io, hipStream_t st);

// Fused GRU steps (csrc/gru.hip). mode: 0 fwd r/z, 1 fwd n + h, 2 bwd dh_t + dn/dz, 3 bwd dr + r-path, 4 bwd dh_0.
// GEMM D[b][n] = sum_k A[b][k] W[n][k] (A rows lda apart; W [N][K] contiguous); row strides of the fp32 per-step
// views (xg, hprev, hout, dout, dx) are in elements; every other buffer is a contiguous [B][H] ([B][2H] drz16).
typedef struct {
  const uint16_t* A; long lda; const uint16_t* W; int B, H, K, N, mode;
  const float* xg; long ldx; const float* hprev; long ldhp; float* r; float* z; float* n; uint16_t* rh16;
  float* hout; long ldho; uint16_t* h16out; const float* dout; long ldd; float* dhp; float* dx; long lddx;
  uint16_t* dn16; uint16_t* drz16; float* dh0;
} GruStepArgs;
int bigdl_gru_step(const GruStepArgs* a, hipStream_t st);

// Layer normalisation over the last dimension (csrc/layernorm.hip), D <= 4096, fp32 rows.
int bigdl_layernorm_fwd(const float* x, const float* g, const float* b, float* y, float* mean, float* rstd, long rows,
                        int D, float eps, hipStream_t st);
int bigdl_layernorm_bwd(const float* dy, const float* x, const float* g, const float* mean, const float* rstd,
                        float* dx, float* dg, float* db, long rows, int D, hipStream_t st);

// Fused attention (csrc/attention.hip). q/k/v bf16 [BH][L][D] (D = 32, 64, 96 or 128), bias fp32 through element
// strides (sb, sh, sq, sk) or nullptr, o / dq / dk / dv / dout fp32, lse / delta fp32 [BH][Lq]; attention dropout
// with probability drop_p (0: none) from a counter-based hash of (seed, row, key), regenerated by the backward.
typedef struct {
  const uint16_t* q; const uint16_t* k; const uint16_t* v; const float* bias; long sb, sh, sq, sk;
  float* o; float* lse; const float* dout; const float* delta; float* dq; float* dk; float* dv;
  int BH, H, Lq, Lk, D, causal;
  float drop_p; unsigned long long seed;
} AttnCall;
int bigdl_attn_fwd(const AttnCall* c, hipStream_t st);
int bigdl_attn_bwd(const AttnCall* c, float* delta_ws, hipStream_t st);

// Adaptive OptimMethod updates on flat fp32 buffers (csrc/optim.hip): method 0 Adagrad (a = lr, b = weight decay),
// 1 RMSprop (a = lr, b = decay rate, c = eps), 2 Adadelta (a = decay rate, b = eps), 3 Adamax (a = lr / (1 - b1^t),
// b = b1, c = b2, d = eps), 4 Ftrl (a = lr, b = lr power, c = l1, d = l2, e = l2 shrinkage); s1 / s2 are the state
// buffers (s2 may be null for Adagrad / RMSprop); w16 (optional) receives the bf16 copy of the updated weights.
typedef struct { float a, b, c, d, e; } OptimHP;
int bigdl_optim_step(int method, const OptimHP* hp, float* x, const float* g, float* s1, float* s2, uint16_t* w16,
                     long n, hipStream_t st);

// Point-wise activations (csrc/activation.hip): kind codes in bigdl_amd/nn/activation.py _NATIVE_KIND; x, y, dy, dx
// are contiguous bf16 (bf16 = 1) or fp32 buffers of n elements; returns -1 for an unknown kind.
int bigdl_act_fwd(const void* x, void* y, long n, int bf16, int kind, float a, float b, hipStream_t st);
int bigdl_act_bwd(const void* x, const void* y, const void* dy, void* dx, long n, int bf16, int kind, float a,
                  float b, hipStream_t st);

// N-d window pooling / nearest up-sampling (csrc/pool_nd.hip) over a dense [B][D][H][W][C] view (C innermost):
// input D x H x W, output OD x OH x OW, window (kd, kh, kw), stride, padding (for up-sampling kd / kh / kw are the
// integer scale factors and stride / padding are unused). idx (max pooling) holds the input position (d*H+h)*W+w.
typedef struct { int B, D, H, W, C, OD, OH, OW, kd, kh, kw, sd, sh, sw, pd, ph, pw; } PoolNdGeo;
int bigdl_poolnd_fwd(const void* x, void* y, int* idx, const PoolNdGeo* g, int max_mode, int count_pad, int bf16,
                     hipStream_t st);
int bigdl_poolnd_bwd(const void* dy, const int* idx, void* dx, const PoolNdGeo* g, int max_mode, int count_pad,
                     int bf16, hipStream_t st);
int bigdl_upsample_nearest(const void* src, void* dst, const PoolNdGeo* g, int backward, int bf16, hipStream_t st);

// Direct grouped / depthwise convolution, fp32 NCHW (csrc/grouped_conv.hip). pass 0 forward (x, w, b -> y),
// 1 data gradient (dy, w -> dx), 2 weight / bias gradient (dy, x -> dwt, db accumulated).
typedef struct {
  const float* x; const float* w; const float* b; float* y; const float* dy; float* dx; float* dwt; float* db;
  int N, C, H, W, K, OH, OW, R, S, sh, sw, ph, pw, dh, dw, G;
} GConvCall;
int bigdl_gconv(const GConvCall* c, int pass, hipStream_t st);
}
