// Pixel-pair packing for small-channel, width-stride-2 input convolutions (the ResNet / Inception stems: 3
// channels, 7x7 or 3x3, stride 2) on gfx950.
//
// The implicit-GEMM kernels (conv_igemm.hip) gather 16-byte granules of 8 channels of ONE pixel; a 3-channel image
// padded to 8 channels makes 5/8 of every MFMA operand zeros (reference stem: S/nn/SpatialConvolution.scala with
// nInputPlane = 3; MKL-DNN pads the same way). With stride 2 along the width, the taps s = 2j and s = 2j + 1 of
// output column ow read the adjacent input pixels 2(ow + j) and 2(ow + j) + 1 of the zero-padded image. So the
// image is stored zero-padded as NHWC with 4 channels (8 bytes per pixel) and viewed as [N][Hp][Wp/2][8] pixel
// PAIRS: one granule = (pixel 2q, channels 0..3 | pixel 2q + 1, channels 0..3) = two taps. The convolution over
// that view has S2 = ceil(S/2) pair taps, width stride 1, no padding (the image is pre-padded), and a reduction of
// R * S2 * 8 instead of R * S * 8 (7x7: 224 vs 392, 1.75x fewer MFMA FLOPs and operand bytes), with no bounds
// checks on the gather. Weights are repacked to w'[k][r][j][e*4 + c] = w[k][c][r][2j + e] (zero past C or S); the
// weight gradient of the pair view is scattered back through the same map.
#include "common.h"
#include "kernels.h"

namespace {

// y[n][hp][wp][0..3] = x[n][c][hp - ph][wp - pw] (0 outside the image or for c >= C); one 8-byte store per pixel.
__global__ __launch_bounds__(256) void nchw_to_pairs_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                            int N, int C, int H, int W, int Hp, int Wp, int ph,
                                                            int pw) {
  const long total = (long)N * Hp * Wp;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int wp = (int)(i % Wp);
    const long t = i / Wp;
    const int hp = (int)(t % Hp);
    const int n = (int)(t / Hp);
    const int h = hp - ph, w = wp - pw;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
      const float* p = x + ((size_t)n * C * H + h) * W + w;
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < C) v[c] = p[(size_t)c * H * W];
    }
    *reinterpret_cast<v2u*>(y + (size_t)i * 4) = v2u{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
  }
}

// wp[k][r][j][e*4 + c] = w[k][c][r][2j + e] (element strides of w given), zero for c >= C or 2j + e >= S.
__global__ __launch_bounds__(256) void pair_weight_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wp,
                                                          int K, int C, int R, int S, int S2, long sk, long sc,
                                                          long sr, long ss) {
  const int total = K * R * S2 * 8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int q = i & 7;
    int t = i >> 3;
    const int j = t % S2;
    t /= S2;
    const int r = t % R;
    const int k = t / R;
    const int e = q >> 2, c = q & 3, s = 2 * j + e;
    wp[i] = (c < C && s < S) ? w[k * sk + c * sc + r * sr + s * ss] : (bf16_t)0;
  }
}

// gw[k][c][r][s] += scale * dwp[k][r][j][e*4 + c] for s = 2j + e < S, c < C (element strides of gw given).
__global__ __launch_bounds__(256) void pair_wgrad_add_kernel(const float* __restrict__ dwp, float* __restrict__ gw,
                                                             int K, int C, int R, int S, int S2, long sk, long sc,
                                                             long sr, long ss, float scale) {
  const int total = K * C * R * S;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int s = i % S;
    int t = i / S;
    const int r = t % R;
    t /= R;
    const int c = t % C;
    const int k = t / C;
    const int j = s >> 1, e = s & 1;
    gw[k * sk + c * sc + r * sr + s * ss] += scale * dwp[(((size_t)k * R + r) * S2 + j) * 8 + e * 4 + c];
  }
}

int blocks_for(long n) {
  long b = (n + 255) / 256;
  return (int)(b > 16384 ? 16384 : (b < 1 ? 1 : b));
}

}  // namespace

extern "C" {

void bigdl_nchw_to_pairs(const float* x, uint16_t* y, int N, int C, int H, int W, int Hp, int Wp, int ph, int pw,
                         hipStream_t st) {
  nchw_to_pairs_kernel<<<blocks_for((long)N * Hp * Wp), 256, 0, st>>>(x, y, N, C, H, W, Hp, Wp, ph, pw);
  HIP_LAUNCH_CHECK();
}

void bigdl_pair_weight(const uint16_t* w, uint16_t* wp, int K, int C, int R, int S, const long* strides,
                       hipStream_t st) {
  const int S2 = (S + 1) / 2;
  pair_weight_kernel<<<blocks_for((long)K * R * S2 * 8), 256, 0, st>>>(w, wp, K, C, R, S, S2, strides[0], strides[1],
                                                                        strides[2], strides[3]);
  HIP_LAUNCH_CHECK();
}

void bigdl_pair_wgrad_add(const float* dwp, float* gw, int K, int C, int R, int S, const long* strides, float scale,
                          hipStream_t st) {
  const int S2 = (S + 1) / 2;
  pair_wgrad_add_kernel<<<blocks_for((long)K * C * R * S), 256, 0, st>>>(dwp, gw, K, C, R, S, S2, strides[0],
                                                                          strides[1], strides[2], strides[3], scale);
  HIP_LAUNCH_CHECK();
}

}  // extern "C"
