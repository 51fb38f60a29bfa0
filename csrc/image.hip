// Device-side input pipeline for gfx950: one kernel does crop + horizontal flip + BGR->RGB reorder +
// per-channel (x - mean) * inv_std + layout/dtype conversion of a whole decoded uint8 batch.
//
// Replaces the per-image host loops of the reference (S/dataset/image/BGRImgCropper.scala, HFlip.scala,
// BGRImgNormalizer.scala, BGRImage.copyTo in Types.scala:153, MTLabeledBGRImgToBatch.scala): the host only
// decodes into a pinned uint8 HWC batch; the device produces the training tensor directly.
// Memory-bound: 3 bytes in, 3 outputs out per thread; each thread handles PIX consecutive output pixels of
// one row so the uint8 loads of a wave cover contiguous bytes.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int PIX = 4;

template <bool NHWC_BF16>
__global__ void __launch_bounds__(256) augment_kernel(const uint8_t* __restrict__ src, const int* __restrict__ params,
                                                      void* __restrict__ out, int N, int H, int W, int OH, int OW,
                                                      float m0, float m1, float m2, float i0, float i1, float i2,
                                                      int rgb) {
  const int groups_per_row = (OW + PIX - 1) / PIX;
  const long total = (long)N * OH * groups_per_row;
  for (long g = blockIdx.x * (long)blockDim.x + threadIdx.x; g < total; g += (long)gridDim.x * blockDim.x) {
    const int gx = (int)(g % groups_per_row);
    const long r = g / groups_per_row;
    const int oy = (int)(r % OH);
    const int n = (int)(r / OH);
    const int y0 = params[3 * n], x0 = params[3 * n + 1], flip = params[3 * n + 2];
    const int sy = y0 + oy;
    const uint8_t* row = src + ((long)n * H + sy) * (long)W * 3;
#pragma unroll
    for (int k = 0; k < PIX; ++k) {
      const int ox = gx * PIX + k;
      if (ox >= OW) break;
      const int sx = flip ? x0 + OW - 1 - ox : x0 + ox;
      const uint8_t* px = row + (long)sx * 3;
      const float b = px[0], gch = px[1], rch = px[2];
      const float c0 = rgb ? rch : b, c2 = rgb ? b : rch;
      const float v0 = (c0 - m0) * i0, v1 = (gch - m1) * i1, v2 = (c2 - m2) * i2;
      if (NHWC_BF16) {
        uint16_t* o = reinterpret_cast<uint16_t*>(out) + (((long)n * OH + oy) * OW + ox) * 3;
        o[0] = f2bf(v0);
        o[1] = f2bf(v1);
        o[2] = f2bf(v2);
      } else {
        float* o = reinterpret_cast<float*>(out);
        const long plane = (long)OH * OW;
        const long base = (long)n * 3 * plane + (long)oy * OW + ox;
        o[base] = v0;
        o[base + plane] = v1;
        o[base + 2 * plane] = v2;
      }
    }
  }
}

}  // namespace

extern "C" void bigdl_image_augment(const uint8_t* src, const int* params, void* out, int N, int H, int W, int OH,
                                    int OW, const float* mean, const float* inv_std, int rgb, int nhwc_bf16,
                                    hipStream_t st) {
  const long groups = (long)N * OH * ((OW + PIX - 1) / PIX);
  const int blocks = (int)std::min<long>((groups + 255) / 256, 16384);
  if (nhwc_bf16)
    augment_kernel<true><<<blocks, 256, 0, st>>>(src, params, out, N, H, W, OH, OW, mean[0], mean[1], mean[2],
                                                 inv_std[0], inv_std[1], inv_std[2], rgb);
  else
    augment_kernel<false><<<blocks, 256, 0, st>>>(src, params, out, N, H, W, OH, OW, mean[0], mean[1], mean[2],
                                                  inv_std[0], inv_std[1], inv_std[2], rgb);
  HIP_LAUNCH_CHECK();
}
