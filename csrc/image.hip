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

// ------------------------------------------------------------------------------------------------------------
// Variable-size batch pipeline: random-resized crop (bilinear, half-pixel centres, the crop box resized to OH x OW),
// horizontal flip, colour jitter (brightness / contrast / saturation / hue in a per-image order) and channel
// normalisation, from a packed uint8 BGR buffer of differently sized decoded images straight to the training
// tensor. Reference: S/transform/vision/image/augmentation/{RandomResize, Resize, Crop, HFlip, Brightness, Contrast,
// Saturation, Hue, ColorJitter, ChannelNormalize}.scala; the float math (OpenCV convertTo saturation to [0, 255],
// 8-bit HSV convention) is the host implementation's in bigdl_amd/transform/vision/image/augmentation.py, so the
// device batch equals the host chain on the same parameters.
// Per image: offs[n] = byte offset of its H x W x 3 image; prm[n * IMG_P ..] = {H, W, y0, x0, ch, cw, flip, nops,
// op0, a0, op1, a1, op2, a2, op3, a3}; op codes 1 brightness (+a), 2 contrast (*a), 3 saturation (S*a), 4 hue (H+a).
constexpr int IMG_P = 16;

__device__ __forceinline__ float sat255(float v) { return fminf(fmaxf(v, 0.f), 255.f); }

__device__ __forceinline__ void bgr2hsv(float b8, float g8, float r8, float& h, float& s, float& v) {
  const float b = b8 / 255.f, g = g8 / 255.f, r = r8 / 255.f;
  const float mx = fmaxf(r, fmaxf(g, b)), mn = fminf(r, fminf(g, b)), d = mx - mn;
  s = mx > 0.f ? d / fmaxf(mx, 1e-12f) : 0.f;
  const float dz = fmaxf(d, 1e-12f);
  float hh = 0.f;
  if (mx == r) hh = 60.f * (g - b) / dz;
  else if (mx == g) hh = 120.f + 60.f * (b - r) / dz;
  else hh = 240.f + 60.f * (r - g) / dz;
  if (d == 0.f) hh = 0.f;
  hh = hh - 360.f * floorf(hh / 360.f);
  h = hh * 0.5f;
  s *= 255.f;
  v = mx * 255.f;
}

__device__ __forceinline__ void hsv2bgr(float h8, float s8, float v8, float& b, float& g, float& r) {
  float h = h8 * 2.f;
  h = h - 360.f * floorf(h / 360.f);
  const float s = fminf(fmaxf(s8 / 255.f, 0.f), 1.f), v = fminf(fmaxf(v8 / 255.f, 0.f), 1.f);
  const float c = v * s, hp = h / 60.f;
  const float x = c * (1.f - fabsf(hp - 2.f * floorf(hp / 2.f) - 1.f));
  const int i = min(max((int)floorf(hp), 0), 5);
  float rr, gg, bb;
  switch (i) {
    case 0: rr = c; gg = x; bb = 0.f; break;
    case 1: rr = x; gg = c; bb = 0.f; break;
    case 2: rr = 0.f; gg = c; bb = x; break;
    case 3: rr = 0.f; gg = x; bb = c; break;
    case 4: rr = x; gg = 0.f; bb = c; break;
    default: rr = c; gg = 0.f; bb = x; break;
  }
  const float m = v - c;
  b = (bb + m) * 255.f; g = (gg + m) * 255.f; r = (rr + m) * 255.f;
}

template <bool NHWC_BF16>
__global__ void __launch_bounds__(256) image_pipeline_kernel(const uint8_t* __restrict__ src, const long* __restrict__ offs,
                                                             const float* __restrict__ prm, void* __restrict__ out,
                                                             int N, int OH, int OW, float m0, float m1, float m2,
                                                             float i0, float i1, float i2, int rgb) {
  const long total = (long)N * OH * OW;
  for (long e = blockIdx.x * 256l + threadIdx.x; e < total; e += (long)gridDim.x * 256) {
    const int ox = (int)(e % OW);
    const long r0 = e / OW;
    const int oy = (int)(r0 % OH);
    const int n = (int)(r0 / OH);
    const float* p = prm + (long)n * IMG_P;
    const int H = (int)p[0], W = (int)p[1];
    const int y0 = (int)p[2], x0 = (int)p[3], ch = (int)p[4], cw = (int)p[5];
    const int fx = p[6] != 0.f ? OW - 1 - ox : ox;
    // bilinear, align_corners = false, inside the crop box
    const float sy = fmaxf((oy + 0.5f) * ((float)ch / OH) - 0.5f, 0.f);
    const float sx = fmaxf((fx + 0.5f) * ((float)cw / OW) - 0.5f, 0.f);
    const int iy = min((int)sy, ch - 1), ix = min((int)sx, cw - 1);
    const int iy1 = min(iy + 1, ch - 1), ix1 = min(ix + 1, cw - 1);
    const float ly = sy - iy, lx = sx - ix;
    const uint8_t* img = src + offs[n];
    const long r_a = ((long)(y0 + iy) * W) * 3, r_b = ((long)(y0 + iy1) * W) * 3;
    const long c_a = (long)(x0 + ix) * 3, c_b = (long)(x0 + ix1) * 3;
    float c[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float v00 = img[r_a + c_a + k], v01 = img[r_a + c_b + k];
      const float v10 = img[r_b + c_a + k], v11 = img[r_b + c_b + k];
      c[k] = (1.f - ly) * ((1.f - lx) * v00 + lx * v01) + ly * ((1.f - lx) * v10 + lx * v11);
    }
    (void)H;
    const int nops = (int)p[7];
    for (int o = 0; o < nops; ++o) {
      const int op = (int)p[8 + 2 * o];
      const float a = p[9 + 2 * o];
      if (op == 1) {
        c[0] = sat255(c[0] + a); c[1] = sat255(c[1] + a); c[2] = sat255(c[2] + a);
      } else if (op == 2) {
        c[0] = sat255(c[0] * a); c[1] = sat255(c[1] * a); c[2] = sat255(c[2] * a);
      } else if (op == 3 || op == 4) {
        float h, s, v;
        bgr2hsv(c[0], c[1], c[2], h, s, v);
        if (op == 3) s = fminf(fmaxf(s * a, 0.f), 255.f);
        else { h = h + a; h = h - 180.f * floorf(h / 180.f); }
        hsv2bgr(h, s, v, c[0], c[1], c[2]);
        c[0] = sat255(c[0]); c[1] = sat255(c[1]); c[2] = sat255(c[2]);
      }
    }
    const float o0 = ((rgb ? c[2] : c[0]) - m0) * i0, o1 = (c[1] - m1) * i1, o2 = ((rgb ? c[0] : c[2]) - m2) * i2;
    if (NHWC_BF16) {
      uint16_t* q = reinterpret_cast<uint16_t*>(out) + e * 3;
      q[0] = f2bf(o0); q[1] = f2bf(o1); q[2] = f2bf(o2);
    } else {
      float* q = reinterpret_cast<float*>(out);
      const long plane = (long)OH * OW;
      const long base = (long)n * 3 * plane + (long)oy * OW + ox;
      q[base] = o0; q[base + plane] = o1; q[base + 2 * plane] = o2;
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

extern "C" void bigdl_image_pipeline(const uint8_t* src, const long* offs, const float* prm, void* out, int N, int OH,
                                     int OW, const float* mean, const float* inv_std, int rgb, int nhwc_bf16,
                                     hipStream_t st) {
  const long total = (long)N * OH * OW;
  if (total == 0) return;
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  if (nhwc_bf16)
    image_pipeline_kernel<true><<<blocks, 256, 0, st>>>(src, offs, prm, out, N, OH, OW, mean[0], mean[1], mean[2],
                                                        inv_std[0], inv_std[1], inv_std[2], rgb);
  else
    image_pipeline_kernel<false><<<blocks, 256, 0, st>>>(src, offs, prm, out, N, OH, OW, mean[0], mean[1], mean[2],
                                                         inv_std[0], inv_std[1], inv_std[2], rgb);
  HIP_LAUNCH_CHECK();
}
