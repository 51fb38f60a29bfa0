// Detection kernels for gfx950: greedy NMS (64-bit IoU masks + single-wave scan), RoiAlign forward,
// RoiPooling forward/backward.
//
// Reference semantics: S/nn/Nms.scala:50-236 (greedy NMS over score-sorted boxes, "IoU > thresh" suppresses,
// pixel areas (x2-x1+1)(y2-y1+1) unless normalized), S/nn/RoiAlign.scala:45-420 (bilinear sampling grid,
// out-of-map samples contribute 0 but are counted, average over the grid), S/nn/RoiPooling.scala:42-366
// (Fast R-CNN max pooling over rounded, scaled rois, argmax kept for backward).
//
// NMS mapping: a wave is 64 lanes and a suppression row is a 64-bit word, so block (i, j) of the IoU matrix
// is one wave: lane l tests box j*64+l against box i*64+r for each r and __ballot turns the 64 predicates
// into one word. The greedy pass is then one wave walking the boxes in score order with the "removed" bitset
// held in registers (lane l owns words l, l+64, ...): no barrier, no atomics, and the result never leaves
// the device.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int NMS_MAX_WORDS_PER_LANE = 4;   // up to 64 * 64 * 4 = 16384 boxes

__device__ __forceinline__ bool iou_gt(const float* a, const float* b, float area_a, float area_b, float thresh,
                                       float one) {
  const float w = fminf(a[2], b[2]) - fmaxf(a[0], b[0]) + one;
  if (w < 0.f) return false;
  const float h = fminf(a[3], b[3]) - fmaxf(a[1], b[1]) + one;
  if (h < 0.f) return false;
  const float inter = w * h;
  return inter / (area_a + area_b - inter) > thresh;
}

// boxes: [n][4] sorted by descending score. mask: [n][words] uint64, bit l of word j in row i set when box
// j*64+l (j*64+l > i) overlaps box i above thresh.
__global__ void __launch_bounds__(64) nms_mask_kernel(const float* __restrict__ boxes, int n, float thresh,
                                                      int normalized, unsigned long long* __restrict__ mask,
                                                      int words) {
  const int jb = blockIdx.x, ib = blockIdx.y, lane = threadIdx.x;
  const float one = normalized ? 0.f : 1.f;
  __shared__ float col[64][4];
  __shared__ float col_area[64];
  const int j = jb * 64 + lane;
  if (j < n) {
    const float4 b = *reinterpret_cast<const float4*>(boxes + 4 * (size_t)j);
    col[lane][0] = b.x; col[lane][1] = b.y; col[lane][2] = b.z; col[lane][3] = b.w;
    col_area[lane] = (b.z - b.x + one) * (b.w - b.y + one);
  }
  __syncthreads();
  const int rows = min(64, n - ib * 64);
  for (int r = 0; r < rows; ++r) {
    const int i = ib * 64 + r;
    const float4 bi = *reinterpret_cast<const float4*>(boxes + 4 * (size_t)i);   // wave-uniform load
    const float a[4] = {bi.x, bi.y, bi.z, bi.w};
    const float area_i = (bi.z - bi.x + one) * (bi.w - bi.y + one);
    const bool p = (j < n) && (j > i) && iou_gt(a, col[lane], area_i, col_area[lane], thresh, one);
    const unsigned long long word = __ballot(p);
    if (lane == 0) mask[(size_t)i * words + jb] = word;
  }
}

// Single wave: greedy scan in sorted order. keep_out[k] = sorted position of the k-th kept box; count_out[0] = k.
__global__ void __launch_bounds__(64) nms_scan_kernel(const unsigned long long* __restrict__ mask, int n, int words,
                                                      int max_keep, int* __restrict__ keep_out,
                                                      int* __restrict__ count_out) {
  const int lane = threadIdx.x;
  unsigned long long removed[NMS_MAX_WORDS_PER_LANE];
#pragma unroll
  for (int k = 0; k < NMS_MAX_WORDS_PER_LANE; ++k) removed[k] = 0ull;
  int kept = 0;
  for (int i = 0; i < n; ++i) {
    const int w = i >> 6, owner = w & 63, slot = w >> 6;
    unsigned long long mine = 0ull;
#pragma unroll
    for (int k = 0; k < NMS_MAX_WORDS_PER_LANE; ++k)
      if (k == slot) mine = removed[k];
    const unsigned long long ow = __shfl(mine, owner, 64);
    if ((ow >> (i & 63)) & 1ull) continue;          // wave-uniform branch
    if (lane == 0) keep_out[kept] = i;
    ++kept;
    if (max_keep > 0 && kept >= max_keep) break;
    const unsigned long long* row = mask + (size_t)i * words;
#pragma unroll
    for (int k = 0; k < NMS_MAX_WORDS_PER_LANE; ++k) {
      const int wd = lane + 64 * k;
      if (wd < words) removed[k] |= row[wd];
    }
  }
  if (lane == 0) count_out[0] = kept;
}

// ---------------------------------------------------------------------------------------------- RoiAlign
// x: [N][C][H][W] fp32; rois: [R][rcols] (rcols 4: batch 0, (x1,y1,x2,y2); rcols 5: (b, x1, y1, x2, y2)).
// One thread per output element (r, c, ph, pw): the sampling grid of one bin is at most a few dozen taps.
__global__ void __launch_bounds__(256) roi_align_fwd_kernel(const float* __restrict__ x, const float* __restrict__ rois,
                                                            float* __restrict__ out, int R, int rcols, int C, int H,
                                                            int W, int PH, int PW, float scale, int sampling) {
  const long total = (long)R * C * PH * PW;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int pw = (int)(idx % PW);
    const int ph = (int)((idx / PW) % PH);
    const int c = (int)((idx / ((long)PW * PH)) % C);
    const int r = (int)(idx / ((long)PW * PH * C));
    const float* roi = rois + (size_t)r * rcols;
    const int b = rcols == 5 ? (int)roi[0] : 0;
    const float* rb = roi + (rcols == 5 ? 1 : 0);
    const float sw = rb[0] * scale, sh = rb[1] * scale, ew = rb[2] * scale, eh = rb[3] * scale;
    const float rw = fmaxf(ew - sw, 1.f), rh = fmaxf(eh - sh, 1.f);
    const float bh = rh / PH, bw = rw / PW;
    const int gh = sampling > 0 ? sampling : (int)ceilf(rh / PH);
    const int gw = sampling > 0 ? sampling : (int)ceilf(rw / PW);
    const float* xc = x + ((size_t)b * C + c) * (size_t)H * W;
    float acc = 0.f;
    for (int iy = 0; iy < gh; ++iy) {
      const float yy = sh + ph * bh + (iy + 0.5f) * bh / gh;
      for (int ix = 0; ix < gw; ++ix) {
        const float xx = sw + pw * bw + (ix + 0.5f) * bw / gw;
        if (yy < -1.f || yy > (float)H || xx < -1.f || xx > (float)W) continue;
        float y = fmaxf(yy, 0.f), xv = fmaxf(xx, 0.f);
        int yl = (int)y, xl = (int)xv, yh, xh;
        if (yl >= H - 1) { yl = yh = H - 1; y = (float)yl; } else { yh = yl + 1; }
        if (xl >= W - 1) { xl = xh = W - 1; xv = (float)xl; } else { xh = xl + 1; }
        const float ly = y - yl, lx = xv - xl, hy = 1.f - ly, hx = 1.f - lx;
        acc += hy * hx * xc[yl * W + xl] + hy * lx * xc[yl * W + xh] + ly * hx * xc[yh * W + xl] +
               ly * lx * xc[yh * W + xh];
      }
    }
    out[idx] = acc / (float)(gh * gw);
  }
}

// --------------------------------------------------------------------------------------------- RoiPooling
__global__ void __launch_bounds__(256) roi_pool_fwd_kernel(const float* __restrict__ x, const float* __restrict__ rois,
                                                           float* __restrict__ out, int* __restrict__ argmax, int R,
                                                           int C, int H, int W, int PH, int PW, float scale) {
  const long total = (long)R * C * PH * PW;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int pw = (int)(idx % PW);
    const int ph = (int)((idx / PW) % PH);
    const int c = (int)((idx / ((long)PW * PH)) % C);
    const int r = (int)(idx / ((long)PW * PH * C));
    const float* roi = rois + (size_t)r * 5;
    const int b = (int)roi[0];
    const int sw = (int)floorf(roi[1] * scale + 0.5f), sh = (int)floorf(roi[2] * scale + 0.5f);
    const int ew = (int)floorf(roi[3] * scale + 0.5f), eh = (int)floorf(roi[4] * scale + 0.5f);
    const float bh = fmaxf((float)(eh - sh + 1), 1.f) / PH, bw = fmaxf((float)(ew - sw + 1), 1.f) / PW;
    int hs = (int)floorf(ph * bh) + sh, he = (int)ceilf((ph + 1) * bh) + sh;
    int ws = (int)floorf(pw * bw) + sw, we = (int)ceilf((pw + 1) * bw) + sw;
    hs = min(max(hs, 0), H); he = min(max(he, 0), H);
    ws = min(max(ws, 0), W); we = min(max(we, 0), W);
    const float* xc = x + ((size_t)b * C + c) * (size_t)H * W;
    float best = (he <= hs || we <= ws) ? 0.f : -3.402823466e38f;
    int arg = -1;
    for (int h = hs; h < he; ++h)
      for (int w = ws; w < we; ++w) {
        const float v = xc[h * W + w];
        if (v > best) { best = v; arg = h * W + w; }
      }
    out[idx] = best;
    argmax[idx] = arg;
  }
}

__global__ void __launch_bounds__(256) roi_pool_bwd_kernel(const float* __restrict__ gy, const int* __restrict__ argmax,
                                                           const float* __restrict__ rois, float* __restrict__ gx,
                                                           int R, int C, int H, int W, int PH, int PW) {
  const long total = (long)R * C * PH * PW;
  for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total; idx += (long)gridDim.x * blockDim.x) {
    const int a = argmax[idx];
    if (a < 0) continue;
    const int c = (int)((idx / ((long)PW * PH)) % C);
    const int r = (int)(idx / ((long)PW * PH * C));
    const int b = (int)rois[(size_t)r * 5];
    atomicAdd(gx + ((size_t)b * C + c) * (size_t)H * W + a, gy[idx]);
  }
}

int grid_for(long total) { return (int)std::min<long>((total + 255) / 256, 65536); }

}  // namespace

extern "C" {

int bigdl_nms(const float* boxes_sorted, int n, float thresh, int normalized, int max_keep,
              unsigned long long* mask_ws, int* keep_out, int* count_out, hipStream_t st) {
  const int words = (n + 63) / 64;
  if (n <= 0) return bigdl_fill_bytes(count_out, 0, (long)sizeof(int), st), 0;
  if (words > 64 * NMS_MAX_WORDS_PER_LANE) return -1;
  nms_mask_kernel<<<dim3(words, words), 64, 0, st>>>(boxes_sorted, n, thresh, normalized, mask_ws, words);
  nms_scan_kernel<<<1, 64, 0, st>>>(mask_ws, n, words, max_keep, keep_out, count_out);
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_roi_align_fwd(const float* x, const float* rois, float* out, int R, int rcols, int C, int H, int W,
                        int PH, int PW, float scale, int sampling, hipStream_t st) {
  const long total = (long)R * C * PH * PW;
  if (total <= 0) return 0;
  roi_align_fwd_kernel<<<grid_for(total), 256, 0, st>>>(x, rois, out, R, rcols, C, H, W, PH, PW, scale, sampling);
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_roi_pool_fwd(const float* x, const float* rois, float* out, int* argmax, int R, int C, int H, int W,
                       int PH, int PW, float scale, hipStream_t st) {
  const long total = (long)R * C * PH * PW;
  if (total <= 0) return 0;
  roi_pool_fwd_kernel<<<grid_for(total), 256, 0, st>>>(x, rois, out, argmax, R, C, H, W, PH, PW, scale);
  HIP_LAUNCH_CHECK();
  return 0;
}

int bigdl_roi_pool_bwd(const float* gy, const int* argmax, const float* rois, float* gx, int R, int C, int H, int W,
                       int PH, int PW, hipStream_t st) {
  const long total = (long)R * C * PH * PW;
  if (total <= 0) return 0;
  roi_pool_bwd_kernel<<<grid_for(total), 256, 0, st>>>(gy, argmax, rois, gx, R, C, H, W, PH, PW);
  HIP_LAUNCH_CHECK();
  return 0;
}

}  // extern "C"
