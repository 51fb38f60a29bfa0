"""Image augmentations on BGR mats (reference S/transform/vision/image/augmentation/*: Brightness, Contrast,
Saturation, Hue, ChannelNormalize, ChannelOrder, ChannelScaledNormalizer, ColorJitter, Crop (CenterCrop,
RandomCrop, FixedCrop, DetectionCrop), Expand, Filler, HFlip, PixelNormalizer, RandomAlterAspect,
RandomCropper, RandomResize, RandomTransformer, Resize, ScaleResize).

OpenCV semantics are reproduced on torch tensors: ``convertTo`` saturates to [0, 255]; HSV uses the 8-bit
convention (H in [0, 180), S and V in [0, 255]).
"""
import math

import torch
import torch.nn.functional as F

from ....utils.random_generator import RNG
from .feature import FeatureTransformer, ImageFeature

CropRandom, CropCenter = "CropRandom", "CropCenter"

INTER_NEAREST, INTER_LINEAR, INTER_CUBIC, INTER_AREA, INTER_LANCZOS4 = 0, 1, 2, 3, 4


def _sat(m):
    return m.clamp(0.0, 255.0)


def _resize(m, w, h, mode=INTER_LINEAR):
    x = m.permute(2, 0, 1).unsqueeze(0).float()
    if mode == INTER_NEAREST:
        y = F.interpolate(x, size=(h, w), mode="nearest")
    elif mode == INTER_AREA:
        y = F.interpolate(x, size=(h, w), mode="area")
    elif mode in (INTER_CUBIC, INTER_LANCZOS4):
        y = F.interpolate(x, size=(h, w), mode="bicubic", align_corners=False)
    else:
        y = F.interpolate(x, size=(h, w), mode="bilinear", align_corners=False)
    return y[0].permute(1, 2, 0).contiguous()


def bgr_to_hsv(m):
    """8-bit OpenCV convention: H in [0, 180), S, V in [0, 255]."""
    b, g, r = m[..., 0] / 255.0, m[..., 1] / 255.0, m[..., 2] / 255.0
    v, _ = torch.max(torch.stack([r, g, b]), 0)
    mn, _ = torch.min(torch.stack([r, g, b]), 0)
    d = v - mn
    s = torch.where(v > 0, d / v.clamp_min(1e-12), torch.zeros_like(v))
    h = torch.zeros_like(v)
    dz = d.clamp_min(1e-12)
    h = torch.where(v == r, 60.0 * (g - b) / dz, h)
    h = torch.where((v == g) & (v != r), 120.0 + 60.0 * (b - r) / dz, h)
    h = torch.where((v == b) & (v != r) & (v != g), 240.0 + 60.0 * (r - g) / dz, h)
    h = torch.where(d == 0, torch.zeros_like(h), h)
    h = torch.remainder(h, 360.0)
    return torch.stack([h / 2.0, s * 255.0, v * 255.0], -1)


def hsv_to_bgr(hsv):
    h = torch.remainder(hsv[..., 0] * 2.0, 360.0)
    s = (hsv[..., 1] / 255.0).clamp(0, 1)
    v = (hsv[..., 2] / 255.0).clamp(0, 1)
    c = v * s
    hp = h / 60.0
    x = c * (1 - torch.abs(torch.remainder(hp, 2.0) - 1))
    z = torch.zeros_like(h)
    i = hp.floor().clamp(0, 5).long()
    rs = torch.stack([c, x, z, z, x, c])
    gs = torch.stack([x, c, c, x, z, z])
    bs = torch.stack([z, z, x, c, c, x])
    idx = i.unsqueeze(0)
    r = torch.gather(rs, 0, idx)[0] + (v - c)
    g = torch.gather(gs, 0, idx)[0] + (v - c)
    b = torch.gather(bs, 0, idx)[0] + (v - c)
    return torch.stack([b, g, r], -1) * 255.0


# ---------------------------------------------------------------------------------------------- colour
class Brightness(FeatureTransformer):
    def __init__(self, deltaLow, deltaHigh):
        assert deltaLow <= deltaHigh
        self.lo, self.hi = deltaLow, deltaHigh

    @staticmethod
    def transform_mat(m, delta):
        return _sat(m + delta) if delta != 0 else m

    def transformMat(self, f):
        f[ImageFeature.mat] = self.transform_mat(f.opencvMat(), RNG.uniform(self.lo, self.hi))


class Contrast(FeatureTransformer):
    def __init__(self, deltaLow, deltaHigh):
        assert deltaHigh >= deltaLow >= 0
        self.lo, self.hi = deltaLow, deltaHigh

    @staticmethod
    def transform_mat(m, delta):
        return _sat(m * delta) if abs(delta - 1) > 1e-3 else m

    def transformMat(self, f):
        f[ImageFeature.mat] = self.transform_mat(f.opencvMat(), RNG.uniform(self.lo, self.hi))


class Saturation(FeatureTransformer):
    def __init__(self, deltaLow, deltaHigh):
        assert deltaHigh >= deltaLow >= 0
        self.lo, self.hi = deltaLow, deltaHigh

    @staticmethod
    def transform_mat(m, delta):
        hsv = bgr_to_hsv(m)
        hsv[..., 1] = (hsv[..., 1] * delta).clamp(0, 255)
        return _sat(hsv_to_bgr(hsv))

    def transformMat(self, f):
        f[ImageFeature.mat] = self.transform_mat(f.opencvMat(), RNG.uniform(self.lo, self.hi))


class Hue(FeatureTransformer):
    def __init__(self, deltaLow, deltaHigh):
        self.lo, self.hi = deltaLow, deltaHigh

    @staticmethod
    def transform_mat(m, delta):
        if delta == 0:
            return m
        hsv = bgr_to_hsv(m)
        hsv[..., 0] = torch.remainder(hsv[..., 0] + delta, 180.0)
        return _sat(hsv_to_bgr(hsv))

    def transformMat(self, f):
        f[ImageFeature.mat] = self.transform_mat(f.opencvMat(), RNG.uniform(self.lo, self.hi))


class ChannelOrder(FeatureTransformer):
    """Randomly permute the channels."""

    def transformMat(self, f):
        m = f.opencvMat()
        f[ImageFeature.mat] = m[..., torch.randperm(m.shape[2])].contiguous()


class ColorJitter(FeatureTransformer):
    """Random brightness / contrast / saturation / hue in the SSD order (ColorJitter.scala)."""

    def __init__(self, brightnessProb=0.5, brightnessDelta=32, contrastProb=0.5, contrastLower=0.5,
                 contrastUpper=1.5, hueProb=0.5, hueDelta=18, saturationProb=0.5, saturationLower=0.5,
                 saturationUpper=1.5, randomOrderProb=0, shuffle=False):
        self.bp, self.bd = brightnessProb, brightnessDelta
        self.cp, self.cl, self.cu = contrastProb, contrastLower, contrastUpper
        self.hp, self.hd = hueProb, hueDelta
        self.sp, self.sl, self.su = saturationProb, saturationLower, saturationUpper
        self.rp = randomOrderProb

    def transformMat(self, f):
        m = f.opencvMat()
        ops = []
        if RNG.uniform(0, 1) < self.bp:
            ops.append(lambda x: Brightness.transform_mat(x, RNG.uniform(-self.bd, self.bd)))
        if RNG.uniform(0, 1) < self.cp:
            ops.append(lambda x: Contrast.transform_mat(x, RNG.uniform(self.cl, self.cu)))
        if RNG.uniform(0, 1) < self.sp:
            ops.append(lambda x: Saturation.transform_mat(x, RNG.uniform(self.sl, self.su)))
        if RNG.uniform(0, 1) < self.hp:
            ops.append(lambda x: Hue.transform_mat(x, RNG.uniform(-self.hd, self.hd)))
        if RNG.uniform(0, 1) < self.rp:
            ops = [ops[i] for i in torch.randperm(len(ops)).tolist()]
        for op in ops:
            m = op(m)
        f[ImageFeature.mat] = m


# ---------------------------------------------------------------------------------------------- normalise
class ChannelNormalize(FeatureTransformer):
    """(x - mean) / std per channel; ``ChannelNormalize(meanR, meanG, meanB, stdR, stdG, stdB)``. As in the
    reference the means are stored in B, G, R order but the stds in R, G, B order (ChannelNormalize.scala:40)."""

    def __init__(self, meanR, meanG=None, meanB=None, stdR=1.0, stdG=1.0, stdB=1.0):
        if meanG is None:
            self.means, self.stds = [float(meanR)], [float(stdR)]
        else:
            self.means = [meanB, meanG, meanR]
            self.stds = [stdR, stdG, stdB]

    def transformMat(self, f):
        m = f.opencvMat().float()
        mean = torch.tensor(self.means, dtype=torch.float32, device=m.device)
        std = torch.tensor(self.stds, dtype=torch.float32, device=m.device)
        f[ImageFeature.mat] = (m - mean) / std


class ChannelScaledNormalizer(FeatureTransformer):
    def __init__(self, meanR, meanG, meanB, scale):
        self.mean = [meanR, meanG, meanB]
        self.scale = scale

    def transformMat(self, f):
        m = f.opencvMat().float()
        # reference indexes the float pixel buffer planar-by-channel with means (R, G, B) (ChannelScaledNormalizer.scala)
        planar = m.permute(2, 0, 1).reshape(3, -1)
        planar = (planar - torch.tensor(self.mean, dtype=torch.float32).view(3, 1)) * self.scale
        f[ImageFeature.mat] = planar.reshape(3, m.shape[0], m.shape[1]).permute(1, 2, 0).contiguous()


class PixelNormalizer(FeatureTransformer):
    def __init__(self, means):
        self.means = torch.as_tensor(means, dtype=torch.float32)

    def transformMat(self, f):
        m = f.opencvMat().float()
        assert self.means.numel() == m.numel(), "the means provided must have the same length as image"
        f[ImageFeature.mat] = m - self.means.reshape(m.shape)


# ---------------------------------------------------------------------------------------------- geometry
class Resize(FeatureTransformer):
    def __init__(self, resizeH, resizeW, resizeMode=INTER_LINEAR, useScaleFactor=True):
        self.h, self.w, self.mode = resizeH, resizeW, resizeMode

    @staticmethod
    def transform_mat(m, w, h, mode=INTER_LINEAR):
        return _resize(m, w, h, mode)

    def transformMat(self, f):
        mode = self.mode if self.mode != -1 else int(RNG.uniform(0, 5))
        f[ImageFeature.mat] = _resize(f.opencvMat(), self.w, self.h, mode)


def aspect_scale_hw(h, w, scaleTo, maxSize, scaleMultipleOf=1, minScale=None):
    """(height, width) after scaling the short side to ``scaleTo`` with the long side capped at ``maxSize`` and
    both sides floored to multiples of ``scaleMultipleOf`` (reference AspectScale.getHeightWidthAfterRatioScale,
    S/transform/vision/image/augmentation/Resize.scala:117-141; Java Math.round = floor(x + 0.5))."""
    lo, hi = min(h, w), max(h, w)
    s = float(scaleTo) / lo
    if minScale is not None:
        s = max(minScale, s)
    if math.floor(s * hi + 0.5) > maxSize:
        s = maxSize / float(hi)
    sh = sw = s
    if scaleMultipleOf > 1:
        sh = math.floor(h * s / scaleMultipleOf) * scaleMultipleOf / h
        sw = math.floor(w * s / scaleMultipleOf) * scaleMultipleOf / w
    return int(math.floor(sh * h + 0.5)), int(math.floor(sw * w + 0.5))


class AspectScale(FeatureTransformer):
    """Resize so the short side equals ``scale`` with the long side capped at ``maxSize``."""

    def __init__(self, scale, scaleMultipleOf=1, maxSize=1000, resizeMode=INTER_LINEAR, minScale=None):
        self.scale, self.mult, self.maxSize, self.mode = scale, scaleMultipleOf, maxSize, resizeMode
        self.minScale = minScale

    def transformMat(self, f):
        m = f.opencvMat()
        nh, nw = aspect_scale_hw(m.shape[0], m.shape[1], self.scale, self.maxSize, self.mult, self.minScale)
        f[ImageFeature.mat] = _resize(m, nw, nh, self.mode)


class RandomAspectScale(FeatureTransformer):
    """AspectScale to a scale drawn uniformly from ``scales`` (reference Resize.scala:151-160)."""

    def __init__(self, scales, scaleMultipleOf=1, maxSize=1000):
        self.scales, self.mult, self.maxSize = list(scales), scaleMultipleOf, maxSize

    def transformMat(self, f):
        m = f.opencvMat()
        scale = self.scales[min(int(RNG.uniform(0, len(self.scales))), len(self.scales) - 1)]
        nh, nw = aspect_scale_hw(m.shape[0], m.shape[1], scale, self.maxSize, self.mult)
        f[ImageFeature.mat] = _resize(m, nw, nh)


class RandomResize(FeatureTransformer):
    def __init__(self, minSize, maxSize):
        self.minSize, self.maxSize = minSize, maxSize

    def transformMat(self, f):
        m = f.opencvMat()
        h, w = m.shape[:2]
        short = int(RNG.uniform(1e-2, self.maxSize - self.minSize + 1)) + self.minSize
        if h < w:
            w, h = int(w / h * short), short
        else:
            h, w = int(h / w * short), short
        f[ImageFeature.mat] = _resize(m, w, h, INTER_CUBIC)


class ScaleResize(FeatureTransformer):
    def __init__(self, minSize, maxSize=-1, resizeROI=False):
        self.minSize, self.maxSize, self.resizeROI = minSize, maxSize, resizeROI

    def _size(self, h, w):
        size = self.minSize
        if self.maxSize > 0:
            mn, mx = min(h, w), max(h, w)
            if mx / mn * size > self.maxSize:
                size = int(round(self.maxSize * mn / mx))
        if (w <= h and w == size) or (h <= w and h == size):
            return h, w
        if w < h:
            return size * h // w, size
        return size, size * w // h

    def transformMat(self, f):
        m = f.opencvMat()
        h, w = m.shape[:2]
        nh, nw = self._size(h, w)
        f[ImageFeature.mat] = _resize(m, nw, nh, INTER_LINEAR)
        if self.resizeROI and f.get(ImageFeature.label) is not None and hasattr(f[ImageFeature.label], "bboxes"):
            lab = f[ImageFeature.label]
            lab.bboxes = lab.bboxes * torch.tensor([nw / w, nh / h, nw / w, nh / h])


class HFlip(FeatureTransformer):
    def transformMat(self, f):
        f[ImageFeature.mat] = f.opencvMat().flip(1).contiguous()


class Crop(FeatureTransformer):
    """Crop to a box (x1, y1, x2, y2), normalized to [0, 1] or in pixels; ``isClip`` clips to the image."""

    def __init__(self, normalized=True, isClip=True):
        self.normalized, self.isClip = normalized, isClip

    def box(self, f):
        raise NotImplementedError

    def transformMat(self, f):
        m = f.opencvMat()
        h, w = m.shape[:2]
        x1, y1, x2, y2 = self._last_box = self.box(f)
        if self.normalized:
            x1, x2, y1, y2 = x1 * w, x2 * w, y1 * h, y2 * h
        if self.isClip:
            x1, x2 = max(0.0, min(x1, w)), max(0.0, min(x2, w))
            y1, y2 = max(0.0, min(y1, h)), max(0.0, min(y2, h))
        # OpenCV Rect(x1, y1, width, height) with truncated float coordinates (Crop.scala transform)
        rx, ry, rw, rh = int(x1), int(y1), int(x2 - x1), int(y2 - y1)
        f[ImageFeature.mat] = m[ry:ry + rh, rx:rx + rw].contiguous()
        if f.get(ImageFeature.label) is not None:      # the crop box, for RoiProject (Crop.scala:35-37)
            from .roi import BoundingBox

            f[ImageFeature.boundingBox] = BoundingBox(*self._last_box, normalized=self.normalized)


class CenterCrop(Crop):
    def __init__(self, cropWidth, cropHeight, isClip=True):
        super().__init__(False, isClip)
        self.cw, self.ch = cropWidth, cropHeight

    def box(self, f):
        h, w = f.getHeight(), f.getWidth()
        x1, y1 = (w - self.cw) / 2.0, (h - self.ch) / 2.0
        return x1, y1, x1 + self.cw, y1 + self.ch


class RandomCrop(Crop):
    def __init__(self, cropWidth, cropHeight, isClip=True):
        super().__init__(False, isClip)
        self.cw, self.ch = cropWidth, cropHeight

    def box(self, f):
        h, w = f.getHeight(), f.getWidth()
        x1 = math.floor(RNG.uniform(0, w - self.cw))
        y1 = math.floor(RNG.uniform(0, h - self.ch))
        return x1, y1, x1 + self.cw, y1 + self.ch


class FixedCrop(Crop):
    def __init__(self, x1, y1, x2, y2, normalized, isClip=True):
        super().__init__(normalized, isClip)
        self.b = (x1, y1, x2, y2)

    def box(self, f):
        return self.b


class DetectionCrop(Crop):
    def __init__(self, roiKey, normalized=True):
        super().__init__(normalized, True)
        self.roiKey = roiKey

    def box(self, f):
        return tuple(float(v) for v in torch.as_tensor(f[self.roiKey]).reshape(-1)[:4])


class RandomCropper(FeatureTransformer):
    def __init__(self, cropWidth, cropHeight, mirror, cropperMethod=CropRandom, channels=3):
        self.cw, self.ch, self.mirror, self.method = cropWidth, cropHeight, mirror, cropperMethod

    def transformMat(self, f):
        m = f.opencvMat().float()
        h, w = m.shape[:2]
        if self.method == CropRandom:
            sh = int(math.ceil(RNG.uniform(0, h - self.ch)))
            sw = int(math.ceil(RNG.uniform(0, w - self.cw)))
        else:
            sh, sw = (h - self.ch) // 2, (w - self.cw) // 2
        out = m[sh:sh + self.ch, sw:sw + self.cw]
        if self.mirror and int(RNG.uniform(0, 2)) != 0:
            out = out.flip(1)
        f[ImageFeature.mat] = out.contiguous()


class RandomAlterAspect(FeatureTransformer):
    """Inception-style random area / aspect crop resized to ``cropLength`` (RandomAlterAspect.scala)."""

    def __init__(self, min_area_ratio=0.08, max_area_ratio=1, min_aspect_ratio_change=0.75, interp_mode="CUBIC",
                 cropLength=224):
        self.amin, self.amax, self.asp = min_area_ratio, max_area_ratio, min_aspect_ratio_change
        self.mode = {"CUBIC": INTER_CUBIC, "LINEAR": INTER_LINEAR, "NEAREST": INTER_NEAREST,
                     "AREA": INTER_AREA}.get(interp_mode, INTER_CUBIC)
        self.L = cropLength

    @staticmethod
    def _ratio(lo, hi):
        return (RNG.uniform(1e-2, (hi - lo) * 1000 + 1) + lo * 1000) / 1000

    def transformMat(self, f):
        m = f.opencvMat()
        h, w = m.shape[:2]
        area = h * w
        for _ in range(10):
            ar = self._ratio(self.amin, self.amax)
            ch = self._ratio(self.asp, 1 / self.asp)
            na = ar * area
            nh, nw = int(math.sqrt(na) * ch), int(math.sqrt(na) / ch)
            if self._ratio(0, 1) < 0.5:
                nh, nw = nw, nh
            if nh <= h and nw <= w:
                y = int(RNG.uniform(1e-2, h - nh + 1))
                x = int(RNG.uniform(1e-2, w - nw + 1))
                f[ImageFeature.mat] = _resize(m[y:y + nh, x:x + nw], self.L, self.L, self.mode)
                return
        # fallback: center crop of the short side
        s = min(h, w)
        y, x = (h - s) // 2, (w - s) // 2
        f[ImageFeature.mat] = _resize(m[y:y + s, x:x + s], self.L, self.L, self.mode)


class FixExpand(FeatureTransformer):
    """Place the image in the centre of a zero ``expandHeight`` x ``expandWidth`` canvas and record the placed box
    (reference Expand.scala:102-129)."""

    def __init__(self, expandHeight, expandWidth):
        self.eh, self.ew = expandHeight, expandWidth

    def transformMat(self, f):
        from .roi import BoundingBox

        m = f.opencvMat()
        h, w = m.shape[:2]
        assert w <= self.ew and h <= self.eh, f"image {h}x{w} larger than the {self.eh}x{self.ew} canvas"
        top, left = (self.eh - h) // 2, (self.ew - w) // 2
        out = torch.zeros((self.eh, self.ew) + tuple(m.shape[2:]), dtype=m.dtype, device=m.device)
        out[top:top + h, left:left + w] = m
        f[ImageFeature.mat] = out
        f[ImageFeature.boundingBox] = BoundingBox(float(left), float(top), float(left + w), float(top + h))


class PixelNormalize(PixelNormalizer):
    """Reference name (P/transform/vision/image.py PixelNormalize) of PixelNormalizer: data(i) - mean(i)."""


class Pipeline(FeatureTransformer):
    """A list of FeatureTransformers applied in order (reference image.py Pipeline)."""

    def __init__(self, transformers):
        assert all(isinstance(t, FeatureTransformer) for t in transformers), "Pipeline takes FeatureTransformers"
        self.transformers = list(transformers)

    def transform(self, f):
        for t in self.transformers:
            f = t.transform(f)
        return f


class Expand(FeatureTransformer):
    """Place the image on a mean-filled canvas up to ``maxExpandRatio`` times larger (SSD zoom-out)."""

    def __init__(self, meansR=123, meansG=117, meansB=104, minExpandRatio=1.0, maxExpandRatio=4.0):
        self.means = (meansB, meansG, meansR)
        self.lo, self.hi = minExpandRatio, maxExpandRatio

    def transformMat(self, f):
        if abs(self.hi - 1) < 1e-2:
            return
        m = f.opencvMat()
        h, w, c = m.shape
        r = RNG.uniform(self.lo, self.hi)
        H, W = int(h * r), int(w * r)
        ho = math.floor(RNG.uniform(0, H - h))
        wo = math.floor(RNG.uniform(0, W - w))
        canvas = torch.empty(H, W, c, dtype=m.dtype, device=m.device)
        canvas[:] = torch.tensor(self.means[:c], dtype=m.dtype)
        canvas[ho:ho + h, wo:wo + w] = m
        f[ImageFeature.mat] = canvas
        f["expandBbox"] = torch.tensor([-wo / w, -ho / h, (W - wo) / w, (H - ho) / h])


class Filler(FeatureTransformer):
    def __init__(self, startX, startY, endX, endY, value=255):
        assert 0 <= startX < endX <= 1 and 0 <= startY < endY <= 1
        self.b = (startX, startY, endX, endY)
        self.value = value

    def transformMat(self, f):
        m = f.opencvMat().clone()
        h, w = m.shape[:2]
        x1, y1 = math.ceil(self.b[0] * w), math.ceil(self.b[1] * h)
        x2, y2 = math.ceil(self.b[2] * w), math.ceil(self.b[3] * h)
        m[y1:y2, x1:x2] = float(self.value)
        f[ImageFeature.mat] = m


class RandomTransformer(FeatureTransformer):
    """Apply ``transformer`` with probability ``maxProb``."""

    def __init__(self, transformer, maxProb):
        self.t, self.p = transformer, maxProb

    def transform(self, f):
        if RNG.uniform(0, 1) < self.p:
            return self.t.transform(f)
        return f
