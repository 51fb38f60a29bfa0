"""Detection labels and their geometric transforms.

Reference: S/transform/vision/image/label/roi/RoiLabel.scala (classes [2, n] = (label, difficult) or [n],
bboxes [n, 4] x1 y1 x2 y2, optional masks; ``fromTensor``), RoiTransformer.scala (RoiNormalize, RoiHFlip,
RoiResize, RoiProject with the SSD emit-center constraint), BatchSampler.scala / RandomSampler.scala (SSD
crop sampling: random scale / aspect ratio boxes accepted by Jaccard-overlap constraints with the ground truth,
then crop + project), util/BoundingBox.scala (jaccard overlap, meetEmitCenterConstraint, projectBbox).
"""
import math
import random

import torch

from .augmentation import Crop
from .feature import FeatureTransformer, ImageFeature


class RoiLabel:
    CLASSES, BBOXES, MASKS, ISCROWD, ORIGSIZE, SCORES = "classes", "bboxes", "masks", "is_crowd", "size", "scores"

    def __init__(self, classes, bboxes, masks=None):
        self.classes = torch.as_tensor(classes, dtype=torch.float32)
        self.bboxes = torch.as_tensor(bboxes, dtype=torch.float32).reshape(-1, 4)
        self.masks = masks
        n = self.bboxes.shape[0]
        if self.classes.dim() == 1:
            assert self.classes.numel() == n, "number of classes must equal number of boxes"
        elif self.classes.numel() > 0:
            assert self.classes.shape[1] == n, "number of classes must equal number of boxes"

    def size(self):
        return 0 if self.bboxes.numel() < 4 else self.bboxes.shape[0]

    def copy(self, other):
        self.classes = other.classes.clone()
        self.bboxes = other.bboxes.clone()
        return self

    def toTable(self):
        from ...utils.table import Table

        t = Table()
        t[RoiLabel.CLASSES] = self.classes
        t[RoiLabel.BBOXES] = self.bboxes
        if self.masks is not None:
            t[RoiLabel.MASKS] = self.masks
        return t

    @staticmethod
    def fromTensor(t):
        """[n, 6] rows (label, difficult, x1, y1, x2, y2) -> RoiLabel."""
        return RoiLabel(t[:, 0:2].t().contiguous(), t[:, 2:6].contiguous())

    def _label_cols(self):
        if self.classes.dim() == 1:
            return self.classes, torch.zeros_like(self.classes)
        return self.classes[0], self.classes[1]


class BoundingBox:
    def __init__(self, x1=0.0, y1=0.0, x2=1.0, y2=1.0, normalized=True):
        self.x1, self.y1, self.x2, self.y2, self.normalized = float(x1), float(y1), float(x2), float(y2), normalized
        self.label, self.difficult = -1.0, 0.0

    def width(self):
        return self.x2 - self.x1

    def height(self):
        return self.y2 - self.y1

    def area(self):
        if self.x2 < self.x1 or self.y2 < self.y1:
            return 0.0
        w, h = self.width(), self.height()
        return w * h if self.normalized else (w + 1) * (h + 1)

    def jaccardOverlap(self, o):
        ix1, iy1 = max(self.x1, o.x1), max(self.y1, o.y1)
        ix2, iy2 = min(self.x2, o.x2), min(self.y2, o.y2)
        if ix2 < ix1 or iy2 < iy1:
            return 0.0
        inter = BoundingBox(ix1, iy1, ix2, iy2, self.normalized).area()
        return inter / (self.area() + o.area() - inter)

    def meetEmitCenterConstraint(self, gt):
        cx, cy = (gt.x1 + gt.x2) / 2, (gt.y1 + gt.y2) / 2
        return self.x1 <= cx <= self.x2 and self.y1 <= cy <= self.y2

    def projectBbox(self, src, dst):
        """Project ``src`` into this box's frame (normalized), clipped; False when they do not overlap."""
        if src.x1 >= self.x2 or src.x2 <= self.x1 or src.y1 >= self.y2 or src.y2 <= self.y1:
            return False
        w, h = self.width(), self.height()
        dst.x1 = min(max((src.x1 - self.x1) / w, 0.0), 1.0)
        dst.y1 = min(max((src.y1 - self.y1) / h, 0.0), 1.0)
        dst.x2 = min(max((src.x2 - self.x1) / w, 0.0), 1.0)
        dst.y2 = min(max((src.y2 - self.y1) / h, 0.0), 1.0)
        dst.normalized = True
        return dst.area() > 0

    def scaleBox(self, sh, sw, dst=None):
        dst = dst if dst is not None else self
        dst.x1, dst.y1, dst.x2, dst.y2 = self.x1 * sw, self.y1 * sh, self.x2 * sw, self.y2 * sh
        return dst

    def __repr__(self):
        return f"BoundingBox({self.x1:.4f}, {self.y1:.4f}, {self.x2:.4f}, {self.y2:.4f})"


def _scale_bboxes(b, sh, sw):
    b[:, 0::2] *= sw
    b[:, 1::2] *= sh


class RoiNormalize(FeatureTransformer):
    """Pixel boxes -> [0, 1] by the image size."""

    def transformMat(self, f):
        _scale_bboxes(f[ImageFeature.label].bboxes, 1.0 / f.getHeight(), 1.0 / f.getWidth())


class RoiHFlip(FeatureTransformer):
    def __init__(self, normalized=True):
        self.normalized = normalized

    def transformMat(self, f):
        b = f[ImageFeature.label].bboxes
        w = 1.0 if self.normalized else float(f.getWidth())
        x1 = w - b[:, 0].clone()
        b[:, 0] = w - b[:, 2]
        b[:, 2] = x1


class RoiResize(FeatureTransformer):
    """Pixel boxes follow an image resize (no-op for normalized boxes)."""

    def __init__(self, normalized=False):
        self.normalized = normalized

    def transformMat(self, f):
        if not self.normalized:
            sw = f.getWidth() / float(f.getOriginalWidth())
            sh = f.getHeight() / float(f.getOriginalHeight())
            _scale_bboxes(f[ImageFeature.label].bboxes, sh, sw)


class RoiProject(FeatureTransformer):
    """Re-express the ground truth in the frame of the crop stored at ``ImageFeature.boundingBox``; boxes
    whose center falls outside the crop are dropped (``needMeetCenterConstraint``)."""

    def __init__(self, needMeetCenterConstraint=True):
        self.needMeetCenterConstraint = needMeetCenterConstraint

    def transformMat(self, f):
        crop = f[ImageFeature.boundingBox]
        if not crop.normalized:
            crop.scaleBox(1.0 / f.getHeight(), 1.0 / f.getWidth())
            crop.normalized = True
        target = f[ImageFeature.label]
        labels, difficult = target._label_cols()
        keep_b, keep_l, keep_d = [], [], []
        for i in range(target.size()):
            gt = BoundingBox(*target.bboxes[i].tolist())
            if self.needMeetCenterConstraint and not crop.meetEmitCenterConstraint(gt):
                continue
            dst = BoundingBox()
            if crop.projectBbox(gt, dst):
                keep_b.append([dst.x1, dst.y1, dst.x2, dst.y2])
                keep_l.append(float(labels[i]))
                keep_d.append(float(difficult[i]))
        target.bboxes = torch.tensor(keep_b, dtype=torch.float32).reshape(-1, 4)
        target.classes = torch.tensor([keep_l, keep_d], dtype=torch.float32).reshape(2, -1)


class BatchSampler:
    """One SSD sampling rule: up to ``maxSample`` boxes from ``maxTrials`` draws of scale in
    [minScale, maxScale] and aspect ratio in [minAspectRatio, maxAspectRatio], accepted when the Jaccard
    overlap with some ground-truth box lies in [minOverlap, maxOverlap]."""

    def __init__(self, maxSample=1, maxTrials=50, minScale=1.0, maxScale=1.0, minAspectRatio=1.0,
                 maxAspectRatio=1.0, minOverlap=None, maxOverlap=None):
        self.maxSample, self.maxTrials = maxSample, maxTrials
        self.minScale, self.maxScale = minScale, maxScale
        self.minAspectRatio, self.maxAspectRatio = minAspectRatio, maxAspectRatio
        self.minOverlap, self.maxOverlap = minOverlap, maxOverlap

    def _sample_box(self, rng):
        scale = rng.uniform(self.minScale, self.maxScale)
        ar = rng.uniform(max(self.minAspectRatio, scale * scale), min(self.maxAspectRatio, 1.0 / (scale * scale)))
        w, h = scale * math.sqrt(ar), scale / math.sqrt(ar)
        x1, y1 = rng.uniform(0, 1 - w), rng.uniform(0, 1 - h)
        return BoundingBox(x1, y1, x1 + w, y1 + h)

    def _satisfy(self, box, gts):
        if self.minOverlap is None and self.maxOverlap is None:
            return True
        for gt in gts:
            o = box.jaccardOverlap(gt)
            if self.minOverlap is not None and o < self.minOverlap:
                continue
            if self.maxOverlap is not None and o > self.maxOverlap:
                continue
            return True
        return False

    def sample(self, gts, out, rng=random):
        found = 0
        for _ in range(self.maxTrials):
            if found >= self.maxSample:
                break
            box = self._sample_box(rng)
            if self._satisfy(box, gts):
                found += 1
                out.append(box)
        return out


def default_ssd_samplers():
    """The standard SSD sampler set (the reference RandomSampler's defaults)."""
    s = [BatchSampler(maxTrials=1)]
    for ov in (0.1, 0.3, 0.5, 0.7, 0.9):
        s.append(BatchSampler(1, 50, 0.3, 1.0, 0.5, 2.0, minOverlap=ov))
    s.append(BatchSampler(1, 50, 0.3, 1.0, 0.5, 2.0, maxOverlap=1.0))
    return s


class _SampledCrop(Crop):
    def box(self, f):
        b = f[ImageFeature.boundingBox]
        return b.x1, b.y1, b.x2, b.y2


class RandomSampler(FeatureTransformer):
    """Pick one of the boxes the samplers produce, crop the image to it and project the ground truth."""

    def __init__(self, samplers=None, seed=None):
        self.samplers = samplers or default_ssd_samplers()
        self.rng = random.Random(seed)
        self.crop = _SampledCrop(normalized=True, isClip=True)
        self.project = RoiProject(True)

    def transformMat(self, f):
        target = f[ImageFeature.label]
        gts = [BoundingBox(*target.bboxes[i].tolist()) for i in range(target.size())]
        boxes = []
        for s in self.samplers:
            s.sample(gts, boxes, self.rng)
        if not boxes:
            return
        box = boxes[self.rng.randrange(len(boxes))]
        f[ImageFeature.boundingBox] = box
        self.crop.transformMat(f)
        self.project.transformMat(f)


__all__ = ["RoiLabel", "BoundingBox", "RoiNormalize", "RoiHFlip", "RoiResize", "RoiProject", "BatchSampler",
           "RandomSampler", "default_ssd_samplers"]
