"""Detection label transforms against the reference RoiTransformerSpec fixtures (pascal image 500 x 375)."""
import torch

from bigdl_amd.transform.vision.image.augmentation import CenterCrop
from bigdl_amd.transform.vision.image.feature import ImageFeature
from bigdl_amd.transform.vision.image.roi import (BatchSampler, BoundingBox, RandomSampler, RoiHFlip, RoiLabel,
                                                  RoiNormalize, RoiProject)

BOXES = [2.0, 84.0, 59.0, 248.0, 68.0, 115.0, 233.0, 279.0, 64.0, 173.0, 377.0, 373.0, 320.0, 2.0, 496.0, 375.0,
         221.0, 4.0, 341.0, 374.0, 135.0, 14.0, 220.0, 148.0, 69.0, 43.0, 156.0, 177.0, 58.0, 54.0, 104.0, 139.0,
         279.0, 1.0, 331.0, 86.0, 320.0, 22.0, 344.0, 96.0, 337.0, 1.0, 390.0, 107.0]
CLASSES = [11.0, 11.0, 11.0, 16.0, 16.0, 16.0, 11.0, 16.0, 16.0, 16.0, 16.0,
           0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0]


def _feature():
    f = ImageFeature()
    f[ImageFeature.mat] = torch.zeros(375, 500, 3)
    f[ImageFeature.originalSize] = (375, 500, 3)
    f[ImageFeature.label] = RoiLabel(torch.tensor(CLASSES).reshape(2, 11), torch.tensor(BOXES).reshape(11, 4))
    return f


def test_roi_normalize():
    f = _feature()
    RoiNormalize().transform(f)
    b = f[ImageFeature.label].bboxes
    assert torch.allclose(b[0], torch.tensor([0.004, 0.22399999, 0.11800001, 0.6613333]), atol=1e-6)
    assert torch.allclose(b[10], torch.tensor([0.674, 0.0026666666, 0.78000003, 0.28533334]), atol=1e-6)


def test_roi_hflip_pixels():
    f = _feature()
    RoiHFlip(False).transform(f)
    b = f[ImageFeature.label].bboxes
    assert b[0].tolist() == [441.0, 84.0, 498.0, 248.0] and b[3].tolist() == [4.0, 2.0, 180.0, 375.0]


def test_roi_project_after_center_crop():
    f = _feature()
    for t in (CenterCrop(300, 300), RoiNormalize(), RoiProject()):
        t.transform(f)
    b = f[ImageFeature.label].bboxes
    exp = torch.tensor([0.0, 0.25833336, 0.44333336, 0.805, 0.0, 0.45166665, 0.9233333, 1.0,
                        0.40333334, 0.0, 0.8033333, 1.0, 0.116666675, 0.0, 0.4, 0.36833334,
                        0.0, 0.01833333, 0.1866667, 0.46500003, 0.5966667, 0.0, 0.77, 0.16166666,
                        0.73333335, 0.0, 0.8133333, 0.195, 0.78999996, 0.0, 0.9666667, 0.23166668]).reshape(8, 4)
    assert b.shape == (8, 4) and torch.allclose(b, exp, atol=1e-5)


def test_batch_sampler_overlap_constraint_and_random_sampler():
    import random

    gts = [BoundingBox(0.1, 0.1, 0.5, 0.5)]
    out = []
    BatchSampler(1, 50, 0.3, 1.0, 0.5, 2.0, minOverlap=0.5).sample(gts, out, random.Random(0))
    assert out and all(b.jaccardOverlap(gts[0]) >= 0.5 for b in out)
    f = _feature()
    RoiNormalize().transform(f)
    RandomSampler(seed=3).transform(f)
    b = f[ImageFeature.label].bboxes
    assert b.numel() == 0 or (b.min() >= 0 and b.max() <= 1)
    assert f[ImageFeature.label].classes.shape[1] == b.shape[0]
