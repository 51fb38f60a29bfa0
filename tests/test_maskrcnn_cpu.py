"""Mask R-CNN end-to-end inference on the CPU engine (reference T/models/maskrcnn/MaskRCNNSpec: structure and
output format; weights are random — no COCO checkpoint is available offline)."""
import torch

from bigdl_amd.dataset.segmentation import RLEMasks, rle_to_binary
from bigdl_amd.models import MaskRCNN, MaskRCNNParams
from bigdl_amd.models.maskrcnn import decode_mask_in_image
from bigdl_amd.utils.random_generator import RNG
from bigdl_amd.utils.table import T


def test_decode_mask_in_image():
    m = torch.ones(1, 4, 4)
    out = decode_mask_in_image(m, torch.tensor([2.0, 3.0, 9.0, 8.0]), 12, 14)
    ys, xs = torch.nonzero(out, as_tuple=True)
    assert out.shape == (12, 14)
    assert int(xs.min()) >= 1 and int(xs.max()) <= 10 and int(ys.min()) >= 2 and int(ys.max()) <= 9


def test_maskrcnn_inference_format():
    RNG.setSeed(1)
    torch.manual_seed(1)
    cfg = MaskRCNNParams(preNmsTopNTest=60, postNmsTopNTest=20, boxScoreThresh=0.0, maxPerImage=6, outputSize=32,
                         layers=[16, 16])
    m = MaskRCNN(16, 16, numClasses=3, config=cfg)
    m.evaluate()
    img = torch.randn(1, 3, 64, 96)
    out = m.forward(T(img, torch.tensor([[64.0, 96.0, 128.0, 192.0]])))
    r = out[1]
    n = r["bboxes"].shape[0]
    assert 0 < n <= 6
    assert r["classes"].shape == (n,) and r["scores"].shape == (n,)
    assert len(r["masks"]) == n and all(isinstance(x, RLEMasks) for x in r["masks"])
    assert (r["masks"][0].height, r["masks"][0].width) == (128, 192)
    assert rle_to_binary(r["masks"][0]).shape == (128, 192)
    assert float(r["bboxes"][:, 2].max()) <= 192
