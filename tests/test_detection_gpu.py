"""Detection HIP kernels (csrc/detection.hip) vs the CPU reference implementations (GPU only)."""
import json
import os

import pytest
import torch

from bigdl_amd import nn
from bigdl_amd.ops import detection as D
from bigdl_amd.utils.table import T

pytestmark = pytest.mark.gpu
FIX = os.path.join(os.path.dirname(__file__), "fixtures", "detection")


def _boxes(n, seed):
    g = torch.Generator().manual_seed(seed)
    xy = torch.rand(n, 2, generator=g) * 500
    wh = torch.rand(n, 2, generator=g) * 120 + 4
    return torch.cat([xy, xy + wh], 1), torch.rand(n, generator=g)


@pytest.mark.parametrize("n,thresh,normalized", [(112, 0.4, False), (1000, 0.7, False), (4100, 0.5, False),
                                                 (300, 0.45, True)])
def test_nms_gpu_matches_cpu(n, thresh, normalized):
    boxes, scores = _boxes(n, n)
    if normalized:
        boxes = boxes / 640.0
    order = torch.sort(scores, descending=True, stable=True).indices
    ref = D.nms_sorted(boxes[order], thresh, normalized)
    got = D.nms_sorted(boxes[order].cuda(), thresh, normalized)
    assert torch.equal(got.cpu(), ref)


def test_nms_fixture_gpu():
    d = json.load(open(os.path.join(FIX, "nms.json")))
    dets = torch.tensor(d["dets"], dtype=torch.float32).reshape(112, 5).cuda()
    keep = D.nms(dets[:, 4], dets[:, :4], 0.4)
    assert (keep.cpu() + 1).tolist() == d["expected_04"]


def test_roi_align_gpu():
    d = json.load(open(os.path.join(FIX, "roialign.json")))
    x = torch.tensor(d["data"]).reshape(1, 2, 6, 8)
    rois = torch.tensor(d["rois"]).reshape(4, 4)
    out = nn.RoiAlign(1.0, 3, 2, 2).forward(T(x.cuda(), rois.cuda()))
    assert torch.allclose(out.cpu().reshape(-1), torch.tensor(d["expectedRes"]), atol=1e-5)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 16, 25, 31, generator=g)
    r = torch.cat([torch.tensor([[0.0], [1.0], [1.0], [0.0]]),
                   torch.tensor([[1.0, 2.0, 60.0, 40.0], [-5.0, 3.0, 20.0, 80.0], [10.0, 10.0, 11.0, 11.0],
                                 [0.0, 0.0, 124.0, 100.0]])], 1)
    for samp in (0, 2):
        ref = D.roi_align(x, r, 0.25, samp, 7, 7)
        got = D.roi_align(x.cuda(), r.cuda(), 0.25, samp, 7, 7)
        assert torch.allclose(got.cpu(), ref, atol=1e-5)


def test_roi_pool_gpu_fwd_bwd():
    d = json.load(open(os.path.join(FIX, "roipool.json")))
    x = torch.tensor(d["data"], dtype=torch.float32).reshape(2, 2, 6, 8).cuda()
    rois = torch.tensor(d["rois"], dtype=torch.float32).reshape(4, 5).cuda()
    m = nn.RoiPooling(3, 2, 1.0)
    out = m.forward(T(x, rois))
    assert torch.allclose(out.cpu().reshape(-1), torch.tensor(d["expectedRes"]), atol=1e-5)
    g = m.backward(T(x, rois), torch.tensor(d["gradOutputData"]).reshape(out.shape).cuda())[1]
    assert torch.allclose(g.cpu().reshape(-1), torch.tensor(d["expectedGradInput"]), atol=1e-5)


def test_box_head_gpu_matches_cpu():
    torch.manual_seed(0)
    layer = nn.BoxHead(6, 7, [0.25, 0.125], 2, 0.012, 0.5, 100, 64, 5)
    layer.evaluate()
    feats = T(torch.randn(1, 6, 12, 16), torch.randn(1, 6, 6, 8))
    props = T(torch.tensor([[1.0, 3.0, 20.0, 26.0], [3.0, 5.0, 36.0, 27.0], [0.0, 0.0, 40.0, 40.0]]))
    info = torch.tensor([48.0, 64.0])
    ref = layer.forward(T(feats, props, info))
    ref_feat, ref_res = ref[1].clone(), ref[2]
    ref_boxes = ref_res[2][1].clone()
    layer.cuda()
    out = layer.forward(T(T(feats[1].cuda(), feats[2].cuda()), T(props[1].cuda()), info.cuda()))
    assert torch.allclose(out[1].float().cpu(), ref_feat, atol=2e-2, rtol=2e-2)
    assert out[2][2][1].shape == ref_boxes.shape
