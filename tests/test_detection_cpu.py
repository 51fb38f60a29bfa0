"""Detection layers vs the reference specs' own fixtures (T/nn/{RoiAlignSpec, RoiPoolingSpec, NmsSpec, PriorBoxSpec,
PoolerSpec, BoxHeadSpec}.scala; numbers extracted with tools/extract_scala_arrays.py / extract_scala_fixture.py)."""
import json
import os

import numpy as np
import pytest
import torch

from bigdl_amd import nn
from bigdl_amd.utils.table import T, Table

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "detection")


def _fx(name):
    return json.load(open(os.path.join(FIX, name)))


def test_roi_align_fixture():
    d = _fx("roialign.json")
    x = torch.tensor(d["data"]).reshape(1, 2, 6, 8)
    rois = torch.tensor(d["rois"]).reshape(4, 4)
    out = nn.RoiAlign(1.0, 3, 2, 2).forward(T(x, rois))
    assert out.shape == (4, 2, 2, 2)
    assert torch.allclose(out.reshape(-1), torch.tensor(d["expectedRes"]), atol=1e-5)


def test_roi_pooling_fixture_fwd_bwd():
    d = _fx("roipool.json")
    x = torch.tensor(d["data"], dtype=torch.float32).reshape(2, 2, 6, 8)
    rois = torch.tensor(d["rois"], dtype=torch.float32).reshape(4, 5)
    m = nn.RoiPooling(3, 2, 1.0)
    out = m.forward(T(x, rois))
    assert torch.allclose(out.reshape(-1), torch.tensor(d["expectedRes"]), atol=1e-5)
    g = m.backward(T(x, rois), torch.tensor(d["gradOutputData"]).reshape(out.shape))[1]
    assert torch.allclose(g.reshape(-1), torch.tensor(d["expectedGradInput"]), atol=1e-5)
    g2 = m.backward(T(x, rois), torch.tensor(d["gradOutputData2"]).reshape(out.shape))[1]
    assert torch.allclose(g2.reshape(-1), torch.tensor(d["expectedGradInput2"]), atol=1e-5)


@pytest.mark.parametrize("thresh,key", [(0.4, "expected_04"), (0.1, "expected_01")])
def test_nms_fixture(thresh, key):
    d = _fx("nms.json")
    dets = torch.tensor(d["dets"], dtype=torch.float32).reshape(112, 5)
    idx = [0] * 112
    n = nn.Nms().nms(dets[:, 4].contiguous(), dets[:, :4].contiguous(), thresh, idx)
    assert idx[:n] == d[key]


def test_prior_box_fixture():
    layer = nn.PriorBox([460.8], [537.6], [2.0], isFlip=True, isClip=False, variances=[0.1, 0.1, 0.2, 0.2],
                        step=0, offset=0.5, imgH=512, imgW=512)
    out = layer.forward(torch.zeros(8, 256, 1, 1))
    exp = [0.0507812, 0.0507812, 0.949219, 0.949219, 0.0146376, 0.0146376, 0.985362, 0.985362, -0.135291, 0.182354,
           1.13529, 0.817646, 0.182354, -0.135291, 0.817646, 1.13529] + [0.1, 0.1, 0.2, 0.2] * 4
    assert out.shape == (1, 2, 16)
    assert torch.allclose(out.reshape(-1), torch.tensor(exp), atol=1e-5)


def test_pooler_fixture():
    d = _fx("pooler.json")
    feats = T(torch.tensor(d["feature1"]).reshape(1, 2, 8, 8), torch.tensor(d["feature2"]).reshape(1, 2, 4, 4),
              torch.tensor(d["feature3"]).reshape(1, 2, 2, 2))
    rois = torch.tensor([[0, 0, 10, 10], [0, 0, 60, 60], [0, 0, 500, 500]], dtype=torch.float32)
    out = nn.Pooler(2, [0.125, 0.0625, 0.03125], 2).forward(T(feats, T(rois)))
    assert torch.allclose(out.reshape(-1), torch.tensor(d["expectedRes"]), atol=1e-4)


def test_anchor_matches_faster_rcnn_table():
    a = nn.Anchor([0.5, 1.0, 2.0], [8.0, 16.0, 32.0]).basicAnchors
    exp = torch.tensor([[-84, -40, 99, 55], [-176, -88, 191, 103], [-360, -184, 375, 199], [-56, -56, 71, 71],
                        [-120, -120, 135, 135], [-248, -248, 263, 263], [-36, -80, 51, 95], [-80, -168, 95, 183],
                        [-168, -344, 183, 359]], dtype=torch.float32)
    assert torch.equal(a, exp)
    all_a = nn.Anchor([0.5, 1.0, 2.0], [8.0, 16.0, 32.0]).generateAnchors(3, 2, 16)
    assert all_a.shape == (2 * 3 * 9, 4)
    assert torch.equal(all_a[9], exp[0] + torch.tensor([16.0, 0, 16.0, 0]))


def test_box_head_fixture():
    d = _fx("boxhead.json")
    layer = nn.BoxHead(6, 7, [0.25, 0.125], 2, 0.012, 0.5, 100, 1024, 81)
    w, _ = layer.getParameters()
    w.fill_(0.001)
    f1 = torch.tensor(d["features1"], dtype=torch.float32)
    f2 = torch.tensor(d["features2"], dtype=torch.float32)
    layer.evaluate()
    out = layer.forward(T(T(f1, f2), T(torch.tensor(d["bbox"])), torch.tensor(d["imageInfo"], dtype=torch.float32)))
    res = out[2]
    labels = res[1]
    assert labels.tolist() == [float(c) for c in range(1, 81) for _ in range(2)]
    boxes = res[2][1]
    assert torch.allclose(boxes, torch.tensor(d["expectedBbox"]), atol=1e-3)


def test_mask_head_and_fpn_shapes():
    fpn = nn.FPN([4, 8, 16], 8, topBlocks=1)
    feats = fpn.forward(T(torch.randn(1, 4, 16, 16), torch.randn(1, 8, 8, 8), torch.randn(1, 16, 4, 4)))
    assert [tuple(feats[i].shape) for i in range(1, 5)] == [(1, 8, 16, 16), (1, 8, 8, 8), (1, 8, 4, 4), (1, 8, 2, 2)]
    mh = nn.MaskHead(8, 14, [0.25, 0.125], 2, [8, 8], 1, 5)
    mh.evaluate()
    props = T(torch.tensor([[0.0, 0.0, 20.0, 20.0], [10.0, 4.0, 40.0, 30.0]]))
    out = mh.forward(T(T(feats[1], feats[2]), props, torch.tensor([1.0, 3.0])))
    assert tuple(out[1].shape) == (2, 8, 14, 14) and tuple(out[2].shape) == (2, 1, 28, 28)
    assert float(out[2].min()) >= 0 and float(out[2].max()) <= 1


def test_region_proposal_and_proposal():
    rp = nn.RegionProposal(8, [32, 64], [0.5, 1.0, 2.0], [4, 8], 50, 20, 50, 20)
    rp.evaluate()
    feats = T(torch.randn(2, 8, 16, 16), torch.randn(2, 8, 8, 8))
    out = rp.forward(T(feats, torch.tensor([64.0, 64.0])))
    assert out.length() == 2 and out[1].shape[1] == 4 and out[1].shape[0] <= 20
    assert float(out[1].min()) >= 0 and float(out[1].max()) <= 63
    prop = nn.Proposal(200, 100, [0.5, 1.0, 2.0], [4.0, 5.0, 6.0])
    prop.evaluate()
    o = prop.forward(T(torch.randn(1, 18, 20, 30), torch.randn(1, 36, 20, 30) * 0.1,
                       torch.tensor([[300.0, 300.0, 1.0, 1.0]])))
    assert o.shape[1] == 5 and 0 < o.shape[0] <= 100 and torch.all(o[:, 0] == 0)


def test_detection_outputs():
    torch.manual_seed(0)
    npri = 30
    prior = nn.PriorBox([30.0], [60.0], [2.0], variances=[0.1, 0.1, 0.2, 0.2], imgH=300, imgW=300).forward(
        torch.zeros(1, 4, 3, 2))
    npri = prior.shape[2] // 4
    ssd = nn.DetectionOutputSSD(nClasses=4, keepTopK=5)
    ssd.evaluate()
    out = ssd.forward(T(torch.randn(2, npri * 4) * 0.1, torch.randn(2, npri * 4), prior))
    assert out.shape[0] == 2 and out.shape[1] == 1 + 5 * 6
    assert int(out[0, 0]) == 5
    rows = out[0, 1:].reshape(5, 6)
    assert set(rows[:, 0].tolist()) <= {1.0, 2.0, 3.0}
    fr = nn.DetectionOutputFrcnn(nClasses=3, maxPerImage=4)
    fr.evaluate()
    rois = torch.tensor([[0, 10, 10, 50, 50], [0, 12, 12, 52, 52], [0, 100, 100, 150, 140]], dtype=torch.float32)
    scores = torch.tensor([[0.1, 0.8, 0.1], [0.1, 0.7, 0.2], [0.2, 0.1, 0.7]])
    o = fr.forward(T(torch.tensor([[200.0, 200.0, 1.0, 1.0]]), rois, torch.zeros(3, 12), scores))
    n = int(o[0, 0])
    det = o[0, 1:].reshape(n, 6)
    assert n == 4 and det[:, 0].tolist() == [1.0, 1.0, 2.0, 2.0]   # the overlapping pair collapses in each class


def test_detection_modules_serialize(tmp_path):
    from bigdl_amd.nn.module import Module

    for m in [nn.RoiAlign(0.5, 2, 3, 3), nn.RoiPooling(3, 2, 0.5), nn.Pooler(2, [0.25, 0.125], 2),
              nn.FPN([4, 8], 4), nn.DetectionOutputSSD(), nn.DetectionOutputFrcnn(),
              nn.PriorBox([30.0], imgH=300, imgW=300)]:
        p = os.path.join(tmp_path, type(m).__name__ + ".bigdl")
        m.saveModule(p, overWrite=True)
        m2 = Module.loadModule(p)
        assert type(m2) is type(m)
    fpn = nn.FPN([4, 8], 4)
    p = os.path.join(tmp_path, "fpn2.bigdl")
    fpn.saveModule(p, overWrite=True)
    f2 = Module.loadModule(p)
    x = T(torch.randn(1, 4, 8, 8), torch.randn(1, 8, 4, 4))
    a, b = fpn.forward(x), f2.forward(x)
    assert torch.allclose(a[1], b[1]) and torch.allclose(a[2], b[2])
