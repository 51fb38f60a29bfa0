"""Deterministic mode (bigdl.deterministic, BIGDL_DETERMINISTIC=1): two ResNet-20 training runs from the same seed
end bitwise equal (reference: DistriOptimizerSpec "be same compare to ref optimizer", T/optim/DistriOptimizerSpec.scala:
378-428 asserts exact equality of trained parameters)."""
import copy
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_resnet20_ten_iterations_bitwise_reproducible():
    from det_check import run

    w1, _ = run(10, True)
    w2, _ = run(10, True)
    assert torch.isfinite(w1).all()
    assert torch.equal(w1, w2), (w1 - w2).abs().max()


def test_engine_property_switches_mode():
    from bigdl_amd.ops import native
    from bigdl_amd.utils.engine import Engine

    e = Engine if not callable(getattr(Engine, "getInstance", None)) else Engine.getInstance()
    try:
        e.setProperty("bigdl.deterministic", "true")
        assert native.deterministic() and native.get().deterministic() == 1
    finally:
        e.setProperty("bigdl.deterministic", "false")
    assert not native.deterministic() and native.get().deterministic() == 0


@pytest.mark.parametrize("K", [64, 256, 2048])
def test_deterministic_reductions_exact_and_repeatable(K):
    """The deterministic-mode column sum (bias gradients) and BN statistics / backward sums (per-block partials summed
    in block order): equal to a float64 reference within fp32 rounding, and bitwise equal run to run."""
    from bigdl_amd.ops import native

    C = native.get()
    torch.manual_seed(K)
    P = 200_000 if K <= 256 else 25_000
    x = torch.randn(P, K, device="cuda").to(torch.bfloat16)
    dz = torch.randn(P, K, device="cuda").to(torch.bfloat16)
    mean = torch.randn(K, device="cuda") * 0.1
    saved = native.deterministic()
    native.set_deterministic(True)
    try:
        runs = []
        for _ in range(2):
            cs = torch.zeros(K, device="cuda")
            C.colsum_bf16(x, cs)
            st = torch.zeros(C.STAT_SLOTS * 2 * K, device="cuda")
            C.bn_stats(x, st, P, K)
            red = torch.zeros(C.STAT_SLOTS * 2 * K, device="cuda")
            C.bn_bwd_reduce(dz, None, x, mean, red, P, K)
            torch.cuda.synchronize()
            runs.append((cs.clone(), st.view(-1, 2 * K).sum(0), red.view(-1, 2 * K).sum(0)))
    finally:
        native.set_deterministic(saved)
    for a, b in zip(runs[0], runs[1]):
        assert torch.equal(a, b)
    xd, dd = x.double(), dz.double()
    ref_cs = xd.sum(0)
    ref_st = torch.cat([xd.sum(0), (xd * xd).sum(0)])
    ref_red = torch.cat([dd.sum(0), (dd * (xd - mean.double())).sum(0)])
    for got, ref in ((runs[0][0], ref_cs), (runs[0][1], ref_st), (runs[0][2], ref_red)):
        err = (got.double() - ref).abs().max().item()
        assert err < 1e-4 * (ref.abs().max().item() + P ** 0.5), err


def test_image_stem_training_bitwise_reproducible():
    """The 7x7/2 ImageNet stem (pair-view stem kernels, BN statistics outside the epilogue in deterministic mode) +
    BN + ReLU + max pool, three SGD steps twice from the same weights: bitwise equal parameters."""
    from bigdl_amd import nn
    from bigdl_amd.ops import native
    from bigdl_amd.optim.sgd import SGD
    from bigdl_amd.optim.train_step import TrainStep

    def build():
        m = nn.Sequential()
        m.add(nn.SpatialConvolution(3, 64, 7, 7, 2, 2, 3, 3)).add(nn.SpatialBatchNormalization(64)).add(nn.ReLU())
        m.add(nn.SpatialMaxPooling(3, 3, 2, 2, 1, 1)).add(nn.View(64 * 56 * 56)).add(nn.Linear(64 * 56 * 56, 10))
        return m

    saved = native.deterministic()
    native.set_deterministic(True)
    try:
        torch.manual_seed(1)
        x = torch.randn(16, 3, 224, 224, device="cuda")
        y = torch.randint(1, 11, (16,), device="cuda").float()
        ws = []
        base = build()          # one initialisation (the layers draw from the framework RNG), copied per run
        for _ in range(2):
            st = TrainStep(copy.deepcopy(base), nn.CrossEntropyCriterion(), SGD(0.01, momentum=0.9, dampening=0.0),
                           device="cuda")
            for _ in range(3):
                st.step(x, y)
            torch.cuda.synchronize()
            ws.append(st.w.detach().clone())
    finally:
        native.set_deterministic(saved)
    assert torch.isfinite(ws[0]).all()
    assert torch.equal(ws[0], ws[1]), (ws[0] - ws[1]).abs().max()
