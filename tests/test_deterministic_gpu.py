"""Deterministic mode (bigdl.deterministic, BIGDL_DETERMINISTIC=1): two ResNet-20 training runs from the same seed
end bitwise equal (reference: DistriOptimizerSpec "be same compare to ref optimizer", T/optim/DistriOptimizerSpec.scala:
378-428 asserts exact equality of trained parameters)."""
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
