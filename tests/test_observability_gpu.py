"""Device-time module timing (getTimes with HIP events, reference AbstractModule.scala:168-196) on the GPU."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _leaves(model):
    from bigdl_amd.nn.containers import Container

    return [m for m in model.flattened_layers() if not isinstance(m, Container)]


def test_get_times_reports_device_time():
    """With device timing on, a ResNet-50 forward / backward at batch 64 reports per-module device times: every conv
    has a non-zero forward time, the leaf forward times add up to the whole model's forward time (the events tile the
    stream), and the model's forward time matches an independent pair of events around model.forward."""
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import DatasetType, ResNet
    from bigdl_amd.nn import abstractnn
    from bigdl_amd.nn.fusion import fuse_for_training

    dev = torch.device("cuda:0")
    model = ResNet(1000, 50, dataSet=DatasetType.ImageNet).to(dev)
    fuse_for_training(model)
    crit = nn.CrossEntropyCriterion()
    x = torch.randn(64, 3, 224, 224, device=dev)
    y = torch.randint(1, 1001, (64,), device=dev).float()
    saved = abstractnn.DEVICE_TIMING[0]
    abstractnn.AbstractModule.setDeviceTiming(True)
    try:
        for it in range(3):
            model.resetTimes()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            out = model.forward(x)
            b.record()
            loss = crit.forward(out, y)
            model.backward(x, crit.backward(out, y))
            torch.cuda.synchronize()
        outer_ms = a.elapsed_time(b)
        times = model.getTimes()
    finally:
        abstractnn.DEVICE_TIMING[0] = saved
    assert torch.isfinite(loss).item()
    top_f, top_b = times[0][1] / 1e6, times[0][2] / 1e6
    assert top_f > 0 and top_b > 0
    convs = [t for t in times if isinstance(t[0], nn.SpatialConvolution)]
    assert len(convs) == 53 and all(f > 0 for _, f, _ in convs)
    # the top-level Sequential's children tile its forward on the stream; leaves inside fused residual blocks are run
    # by their block (nn/fusion.py residual_forward calls the last BN's updateOutput), so the leaf sum is a lower bound
    kid_ids = {id(m) for m in model.modules}
    kid_f = sum(f for m, f, _ in times if id(m) in kid_ids) / 1e6
    assert abs(kid_f - top_f) <= 0.1 * top_f, (kid_f, top_f)
    leaf_ids = {id(m) for m in _leaves(model)}
    leaf_f = sum(f for m, f, _ in times if id(m) in leaf_ids) / 1e6
    assert 0.3 * top_f < leaf_f <= 1.05 * top_f, (leaf_f, top_f)
    assert abs(top_f - outer_ms) <= 0.25 * outer_ms, (top_f, outer_ms)
    # host timing (device timing off) measures the enqueue only: no event pairs are queued
    model.resetTimes()
    model.forward(x)
    assert not model.__dict__.get("_dev_times")
