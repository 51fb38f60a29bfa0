"""TensorFlow op kernels (nn/tf_ops.py, nn/tf.py gradient ops) on the GPU engine vs the CPU engine: Conv2D,
DepthwiseConv2dNative, Conv2DBackpropInput / Filter, Conv3D, Max/AvgPool (SAME, VALID) and their gradient ops run
on the native conv / pooling kernels (torch's vendor convolutions and pooling are patched to raise)."""
import pytest
import torch
import torch.nn.functional as F

from bigdl_amd.nn import tf as tfl
from bigdl_amd.nn.tf_ops import run_op
from bigdl_amd.utils.table import T

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _block(monkeypatch):
    def boom(*a, **k):
        raise AssertionError("vendor conv / pooling reached on the GPU path")

    for n in ("conv2d", "conv3d", "conv_transpose2d", "max_pool2d", "avg_pool2d"):
        monkeypatch.setattr(F, n, boom)


def _bf(*shape):
    return torch.randn(*shape).to(torch.bfloat16).float()


OPS = [
    ("Conv2D", lambda: [_bf(2, 9, 9, 6), _bf(3, 3, 6, 10)], {"strides": [1, 2, 2, 1], "padding": "SAME"}),
    ("Conv2D", lambda: [_bf(2, 8, 7, 5), _bf(2, 3, 5, 8)], {"strides": [1, 1, 1, 1], "padding": "VALID"}),
    ("DepthwiseConv2dNative", lambda: [_bf(2, 8, 8, 6), _bf(3, 3, 6, 2)], {"strides": [1, 1, 1, 1], "padding": "SAME"}),
    ("MaxPool", lambda: [_bf(2, 9, 10, 5)], {"ksize": [1, 3, 3, 1], "strides": [1, 2, 2, 1], "padding": "SAME"}),
    ("AvgPool", lambda: [_bf(2, 9, 10, 5)], {"ksize": [1, 3, 2, 1], "strides": [1, 2, 2, 1], "padding": "SAME"}),
    ("AvgPool", lambda: [_bf(2, 9, 10, 5)], {"ksize": [1, 2, 2, 1], "strides": [1, 2, 2, 1], "padding": "VALID"}),
]


@pytest.mark.parametrize("op,make,attrs", OPS, ids=[f"{o[0]}_{o[2]['padding']}_{i}" for i, o in enumerate(OPS)])
def test_tf_op_gpu_matches_cpu(op, make, attrs, monkeypatch):
    torch.manual_seed(0)
    xs = make()
    ref = run_op(op, xs, attrs)
    _block(monkeypatch)
    out = run_op(op, [x.cuda() for x in xs], attrs)
    assert out.shape == ref.shape
    assert _rel(out, ref) < 1e-2


def test_conv2d_backprop_input_gpu_matches_cpu(monkeypatch):
    torch.manual_seed(1)
    sizes = torch.tensor([2, 9, 9, 6])
    w, dy = _bf(3, 3, 6, 10), _bf(2, 5, 5, 10)
    attrs = {"strides": [1, 2, 2, 1], "padding": "SAME"}
    ref = run_op("Conv2DBackpropInput", [sizes, w, dy], attrs)
    _block(monkeypatch)
    out = run_op("Conv2DBackpropInput", [sizes, w.cuda(), dy.cuda()], attrs)
    assert out.shape == ref.shape and _rel(out, ref) < 1e-2


def test_pool_grad_ops_gpu_match_cpu(monkeypatch):
    torch.manual_seed(2)
    x = _bf(2, 9, 10, 5)
    mp = tfl.MaxPoolGrad(3, 3, 2, 2, "SAME")
    y = run_op("MaxPool", [x], {"ksize": [1, 3, 3, 1], "strides": [1, 2, 2, 1], "padding": "SAME"})
    g = _bf(*y.shape)
    ref = mp.forward(T(x, y, g))
    ap = tfl.AvgPoolGrad(3, 3, 2, 2, "SAME")
    aref = ap.forward(T(torch.tensor(list(x.shape)), g))
    _block(monkeypatch)
    out = mp.forward(T(x.cuda(), y.cuda(), g.cuda()))
    assert _rel(out, ref) < 1e-5
    aout = ap.forward(T(torch.tensor(list(x.shape)), g.cuda()))
    assert _rel(aout, aref) < 1e-5
