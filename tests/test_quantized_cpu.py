"""Int8 inference on the CPU engine (reference T/nn/quantized/{QuantizationSpec, LinearSpec,
SpatialConvolutionSpec, SpatialDilatedConvolutionSpec, QuantizableSpec}.scala). The reference compares against
its BigQuant native library, which is not available here: parity is checked against the float model
(relative error bounds) and, for the integer arithmetic, against exact integer results."""
import os

import pytest
import torch

from bigdl_amd import nn
from bigdl_amd.nn.graph import Input
from bigdl_amd.quantized import (QuantizedLinear, QuantizedSpatialConvolution, QuantizedSpatialDilatedConvolution,
                                 quantization_loss, quantize, quantize_rows)
from bigdl_amd.utils.random_generator import RNG


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


def test_quantize_rows_symmetric():
    w = torch.tensor([[1.0, -2.0, 0.5], [0.0, 0.0, 0.0], [3.0, 3.0, -6.0]])
    q, s = quantize_rows(w)
    assert q.dtype == torch.int8
    assert q[0].tolist() == [64, -127, 32] and q[1].tolist() == [0, 0, 0] and q[2].tolist() == [64, 64, -127]
    assert torch.allclose(s, torch.tensor([2.0, 0.0, 6.0]) / 127)
    w2 = torch.randn(64, 300)
    q2, s2 = quantize_rows(w2)
    assert quantization_loss(w2.abs(), (q2.float() * s2[:, None]).abs()) < 0.02


def test_linear_integer_exact():
    # weights / inputs whose row max is 127: scales are exactly 1, so the result is the exact integer GEMM
    w = torch.randint(-127, 128, (5, 20)).float()
    w[:, 0] = 127
    x = torch.randint(-127, 128, (3, 20)).float()
    x[:, 1] = -127
    b = torch.arange(5).float()
    m = QuantizedLinear(20, 5, initWeight=w, initBias=b)
    assert torch.equal(m.forward(x), x @ w.t() + b)
    assert m.forward(x[0]).shape == (5,)


def test_linear_close_to_float():
    RNG.setSeed(3)
    f = nn.Linear(100, 40)
    x = torch.randn(8, 100)
    q = QuantizedLinear(100, 40, initWeight=f.weight, initBias=f.bias)
    assert _rel(q.forward(x), f.forward(x)) < 0.02
    with pytest.raises(NotImplementedError):
        q.backward(x, torch.ones(8, 40))


@pytest.mark.parametrize("cfg", [
    dict(cin=3, cout=8, k=3, s=1, p=1, g=1),
    dict(cin=16, cout=24, k=1, s=2, p=0, g=1),
    dict(cin=12, cout=8, k=3, s=2, p=1, g=2),
    dict(cin=20, cout=32, k=5, s=1, p=2, g=1),
])
def test_conv_close_to_float(cfg):
    RNG.setSeed(5)
    f = nn.SpatialConvolution(cfg["cin"], cfg["cout"], cfg["k"], cfg["k"], cfg["s"], cfg["s"], cfg["p"], cfg["p"],
                              nGroup=cfg["g"])
    x = torch.randn(2, cfg["cin"], 13, 11)
    q = QuantizedSpatialConvolution(cfg["cin"], cfg["cout"], cfg["k"], cfg["k"], cfg["s"], cfg["s"], cfg["p"],
                                    cfg["p"], nGroup=cfg["g"], initWeight=f.weight, initBias=f.bias)
    y, yf = q.forward(x), f.forward(x)
    assert y.shape == yf.shape
    assert _rel(y, yf) < 0.03


def test_conv_integer_exact_and_nhwc():
    w = torch.randint(-127, 128, (6, 4, 3, 3)).float()
    w[:, 0, 0, 0] = -127
    x = torch.randint(-127, 128, (2, 4, 7, 7)).float()
    x[:, 0, 0, 0] = 127
    m = QuantizedSpatialConvolution(4, 6, 3, 3, 1, 1, 1, 1, initWeight=w)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), None, 1, 1).float()
    assert torch.equal(m.forward(x), ref)
    mn = QuantizedSpatialConvolution(4, 6, 3, 3, 1, 1, 1, 1, initWeight=w, format="NHWC")
    assert torch.equal(mn.forward(x.permute(0, 2, 3, 1)), ref.permute(0, 2, 3, 1))


def test_dilated_conv():
    RNG.setSeed(7)
    f = nn.SpatialDilatedConvolution(8, 8, 3, 3, 1, 1, 2, 2, 2, 2)
    x = torch.randn(1, 8, 12, 12)
    q = QuantizedSpatialDilatedConvolution(8, 8, 3, 3, 1, 1, 2, 2, 2, 2, initWeight=f.weight, initBias=f.bias)
    assert _rel(q.forward(x), f.forward(x)) < 0.03


def _small_cnn():
    m = nn.Sequential()
    m.add(nn.SpatialConvolution(3, 16, 3, 3, 1, 1, 1, 1)).add(nn.SpatialBatchNormalization(16)).add(nn.ReLU())
    m.add(nn.SpatialMaxPooling(2, 2, 2, 2))
    m.add(nn.SpatialConvolution(16, 32, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
    m.add(nn.Reshape([32 * 4 * 4])).add(nn.Linear(32 * 4 * 4, 10)).add(nn.LogSoftMax())
    return m


def test_model_quantize_folds_bn_and_keeps_original():
    RNG.setSeed(11)
    m = _small_cnn()
    bn = m.modules[1]
    bn.runningMean.uniform_(-0.2, 0.2)
    bn.runningVar.uniform_(0.5, 2.0)
    bn.weight.data.uniform_(0.5, 1.5)
    m.evaluate()
    x = torch.randn(4, 3, 8, 8)
    ref = m.forward(x).clone()
    q = m.quantize()
    kinds = [type(c).__name__ for c in q.modules]
    assert "SpatialBatchNormalization" not in kinds
    assert kinds.count("QuantizedSpatialConvolution") == 2 and "QuantizedLinear" in kinds
    assert type(m.modules[0]).__name__ == "SpatialConvolution"          # original untouched
    assert torch.allclose(m.forward(x), ref)
    y = q.forward(x)
    assert _rel(y.exp(), ref.exp()) < 0.05
    q2 = quantize(m, fold_bn=False)
    assert "SpatialBatchNormalization" in [type(c).__name__ for c in q2.modules]
    assert _rel(q2.forward(x).exp(), ref.exp()) < 0.05


def test_graph_quantize_and_serialize(tmp_path):
    RNG.setSeed(13)
    inp = Input()
    c = nn.SpatialConvolution(3, 8, 3, 3, 1, 1, 1, 1).inputs(inp)
    r = nn.ReLU().inputs(c)
    fl = nn.Reshape([8 * 6 * 6]).inputs(r)
    out = nn.Linear(8 * 6 * 6, 5).inputs(fl)
    g = nn.Graph([inp], [out])
    g.evaluate()
    x = torch.randn(2, 3, 6, 6)
    ref = g.forward(x).clone()
    q = g.quantize()
    assert any(type(mm).__name__ == "QuantizedLinear" for mm in q.modules)
    y = q.forward(x)
    assert _rel(y, ref) < 0.03
    p = os.path.join(tmp_path, "q.bigdl")
    q.saveModule(p, overWrite=True)
    from bigdl_amd.nn.module import Module
    q3 = Module.loadModule(p)
    assert torch.equal(q3.forward(x), y)


def test_quantize_graph_folds_bn_and_calibrates():
    """A Graph (e.g. Caffe-imported) quantizes with BN folded through the IR; calibration sets static ranges
    (MklInt8Convertible.calcScales analogue) on every quantized layer."""
    import torch
    from bigdl_amd.models.resnet import DatasetType, ResNet
    from bigdl_amd.quantized.quantizer import quantize

    torch.manual_seed(0)
    m = ResNet(10, 20, dataSet=DatasetType.CIFAR10)
    m.evaluate()
    x = torch.randn(4, 3, 32, 32)
    ref = m.forward(x)
    q = quantize(m.toGraph(), calibration=x)
    qs = [l for l in q.flattened_layers() if "Quantized" in type(l).__name__]
    assert len(qs) == 22 and all(getattr(l, "inputAmax", None) is not None for l in qs)
    assert not any(type(l).__name__ == "SpatialBatchNormalization" for l in q.flattened_layers())
    out = q.forward(x)
    assert ((out - ref).norm() / ref.norm()).item() < 5e-2
