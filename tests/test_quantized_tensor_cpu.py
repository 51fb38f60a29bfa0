"""QuantizedTensor (reference S/tensor/QuantizedTensor.scala, Quantization.scala; QuantizedTensorSpec-style checks):
per-row statistics, Java round-half-up quantization, 1-based size / stride, set (shared) vs copy (deep), equality,
hashing, release, persistence and the int8 layers' weight views."""
import torch

from bigdl_amd.quantized.modules import QuantizedLinear, QuantizedSpatialConvolution
from bigdl_amd.tensor import QuantizedTensor, Tensor


def test_quantize_rows_statistics_and_error_bound():
    torch.manual_seed(0)
    w = torch.randn(6, 3, 2, 2)
    qt = QuantizedTensor(w)
    assert qt.getTensorType() == "QuantizedType"
    assert qt.size() == [6, 3, 2, 2] and qt.size(2) == 3 and qt.dim() == 4 and qt.nElement() == 72
    assert qt.stride() == [12, 4, 2, 1] and qt.stride(1) == 12
    rows = w.reshape(6, -1)
    assert torch.allclose(qt.maxOfRow, rows.amax(1)) and torch.allclose(qt.minOfRow, rows.amin(1))
    assert torch.allclose(qt.sumOfRow, rows.sum(1))
    thr = torch.maximum(rows.amax(1).abs(), rows.amin(1).abs())
    err = (qt.dequantize().reshape(6, -1) - rows).abs()
    assert bool((err <= thr[:, None] / 254 + 1e-7).all())
    assert qt.getStorage().dtype == torch.int8 and qt.getStorage().numel() == 72


def test_round_half_up_like_java():
    # threshold 127: values map to themselves; x.5 rounds up (Java Math.round), -x.5 rounds toward +inf
    x = torch.tensor([[127.0, 2.5, -2.5, 0.5, -0.5, -127.0]])
    qt = QuantizedTensor(x)
    assert qt.getStorage().tolist() == [127, 3, -2, 1, 0, -127]


def test_set_shares_copy_deep_equality_hash_release():
    torch.manual_seed(1)
    a = QuantizedTensor(torch.randn(4, 5))
    b = QuantizedTensor(size=[4, 5]).set(a)
    assert b.getNativeStorage() is a.getNativeStorage() and b == a
    c = QuantizedTensor(size=[4, 5]).copy(a)
    assert c == a and hash(c) == hash(a)
    assert c.getNativeStorage().data_ptr() != a.getNativeStorage().data_ptr()
    c.getNativeStorage()[0, 0] = -a.getNativeStorage()[0, 0] - 1
    assert c != a
    assert QuantizedTensor(torch.randn(4, 6)) != a
    a.release()
    assert a.getStorage() is None and a.size() == [4, 5]
    b.set()
    assert b.getStorage() is None


def test_from_bytes_and_state_dict_round_trip():
    q = torch.randint(-127, 128, (3, 4), dtype=torch.int8)
    mx, mn = torch.tensor([1.0, 2.0, 3.0]), torch.tensor([-0.5, -4.0, 0.0])
    qt = QuantizedTensor.from_bytes(q, mx, mn, None, [3, 4])
    assert torch.allclose(qt.scale(), torch.tensor([1.0, 4.0, 3.0]) / 127)
    back = QuantizedTensor.from_state_dict(qt.state_dict())
    assert back == qt and torch.equal(back.maxOfRow, mx)
    try:
        QuantizedTensor.from_bytes(q, mx, mn, None, [5, 4])
        raise AssertionError("size mismatch accepted")
    except ValueError:
        pass


def test_quantized_layers_expose_weight_views():
    torch.manual_seed(2)
    w = torch.randn(8, 20)
    lin = QuantizedLinear(20, 8, initWeight=w)
    qt = lin.quantized_weight()
    assert qt.size() == [8, 20]
    assert torch.allclose(qt.dequantize(), lin.dequantized_weight(), atol=1e-6)
    conv = QuantizedSpatialConvolution(3, 6, 3, 3)
    conv.set_float_weights(torch.randn(6, 3, 3, 3))
    cq = conv.quantized_weight()
    assert cq.size() == [6, 3, 3, 3]           # NHWC weight order [out, kH, kW, in]
    assert torch.allclose(cq.dequantize().permute(0, 3, 1, 2), conv.dequantized_weight(), atol=1e-6)


def test_accepts_bigdl_tensor():
    t = Tensor(torch.arange(12.0).reshape(3, 4))
    qt = QuantizedTensor(t)
    assert qt.size() == [3, 4] and qt.getStorage()[3].item() == 127
