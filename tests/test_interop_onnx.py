"""ONNX import / export (reference P/contrib/onnx onnx_loader + ops_converter op set: Constant, Sum, Concat, Relu,
Conv, BatchNormalization, Softmax, Gemm, Reshape, Unsqueeze, AveragePool, MaxPool, Shape, Gather). The onnx
package is not installed, so models are produced by our own exporter / hand-built ModelProtos (parity unpinned
against onnxruntime)."""
import os

import torch

from bigdl_amd import nn
from bigdl_amd.interop.onnx import SCHEMA, _tp, load_onnx, save_onnx
from bigdl_amd.utils.random_generator import RNG
from bigdl_amd.utils.table import T


def test_export_import_roundtrip(tmp_path):
    RNG.setSeed(2)
    m = nn.Sequential()
    m.add(nn.SpatialConvolution(3, 8, 3, 3, 1, 1, 1, 1)).add(nn.SpatialBatchNormalization(8)).add(nn.ReLU())
    m.add(nn.SpatialMaxPooling(2, 2, 2, 2)).add(nn.SpatialConvolution(8, 4, 3, 3, 2, 2, 1, 1, nGroup=2))
    m.add(nn.Reshape([4 * 2 * 2])).add(nn.Linear(16, 5)).add(nn.SoftMax())
    bn = m.modules[1]
    bn.runningMean.uniform_(-0.1, 0.1)
    bn.runningVar.uniform_(0.5, 1.5)
    m.evaluate()
    x = torch.randn(2, 3, 8, 8)
    y = m.forward(x)
    p = os.path.join(tmp_path, "m.onnx")
    save_onnx(m, [None, 3, 8, 8], p)
    g = load_onnx(p)
    g.evaluate()
    assert torch.allclose(g.forward(x), y, atol=1e-5)
    kinds = [type(k).__name__ for k in g.modules]
    assert "SpatialConvolution" in kinds and "Linear" in kinds and "SpatialBatchNormalization" in kinds


def _node(op, ins, outs, **attrs):
    at = []
    for k, v in attrs.items():
        if isinstance(v, list):
            at.append({"name": [k], "ints": v, "type": [7]})
        elif isinstance(v, float):
            at.append({"name": [k], "f": [v], "type": [1]})
        else:
            at.append({"name": [k], "i": [v], "type": [2]})
    return {"input": ins, "output": outs, "name": [outs[0]], "op_type": [op], "attribute": at}


def test_reference_op_set(tmp_path):
    w = torch.randn(4, 6)
    nodes = [
        _node("Gemm", ["x", "W", "b"], ["g"], transB=1),
        _node("Relu", ["g"], ["r"]),
        _node("Shape", ["r"], ["s"]),
        _node("Gather", ["s", "one"], ["d1"], axis=0),
        _node("Unsqueeze", ["r"], ["u"], axes=[1]),
        _node("Concat", ["u", "u"], ["c"], axis=1),
        _node("Sum", ["r", "r", "r"], ["sum3"]),
        _node("Reshape", ["c", "shape"], ["rs"]),
        _node("Softmax", ["sum3"], ["sm"], axis=1),
    ]
    inits = [_tp("W", w), _tp("b", torch.zeros(4)), _tp("one", torch.tensor(1, dtype=torch.int64)),
             _tp("shape", torch.tensor([0, -1], dtype=torch.int64))]
    g = {"node": nodes, "initializer": inits, "input": [{"name": ["x"]}],
         "output": [{"name": ["rs"]}, {"name": ["sm"]}]}
    p = os.path.join(tmp_path, "ops.onnx")
    with open(p, "wb") as f:
        f.write(SCHEMA.encode("ModelProto", {"ir_version": [6], "graph": [g], "opset_import": [{"version": [11]}]}))
    model = load_onnx(p)
    x = torch.randn(3, 6)
    out = model.forward(x)
    r = torch.relu(x @ w.t())
    assert torch.allclose(out[1], torch.cat([r, r], 1), atol=1e-5)
    assert torch.allclose(out[2], torch.softmax(3 * r, 1), atol=1e-5)


def test_reference_contrib_onnx_loader(tmp_path):
    """bigdl.contrib.onnx.load / load_model_proto / calc_output_shape under the reference names."""
    import torch

    from bigdl_amd import nn
    from bigdl_amd.compat.contrib import onnx as conx
    from bigdl_amd.interop.onnx import save_onnx

    m = nn.Sequential().add(nn.SpatialConvolution(3, 4, 3, 3, 1, 1, 1, 1)).add(nn.ReLU())
    p = str(tmp_path / "m.onnx")
    save_onnx(m, [1, 3, 8, 8], p)
    x = torch.randn(1, 3, 8, 8)
    a = conx.load(p).value.forward(x)
    with open(p, "rb") as f:
        b = conx.load_model_proto(f.read()).value.forward(x)
    assert torch.allclose(a, m.forward(x), atol=1e-5) and torch.allclose(b, a)
    assert conx.calc_output_shape(224, 3, 1, 2) == 112 and conx.calc_output_shape(7, 2, 0, 2, ceil_mode=True) == 4
