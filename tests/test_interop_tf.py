"""TensorFlow GraphDef import / export (reference T/utils/tf/{TensorflowLoaderSpec, TFUtilsSpec,
TensorflowSaverSpec, SessionSpec}; fixtures test.pb / consts.pbtxt / lenet_batch_2.pbtxt from T/resources/tf)."""
import os

import pytest
import torch

from bigdl_amd import nn
from bigdl_amd.interop.tensorflow import Session, attrs_of, load_tf, read_graph, save_tf
from bigdl_amd.utils.table import T

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "tf")
PB = os.path.join(FIX, "test.pb")


def _ref(x):
    return torch.tanh(x @ torch.full((1, 10), 0.2) + 0.1) @ torch.full((10, 1), 0.2) + 0.1


def test_parse_pb_nodes():
    nodes = read_graph(PB)
    assert len(nodes) == 14
    assert nodes[0]["op"][0] == "Placeholder"


def test_build_graph_and_forward():
    g = load_tf(PB, ["Placeholder"], ["output"])
    assert len(g.modules) == 4
    x = torch.rand(4, 1)
    assert torch.allclose(g.forward(x), _ref(x), atol=1e-6)


def test_sub_graph():
    g = load_tf(PB, ["Tanh"], ["output"])
    assert len(g.modules) == 3
    x = torch.rand(4, 10)
    assert torch.allclose(g.forward(x), torch.tanh(x) @ torch.full((10, 1), 0.2) + 0.1, atol=1e-6)


def test_bad_inputs():
    with pytest.raises(ValueError):
        load_tf(PB, ["Placeholder", "Placeholder"], ["output"])
    with pytest.raises(ValueError):
        load_tf(PB, ["NoSuchNode"], ["output"])


def test_consts_pbtxt_dtypes():
    nodes = {n["name"][0]: attrs_of(n)["value"] for n in read_graph(os.path.join(FIX, "consts.pbtxt"))}
    assert nodes["bool_const"].tolist() == [True, False, True, False]
    assert nodes["float_const"].tolist() == [1.0, 2.0, 3.0, 4.0] and nodes["float_const"].dtype == torch.float32
    assert nodes["double_const"].dtype == torch.float64
    for k in ("int_const", "long_const", "int8_const", "uint8_const", "int16_const", "uint16_const"):
        assert nodes[k].tolist() == [1, 2, 3, 4], k
    assert nodes["string_const"] == [b"a", b"b", b"c", b"d"]


def test_lenet_pbtxt_parses_and_builds_inference_subgraph():
    nodes = read_graph(os.path.join(FIX, "lenet_batch_2.pbtxt"))
    assert len(nodes) == 789
    ops = {n["op"][0] for n in nodes}
    assert {"Conv2D", "MaxPool", "MatMul", "Softmax"} <= ops


def test_trainable_after_import():
    g = load_tf(PB, ["Placeholder"], ["output"])
    x = torch.rand(8, 1)
    y = g.forward(x)
    g.zeroGradParameters()
    g.backward(x, torch.ones_like(y))
    w, gw = g.getParameters()
    assert w.numel() == 1 * 10 + 10 + 10 * 1 + 1 and gw.abs().sum() > 0


def test_save_and_reload_roundtrip(tmp_path):
    torch.manual_seed(0)
    m = nn.Sequential()
    m.add(nn.SpatialConvolution(3, 4, 3, 3, 1, 1, 1, 1, format="NHWC")).add(nn.ReLU())
    m.add(nn.SpatialMaxPooling(2, 2, 2, 2, format="NHWC"))
    m.add(nn.Reshape([4 * 4 * 4])).add(nn.Linear(64, 5)).add(nn.SoftMax())
    m.evaluate()
    x = torch.randn(2, 8, 8, 3)
    y = m.forward(x)
    p = os.path.join(tmp_path, "model.pb")
    out = save_tf(m, [("input", [None, 8, 8, 3])], p)
    g = load_tf(p, ["input"], [out])
    assert torch.allclose(g.forward(x), y, atol=1e-5)


def test_session_train(tmp_path):
    from bigdl_amd.dataset.core import DataSet, Sample
    from bigdl_amd.optim import SGD, Trigger

    samples = [Sample(torch.rand(1), torch.rand(1)) for _ in range(40)]
    model = Session(PB, ["Placeholder"]).train(["output"], DataSet.array(samples), SGD(0.01), nn.MSECriterion(),
                                               Trigger.maxEpoch(2), batchSize=8)
    assert model.forward(torch.rand(3, 1)).shape == (3, 1)


def test_tf_ops_semantics():
    from bigdl_amd.nn.tf_ops import run_op
    x = torch.arange(24.0).reshape(2, 3, 4)
    assert run_op("StridedSlice", [x, torch.tensor([0, 1, 0]), torch.tensor([2, 3, 4]), torch.tensor([1, 1, 2])],
                  {}).shape == (2, 2, 2)
    assert run_op("StridedSlice", [x, torch.tensor([1]), torch.tensor([2]), torch.tensor([1])],
                  {"shrink_axis_mask": 1}).shape == (3, 4)
    assert run_op("Sum", [x, torch.tensor([1])], {"keep_dims": True}).shape == (2, 1, 4)
    oh = run_op("OneHot", [torch.tensor([0, 2, -1]), torch.tensor(3), torch.tensor(1.0), torch.tensor(0.0)], {})
    assert oh.tolist() == [[1, 0, 0], [0, 0, 1], [0, 0, 0]]
    v, i = run_op("TopKV2", [torch.tensor([[1.0, 5.0, 3.0]]), torch.tensor(2)], {})
    assert v.tolist() == [[5.0, 3.0]] and i.tolist() == [[1, 2]]
    img = torch.randn(1, 5, 5, 2)
    w = torch.randn(3, 3, 2, 4)
    y = run_op("Conv2D", [img, w], {"strides": [1, 2, 2, 1], "padding": "SAME"})
    assert y.shape == (1, 3, 3, 4)
    dx = run_op("Conv2DBackpropInput", [torch.tensor([1, 5, 5, 2]), w, y],
                {"strides": [1, 2, 2, 1], "padding": "SAME"})
    assert dx.shape == (1, 5, 5, 2)
    p = run_op("MaxPool", [img], {"ksize": [1, 2, 2, 1], "strides": [1, 2, 2, 1], "padding": "SAME"})
    assert p.shape == (1, 3, 3, 2)
    assert run_op("ConcatV2", [x, x, torch.tensor(-1)], {}).shape == (2, 3, 8)
    parts = run_op("Split", [torch.tensor(1), x], {"num_split": 3})
    assert len(parts) == 3 and parts[0].shape == (2, 1, 4)


def test_reference_tf_utils_save_variables_and_merge_checkpoint(tmp_path):
    """bigdl.util.tf_utils: save_variable_bigdl + merge_checkpoint freeze a graph's variables into Consts (no
    TensorFlow needed), and the frozen graph loads and computes x @ w."""
    import numpy as np
    import torch

    from bigdl_amd.compat.util import tf_utils
    from bigdl_amd.interop.tensorflow import SCHEMA, _attr
    from bigdl_amd.nn.module import Module

    f32 = {"type": ["DT_FLOAT"]}
    nodes = [
        {"name": ["x"], "op": ["Placeholder"], "attr": [_attr("dtype", **f32)]},
        {"name": ["w"], "op": ["VariableV2"], "attr": [_attr("dtype", **f32)]},
        {"name": ["w/read"], "op": ["Identity"], "input": ["w"], "attr": [_attr("T", **f32)]},
        {"name": ["w/init"], "op": ["Const"], "attr": [_attr("dtype", **f32)]},
        {"name": ["w/Assign"], "op": ["Assign"], "input": ["w", "w/init"], "attr": [_attr("T", **f32)]},
        {"name": ["y"], "op": ["MatMul"], "input": ["x", "w/read"], "attr": [_attr("T", **f32)]},
    ]
    g = str(tmp_path / "g.pb")
    with open(g, "wb") as fh:
        fh.write(SCHEMA.encode("GraphDef", {"node": nodes}))
    w = np.arange(6, dtype=np.float32).reshape(3, 2)
    ck = str(tmp_path / "vars.bin")
    tf_utils.save_variable_bigdl({"w": w}, ck)
    out = str(tmp_path / "frozen.pb")
    tf_utils.merge_checkpoint(g, ck, ["y"], out)
    m = Module.loadTF(out, ["x"], ["y"])
    x = torch.randn(4, 3)
    assert torch.allclose(m.forward(x), x @ torch.from_numpy(w), atol=1e-5)
    try:
        tf_utils.export_checkpoint("ckpt")
        raise AssertionError("expected ImportError")
    except ImportError:
        pass
