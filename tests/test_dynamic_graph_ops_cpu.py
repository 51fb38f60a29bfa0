"""DynamicGraph + TF control flow (reference DynamicGraphSpec.scala:1275-1400, tf/ControlOpsSpec.scala), nn.ops
feature columns (ops/CategoricalColHashBucketSpec.scala, CrossColSpec.scala fixtures) and nn.tf modules."""
import os

import numpy as np
import pytest
import torch

from bigdl_amd import nn
from bigdl_amd.nn import ops as O
from bigdl_amd.nn import tf as TF
from bigdl_amd.nn.graph import Graph, Input
from bigdl_amd.utils.table import T, Table


def _while_graph():
    inp = Input("input")
    cin = Input("conditionInput")
    const = TF.Const(torch.tensor([9.0])).inputs()
    ce = TF.Enter("test_frame").inputs(const)
    less = O.Less().inputs(ce, cin)
    uin = Input()
    add = nn.AddConstant(1).inputs(uin)
    ae = TF.Enter("test_frame").inputs(add)
    echo = nn.Echo(feval=lambda m, t: None).inputs(ae)
    ex = TF.ControlNodes.whileLoop(([cin], less), [(uin, echo)], [inp], "while")
    return Graph.dynamic([inp], [ex[0]], None, False)


def test_while_loop_counts_to_ten():
    m = _while_graph()
    assert m.forward(torch.tensor([1.0])).item() == 10
    assert m.forward(torch.tensor([3.0])).item() == 10     # re-runnable


def test_while_loop_const_subgraph_runs_once():
    calls = []
    inp = Input()
    cin = Input()
    const = TF.Const(torch.tensor([9.0])).inputs()
    echo = nn.Echo(feval=lambda m, t: calls.append(1)).inputs(const)
    less = O.Less().inputs(echo, cin)
    uin = Input()
    add = nn.AddConstant(1).inputs(uin)
    ex = TF.ControlNodes.whileLoop(([cin], less), [(uin, add)], [inp])
    m = Graph.dynamic([inp], [ex[0]], None, False)
    m.forward(torch.tensor([1.0]))
    assert m.forward(torch.tensor([1.0])).item() == 10
    assert len(calls) == 1


def test_while_loop_multiple_vars():
    i1, i2, c1, c2 = Input(), Input(), Input(), Input()
    const = TF.Const(torch.tensor([9.0])).inputs()
    less = O.Less().inputs(const, c1)
    u1, u2 = Input(), Input()
    a1 = nn.AddConstant(1).inputs(u1)
    a2 = nn.AddConstant(5).inputs(u2)
    ex = TF.ControlNodes.whileLoop(([c1, c2], less), [(u1, a1), (u2, a2)], [i1, i2], "while")
    m = Graph.dynamic([i1, i2], ex, None, False)
    r = m.forward(T(torch.tensor([1.0]), torch.tensor([2.0])))
    assert r[1].item() == 10 and r[2].item() == 47


def test_switch_merge_takes_one_branch():
    data, pred = Input(), Input()
    sw = TF.ControlNodes.switch(pred, data)          # reference argument order: (data=pred, condition=data)
    neg = nn.MulConstant(-1.0).inputs((sw, 1))
    dbl = nn.MulConstant(2.0).inputs((sw, 2))
    mg = TF.ControlNodes.merge(neg, dbl)
    m = Graph.dynamic([data, pred], [mg], None, False)
    assert m.forward(T(torch.tensor([3.0]), torch.tensor([True]))).item() == 6.0
    assert m.forward(T(torch.tensor([3.0]), torch.tensor([False]))).item() == -3.0


def test_dynamic_graph_backward_matches_static():
    torch.manual_seed(0)
    x = Input()
    l1 = nn.Linear(4, 3).inputs(x)
    r = nn.ReLU().inputs(l1)
    l2 = nn.Linear(3, 2).inputs(r)
    dyn = Graph.dynamic([x], [l2])
    inp = torch.randn(5, 4)
    out = dyn.forward(inp)
    g = dyn.backward(inp, torch.ones_like(out))
    lin1, lin2 = l1.element, l2.element
    ref = torch.nn.functional.linear(torch.relu(torch.nn.functional.linear(inp, lin1.weight, lin1.bias)),
                                     lin2.weight, lin2.bias)
    assert torch.allclose(out, ref, atol=1e-6)
    x2 = inp.clone().requires_grad_(True)
    torch.nn.functional.linear(torch.relu(torch.nn.functional.linear(x2, lin1.weight, lin1.bias)),
                               lin2.weight, lin2.bias).sum().backward()
    assert torch.allclose(g, x2.grad, atol=1e-6)


def test_dynamic_graph_rejects_duplicate_module():
    n1, n2 = nn.Identity().inputs(), nn.Identity().inputs()
    dup = nn.Identity()
    n3, n4 = dup.inputs(n1), dup.inputs(n2)
    with pytest.raises(ValueError):
        Graph.dynamic([n1, n2], [n3, n4])


def test_dynamic_graph_serialization_roundtrip(tmp_path):
    from bigdl_amd.utils.serializer import load_module, save_module

    m = _while_graph()
    p = str(tmp_path / "dyn.bigdl")
    # Echo's lambda is not serializable: rebuild without it
    inp, cin = Input(), Input()
    const = TF.Const(torch.tensor([9.0])).inputs()
    ce = TF.Enter("test_frame").inputs(const)
    less = O.Less().inputs(ce, cin)
    uin = Input()
    add = nn.AddConstant(1).inputs(uin)
    ex = TF.ControlNodes.whileLoop(([cin], less), [(uin, add)], [inp], "while")
    m = Graph.dynamic([inp], [ex[0]], None, False)
    save_module(m, p, overWrite=True)
    m2 = load_module(p)
    assert type(m2).__name__ == "DynamicGraph"
    assert m2.forward(torch.tensor([1.0])).item() == 10


# ---------------------------------------------------------------------------------------------- nn.ops
def test_hash_bucket_matches_reference_fixture():
    out = O.CategoricalColHashBucket(100, isSparse=True).forward([["1"], ["2"], ["3"]])
    assert out.values().tolist() == [5, 53, 77]
    dense = O.CategoricalColHashBucket(100, isSparse=False).forward(["1,2", "2", "1,3,2"])
    assert dense.tolist() == [[5, 53, 0], [53, 0, 0], [5, 77, 53]]


def test_cross_col_matches_reference_fixture():
    out = O.CrossCol(100).forward(T(["A,D", "B", "A,C"], ["1", "2", "3,4"]))
    assert out.indices().tolist() == [[0, 0, 1, 2, 2, 2, 2], [0, 1, 0, 0, 1, 2, 3]]
    assert out.values().tolist() == [80, 98, 50, 99, 27, 89, 33]
    out3 = O.CrossCol(100).forward(T(["A,D", "B", "A,C"], ["1", "2", "3,4"], ["1", "2", "3"]))
    assert out3.values().tolist() == [94, 34, 68, 82, 83, 97, 12]


def test_voca_list_indicator_bucketized_kv():
    sp = O.CategoricalColVocaList(["A", "B", "C"], isSetDefault=True).forward(["A,D", "B", "A,C"])
    assert sp.to_dense().tolist() == [[0, 3, 0, 0], [1, 0, 0, 0], [0, 2, 0, 0]]
    ind = O.IndicatorCol(4, isCount=True).forward(sp)
    assert ind.tolist() == [[1, 0, 0, 1], [0, 1, 0, 0], [1, 0, 1, 0]]
    b = O.BucketizedCol([0.0, 10.0, 100.0]).forward(torch.tensor([[-1.0, 1.0], [101.0, 10.0]]))
    assert b.tolist() == [[0, 1], [3, 2]]
    kv = O.Kv2Tensor(transType=0).forward(T(["0:0.1,1:0.2", "2:0.3"], torch.tensor(3)))
    assert torch.allclose(kv, torch.tensor([[0.1, 0.2, 0.0], [0.0, 0.0, 0.3]]))
    assert O.MkString().forward(torch.tensor([[1, 2], [3, 4]])) == ["1,2", "3,4"]
    assert O.Substr().forward(T(["hello", "world"], torch.tensor(1), torch.tensor(3))) == ["ell", "orl"]


def test_elementwise_ops_and_reductions():
    a, b = torch.tensor([1.0, -2.0, 3.0]), torch.tensor([2.0, -2.0, 1.0])
    assert O.Greater().forward(T(a, b)).tolist() == [False, False, True]
    assert O.Maximum().forward(T(a, b)).tolist() == [2.0, -2.0, 3.0]
    assert O.FloorDiv().forward(T(torch.tensor([7, -7]), torch.tensor([2, 2]))).tolist() == [3, -4]
    x = torch.arange(6.0).reshape(2, 3)
    assert O.Sum().forward(T(x, torch.tensor([2]))).tolist() == [3.0, 12.0]          # 1-based axis
    assert O.Prod(startFromZero=True).forward(T(x, torch.tensor([0]))).tolist() == [0.0, 4.0, 10.0]
    v, i = O.TopK(2).forward(torch.tensor([[1.0, 5.0, 3.0]]))[1], O.TopK(2).forward(torch.tensor([[1.0, 5.0, 3.0]]))[2]
    assert v.tolist() == [[5.0, 3.0]] and i.tolist() == [[2, 3]]
    assert O.InTopK(1).forward(T(torch.tensor([[0.1, 0.9], [0.8, 0.2]]), torch.tensor([2, 2]))).tolist() == [True, False]
    with pytest.raises(RuntimeError):
        O.Greater().backward(T(a, b), torch.ones(3))


def test_tensor_op_algebra():
    op = (O.TensorOp.sqrt() >> O.TensorOp.add(1.0)) * 2.0
    assert op.forward(torch.tensor([4.0, 9.0])).tolist() == [6.0, 8.0]


# ---------------------------------------------------------------------------------------------- nn.tf
def test_tensor_array_and_stack():
    ta = TF.TensorArrayCreator(dynamicSize=True).forward(torch.tensor([2]))
    h = ta[1]
    TF.TensorArrayWrite().forward(T(h, torch.tensor(0), torch.ones(2), ta[2]))
    TF.TensorArrayWrite().forward(T(h, torch.tensor(1), torch.zeros(2), ta[2]))
    assert TF.TensorArraySize().forward(T(h)).item() == 2
    g = TF.TensorArrayGather().forward(T(h, torch.tensor([1, 0]), ta[2]))
    assert g.tolist() == [[0.0, 0.0], [1.0, 1.0]]
    TF.TensorArrayClose().forward(T(h))
    s = TF.StackCreator().forward(None)
    TF.StackPush().forward(T(s, torch.tensor([1.0])))
    TF.StackPush().forward(T(s, torch.tensor([2.0])))
    assert TF.StackPop().forward(s).item() == 2.0


def test_parse_example_roundtrip():
    recs = [TF.encode_example({"x": [1.0, 2.0], "y": [7]}), TF.encode_example({"x": [3.0, 4.0], "y": [8]})]
    out = TF.ParseExample(2, [torch.float32, torch.int64], [[2], [1]]).forward(
        T(recs, None, "x", "y", torch.zeros(2), torch.zeros(1, dtype=torch.int64)))
    assert out[1].tolist() == [[1.0, 2.0], [3.0, 4.0]]
    assert out[2].tolist() == [[7], [8]]


def test_decode_png_and_raw():
    from PIL import Image
    import io

    arr = (np.arange(2 * 3 * 3) % 255).astype(np.uint8).reshape(2, 3, 3)
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    out = TF.DecodePng(3).forward(buf.getvalue())
    assert out.shape == (2, 3, 3) and out.numpy().tolist() == arr.tolist()
    raw = TF.DecodeRaw(torch.int32).forward(np.array([1, 2], dtype="<i4").tobytes())
    assert raw.tolist() == [1, 2]


def test_variable_assign_and_grad_ops():
    v = TF.Variable(torch.ones(2))
    out = v.forward(None)
    v.backward(None, torch.tensor([0.5, 0.5]))
    assert out.tolist() == [1.0, 1.0] and v.gradWeight.tolist() == [0.5, 0.5]
    ref = torch.zeros(2)
    TF.Assign().forward(T(ref, torch.tensor([3.0, 4.0])))
    assert ref.tolist() == [3.0, 4.0]
    y = torch.tanh(torch.tensor([0.3]))
    assert torch.allclose(TF.TanhGrad().forward(T(y, torch.ones(1))), 1 - y * y)
    assert TF.ReluGrad().forward(T(torch.ones(2), torch.tensor([-1.0, 1.0]))).tolist() == [0.0, 1.0]
    # max-pool grad against autograd
    x = torch.randn(1, 4, 4, 2)
    dy = torch.randn(1, 2, 2, 2)
    g = TF.MaxPoolGrad(2, 2, 2, 2, "VALID").forward(T(x, None, dy))
    xx = x.permute(0, 3, 1, 2).clone().requires_grad_(True)
    torch.nn.functional.max_pool2d(xx, 2, 2).backward(dy.permute(0, 3, 1, 2))
    assert torch.allclose(g, xx.grad.permute(0, 2, 3, 1))
    # fused BN grad against autograd
    x = torch.randn(4, 3, 3, 5)
    sc = torch.rand(5) + 0.5
    mean, var = x.mean((0, 1, 2)), x.var((0, 1, 2), unbiased=False)
    dy = torch.randn_like(x)
    dx, dsc, doff = (TF.FusedBatchNormGrad(1e-3).forward(T(dy, x, sc, mean, var))[i] for i in (1, 2, 3))
    xx = x.clone().requires_grad_(True)
    s2 = sc.clone().requires_grad_(True)
    y = (xx - xx.mean((0, 1, 2))) / torch.sqrt(xx.var((0, 1, 2), unbiased=False) + 1e-3) * s2
    y.backward(dy)
    assert torch.allclose(dx, xx.grad, atol=1e-4) and torch.allclose(dsc, s2.grad, atol=1e-4)


def test_resize_bilinear_reference_fixture():
    """S/test/.../nn/ResizeBilinearSpec.scala 'double height' (TF-legacy sampling, NHWC)."""
    x = torch.tensor([[[[1, 2, 3], [4, 5, 6]], [[7, 8, 9], [2, 3, 1]], [[4, 8, 2], [5, 3, 0]]]], dtype=torch.float32)
    assert torch.equal(nn.ResizeBilinear(3, 2, dataFormat="NHWC").forward(x), x)
    out = nn.ResizeBilinear(6, 2, dataFormat="NHWC").forward(x)
    exp = torch.tensor([[[[1, 2, 3], [4, 5, 6]], [[4, 5, 6], [3, 4, 3.5]], [[7, 8, 9], [2, 3, 1]],
                         [[5.5, 8, 5.5], [3.5, 3, 0.5]], [[4, 8, 2], [5, 3, 0]], [[4, 8, 2], [5, 3, 0]]]])
    assert torch.allclose(out, exp)
