"""BigDL Tensor API semantics (reference T/tensor/DenseTensorSpec.scala, DenseTensorMathSpec.scala,
SparseTensorSpec.scala): 1-based dims/indices, in-place math returning self, shared-storage views."""
import numpy as np
import pytest
import torch

from bigdl_amd import nn
from bigdl_amd import tensor as T
from bigdl_amd.tensor import Storage, Tensor


def test_construct_and_index():
    t = Tensor(2, 3)
    assert t.size() == [2, 3] and t.nElement() == 6 and t.dim() == 2
    t.setValue(1, 2, 5.0)
    assert t.valueAt(1, 2) == 5.0 and t(1).valueAt(2) == 5.0
    d = Tensor([1.0, 2.0, 3.0, 4.0, 5.0, 6.0], [2, 3])
    assert d.valueAt(2, 3) == 6.0 and d.size(2) == 3 and d.stride(1) == 3
    assert T.range(1, 5).toArray().tolist() == [1, 2, 3, 4, 5]
    assert sorted(T.randperm(6).toArray().tolist()) == [1, 2, 3, 4, 5, 6]


def test_views_share_storage():
    t = Tensor([[1.0, 2.0, 3.0], [4.0, 5.0, 6.0]])
    n = t.narrow(2, 2, 2)
    assert n.size() == [2, 2] and n.valueAt(1, 1) == 2.0
    n.fill(0.0)
    assert t.toArray().tolist() == [1, 0, 0, 4, 0, 0]
    s = t.select(1, 2)
    s.setValue(1, 9.0)
    assert t.valueAt(2, 1) == 9.0
    tt = t.transpose(1, 2)
    assert tt.size() == [3, 2] and tt.valueAt(1, 2) == 9.0
    assert t.storageOffset() == 1 and n.storageOffset() == 2


def test_storage_set():
    st = Storage([1.0, 2.0, 3.0, 4.0, 5.0, 6.0])
    t = Tensor().set(st, 2, [2, 2], [2, 1])
    assert t.toArray().tolist() == [2, 3, 4, 5]
    st.update(3, 30.0)
    assert t.valueAt(1, 2) == 30.0
    assert st(3) == 30.0 and len(st) == 6


def test_inplace_math():
    x = Tensor([1.0, 2.0, 3.0])
    y = Tensor([10.0, 20.0, 30.0])
    assert x.add(y) is x and x.toArray().tolist() == [11, 22, 33]
    x.add(2.0, y)
    assert x.toArray().tolist() == [31, 62, 93]
    z = Tensor(3).add(x, -1.0, y)
    assert z.toArray().tolist() == [21, 42, 63]
    z.mul(0.5).cmul(Tensor([2.0, 2.0, 2.0]))
    assert z.toArray().tolist() == [21, 42, 63]
    assert z.sum() == 126 and abs(z.mean() - 42) < 1e-6
    assert abs(Tensor([3.0, 4.0]).norm(2) - 5) < 1e-9 and Tensor([1.0, 2.0]).dot(Tensor([3.0, 4.0])) == 11
    m = Tensor(2, 2).addmm(Tensor([[1.0, 2.0], [3.0, 4.0]]), Tensor([[1.0, 0.0], [0.0, 1.0]]))
    assert m.toArray().tolist() == [1, 2, 3, 4]
    m.addmm(0.0, m, 2.0, Tensor([[1.0, 0.0], [0.0, 1.0]]), Tensor([[1.0, 1.0], [1.0, 1.0]]))
    assert m.toArray().tolist() == [2, 2, 2, 2]
    v = Tensor(2).addmv(1.0, Tensor([[1.0, 2.0], [3.0, 4.0]]), Tensor([1.0, 1.0]))
    assert v.toArray().tolist() == [3, 7]
    r = Tensor(2, 2).addr(Tensor([1.0, 2.0]), Tensor([3.0, 4.0]))
    assert r.toArray().tolist() == [3, 4, 6, 8]


def test_reductions_and_indices_are_one_based():
    t = Tensor([[3.0, 1.0, 2.0], [0.0, 5.0, 4.0]])
    v, i = t.max(2)
    assert v.toArray().tolist() == [3, 5] and i.toArray().tolist() == [1, 2]
    v, i = t.min(1)
    assert i.toArray().tolist() == [2, 1, 1]
    assert t.sum(1).size() == [1, 3]
    res, idx = Tensor([5.0, 1.0, 3.0, 2.0]).topk(2)            # increase=True: smallest first
    assert res.toArray().tolist() == [1, 2] and idx.toArray().tolist() == [2, 4]
    res, idx = Tensor([5.0, 1.0, 3.0, 2.0]).topk(2, increase=False)
    assert res.toArray().tolist() == [5, 3] and idx.toArray().tolist() == [1, 3]
    g = Tensor(2, 2).gather(2, Tensor([[1.0, 1.0], [2.0, 1.0]]), Tensor([[1.0, 2.0], [3.0, 4.0]]))
    assert g.toArray().tolist() == [1, 1, 4, 3]
    ix = Tensor(2, 3).index(1, Tensor([2.0, 1.0]), t)
    assert ix.toArray().tolist() == [0, 5, 4, 3, 1, 2]
    s = Tensor(2, 3).zero().scatter(2, Tensor([[3.0], [1.0]]), Tensor([[7.0], [8.0]]))
    assert s.toArray().tolist() == [0, 0, 7, 8, 0, 0]


def test_compare_mask_and_misc():
    x = Tensor([1.0, -2.0, 3.0])
    m = Tensor(3).gt(x, 0.0)
    assert m.toArray().tolist() == [1, 0, 1]
    x.maskedFill(m, 0.0)
    assert x.toArray().tolist() == [0, -2, 0]
    sel = Tensor([1.0, 2.0, 3.0]).maskedSelect(Tensor([1.0, 0.0, 1.0]), Tensor())
    assert sel.toArray().tolist() == [1, 3]
    u, ix = T.unique(Tensor([3.0, 1.0, 3.0, 2.0]))
    assert u.toArray().tolist() == [3, 1, 2] and ix.toArray().tolist() == [1, 2, 1, 3]
    assert Tensor([1.0, 2.0]).almostEqual(Tensor([1.0, 2.0 + 1e-7]), 1e-6)
    x = Tensor(2, 3)
    x.resize(3, 2)
    assert x.size() == [3, 2]
    x.resize(4, 4)
    assert x.nElement() == 16
    c = Tensor([[1.0, 2.0], [3.0, 4.0]]).conv2(Tensor([[1.0, 0.0], [0.0, 1.0]]), "F")
    assert c.size() == [3, 3] and c.valueAt(2, 2) == 5.0


def test_sparse_tensor():
    sp = T.sparse(Tensor([[1.0, 1.0, 2.0], [1.0, 3.0, 2.0]]), Tensor([5.0, 6.0, 7.0]), [2, 3])
    assert sp.nElement() == 3
    assert sp.toDense().toArray().tolist() == [5, 0, 6, 0, 7, 0]
    out = sp.mm(Tensor([[1.0], [1.0], [1.0]]))
    assert out.toArray().tolist() == [11, 7]


def test_modules_accept_bigdl_tensor():
    lin = nn.Linear(3, 2)
    x = Tensor([[1.0, 2.0, 3.0]])
    y = lin.forward(x)
    assert isinstance(y, torch.Tensor) and y.shape == (1, 2)
    g = lin.backward(x, Tensor([[1.0, 1.0]]))
    assert g.shape == (1, 3)
    crit = nn.MSECriterion()
    assert crit.forward(Tensor([1.0, 2.0]), Tensor([1.0, 4.0])) == pytest.approx(2.0)
    assert torch.relu(Tensor([-1.0, 1.0])).tolist() == [0.0, 1.0]
