"""Table layers (reference S/nn/*.scala: CAddTable 191, CSubTable, CMulTable, CDivTable, CMaxTable, CMinTable,
CAveTable, JoinTable 194, SplitTable, BifurcateSplitTable, FlattenTable, NarrowTable, SelectTable,
MixtureTable, DenseToSparse, SparseJoinTable). CAddTable (the ResNet residual add) has a native bf16 path
and is fused into the last BatchNorm of the block on the GPU engine (nn/fusion.py)."""
import torch

from .. import ops
from ..utils.table import Table
from .abstractnn import AutogradModule, TensorModule
from .shape_ops import _bdim

BF16 = torch.bfloat16


class CAddTable(TensorModule):
    def __init__(self, inplace=False):
        super().__init__()
        self.inplace = inplace
        self.passthrough = False    # set by nn.fusion when the residual add is folded into a BatchNorm

    def updateOutput(self, input):
        if self.passthrough:   # the sum was produced in place by input[_pass_index]'s producer
            return input[getattr(self, "_pass_index", 1)]
        ts = input.toSeq()
        out = ts[0]
        for t in ts[1:]:
            if out.is_cuda and out.dtype == BF16 and t.dtype == BF16 and out.shape == t.shape:
                out = ops.add_gpu(out, t)
            else:
                out = out + t
        return out

    def updateGradInput(self, input, gradOutput):
        gi = Table()
        for i in range(1, input.length() + 1):
            t = input[i]
            g = gradOutput
            if t.shape != g.shape:  # broadcast add
                g = _reduce_to(g, t.shape)
            gi[i] = g
        return gi


def _reduce_to(g, shape):
    while g.dim() > len(shape):
        g = g.sum(0)
    for i, s in enumerate(shape):
        if s == 1 and g.shape[i] != 1:
            g = g.sum(i, keepdim=True)
    return g


class CSubTable(AutogradModule):
    def fn(self, x):
        return x[1] - x[2]


class CMulTable(AutogradModule):
    def fn(self, x):
        out = x[1]
        for t in x.toSeq()[1:]:
            out = out * t
        return out


class CDivTable(AutogradModule):
    def fn(self, x):
        return x[1] / x[2]


class CMaxTable(AutogradModule):
    def fn(self, x):
        out = x[1]
        for t in x.toSeq()[1:]:
            out = torch.maximum(out, t)
        return out


class CMinTable(AutogradModule):
    def fn(self, x):
        out = x[1]
        for t in x.toSeq()[1:]:
            out = torch.minimum(out, t)
        return out


class CAveTable(AutogradModule):
    def __init__(self, inplace=False):
        super().__init__()

    def fn(self, x):
        ts = x.toSeq()
        return sum(ts) / len(ts)


class JoinTable(TensorModule):
    """Concatenate the tensors of the input table along 1-based ``dimension``."""

    def __init__(self, dimension, nInputDims=-1):
        super().__init__()
        self.dimension, self.nInputDims = dimension, nInputDims

    def updateOutput(self, input):
        ts = input.toSeq()
        d = _bdim(self.dimension, ts[0], self.nInputDims if self.nInputDims > 0 else None)
        self._d = d
        self._sizes = [t.shape[d] for t in ts]
        buf = getattr(self, "_fuse_buf", None)
        if buf is not None:
            # concat written in place (nn.fusion.fuse_graph_for_inference): producers already wrote their channel
            # slices of ``buf``; inputs that did not (e.g. a pooling branch) are copied into theirs
            self._fuse_buf = None
            off = 0
            for t in ts:
                sl = buf.narrow(d, off, t.shape[d])
                if t.data_ptr() != sl.data_ptr() or t.stride() != sl.stride():
                    sl.copy_(t)
                off += t.shape[d]
            return buf
        out = torch.cat(ts, dim=d)
        if out.is_cuda and out.dim() == 4:
            out = out.contiguous(memory_format=torch.channels_last)
        return out

    def updateGradInput(self, input, gradOutput):
        gi = Table()
        for i, g in enumerate(torch.split(gradOutput, self._sizes, dim=self._d)):
            if g.is_cuda and g.dim() == 4:
                g = g.contiguous(memory_format=torch.channels_last)
            gi[i + 1] = g.contiguous() if not g.is_cuda else g
        return gi


class SplitTable(TensorModule):
    def __init__(self, dimension, nInputDims=-1):
        super().__init__()
        self.dimension, self.nInputDims = dimension, nInputDims

    def updateOutput(self, input):
        d = _bdim(self.dimension, input, self.nInputDims if self.nInputDims > 0 else None)
        self._d = d
        out = Table()
        for i, t in enumerate(torch.unbind(input, d)):
            out[i + 1] = t
        return out

    def updateGradInput(self, input, gradOutput):
        return torch.stack(gradOutput.toSeq(), dim=self._d)


class BifurcateSplitTable(TensorModule):
    def __init__(self, dimension):
        super().__init__()
        self.dimension = dimension

    def updateOutput(self, input):
        d = self.dimension - 1
        n = input.shape[d]
        a, b = torch.split(input, [n // 2, n - n // 2], dim=d)
        return Table(a, b)

    def updateGradInput(self, input, gradOutput):
        return torch.cat([gradOutput[1], gradOutput[2]], dim=self.dimension - 1)


class FlattenTable(TensorModule):
    def updateOutput(self, input):
        out = Table()
        self._struct = []

        def rec(t, path):
            if isinstance(t, Table):
                for k in range(1, t.length() + 1):
                    rec(t[k], path + [k])
            else:
                out.insert(t)
                self._struct.append(path)

        rec(input, [])
        return out

    def updateGradInput(self, input, gradOutput):
        def build(t, prefix):
            if isinstance(t, Table):
                r = Table()
                for k in range(1, t.length() + 1):
                    r[k] = build(t[k], prefix + [k])
                return r
            return gradOutput[self._struct.index(prefix) + 1]

        return build(input, [])


class NarrowTable(TensorModule):
    def __init__(self, offset, length=1):
        super().__init__()
        self.offset, self.length = offset, length

    def updateOutput(self, input):
        n = self.length if self.length > 0 else input.length() - self.offset + self.length + 2
        out = Table()
        for i in range(n):
            out[i + 1] = input[self.offset + i]
        self._n = n
        return out

    def updateGradInput(self, input, gradOutput):
        gi = Table()
        for i in range(1, input.length() + 1):
            k = i - self.offset + 1
            gi[i] = gradOutput[k] if 1 <= k <= self._n else torch.zeros_like(input[i])
        return gi


class SelectTable(TensorModule):
    def __init__(self, index):
        super().__init__()
        self.index = index

    def _i(self, input):
        return self.index if self.index > 0 else input.length() + self.index + 1

    def updateOutput(self, input):
        return input[self._i(input)]

    def updateGradInput(self, input, gradOutput):
        gi = Table()
        k = self._i(input)
        for i in range(1, input.length() + 1):
            gi[i] = gradOutput if i == k else _zeros_like_act(input[i])
        return gi


def _zeros_like_act(a):
    if isinstance(a, torch.Tensor):
        return torch.zeros_like(a)
    t = Table()
    for k, v in a.items():
        t[k] = _zeros_like_act(v)
    return t


class MixtureTable(AutogradModule):
    """Table(gater (B, n), experts Table or tensor (B, n, ...)) -> gated sum of experts."""

    def __init__(self, dim=None):
        super().__init__()
        self.dim = dim

    def fn(self, x):
        gate, experts = x[1], x[2]
        if isinstance(experts, torch.Tensor):
            d = (self.dim - 1) if self.dim else 1
            g = gate.view(gate.shape + (1,) * (experts.dim() - gate.dim()))
            return (experts * g).sum(d)
        ts = experts.toSeq()
        out = 0
        for i, e in enumerate(ts):
            out = out + e * gate[:, i].view((-1,) + (1,) * (e.dim() - 1))
        return out


class DenseToSparse(TensorModule):
    def __init__(self, propagateBack=True):
        super().__init__()

    def updateOutput(self, input):
        return input.to_sparse()

    def updateGradInput(self, input, gradOutput):
        return gradOutput.to_dense() if gradOutput.is_sparse else gradOutput


class SparseJoinTable(TensorModule):
    def __init__(self, dimension):
        super().__init__()
        self.dimension = dimension

    def updateOutput(self, input):
        return torch.cat([t.to_dense() for t in input.toSeq()], dim=self.dimension - 1).to_sparse()

    def updateGradInput(self, input, gradOutput):
        return None


__all__ = ["CAddTable", "CSubTable", "CMulTable", "CDivTable", "CMaxTable", "CMinTable", "CAveTable", "JoinTable",
           "SplitTable", "BifurcateSplitTable", "FlattenTable", "NarrowTable", "SelectTable", "MixtureTable",
           "DenseToSparse", "SparseJoinTable"]
