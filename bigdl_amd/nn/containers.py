"""Containers. Reference: S/nn/Container.scala:40, Sequential.scala:31, Concat.scala:44,
ConcatTable.scala:36, ParallelTable.scala, MapTable.scala, Bottle.scala, DynamicContainer.scala:31.

Dimension arguments are 1-based, as in the reference (``Concat(2)`` concatenates NCHW channels).
"""
import copy

import torch

from ..utils.table import Table
from .abstractnn import AbstractModule, _t_begin, _t_end, activity_apply


def add_activity(a, b):
    """Sum two activities (tensors or tables) — gradient accumulation for fan-out."""
    if a is None:
        return b
    if b is None:
        return a
    if isinstance(a, torch.Tensor):
        if a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.shape == b.shape:
            from .. import ops

            return ops.add_gpu(a, b)
        if a.dtype != b.dtype:  # mixed precision at a graph edge: accumulate in the wider type
            wide = torch.promote_types(a.dtype, b.dtype)
            return a.to(wide) + b.to(wide)
        return a + b
    out = Table()
    for k in set(a.keys()) | set(b.keys()):
        out[k] = add_activity(a.get(k), b.get(k))
    return out


class Container(AbstractModule):
    def __init__(self, *modules):
        super().__init__()
        self.modules = []
        for m in modules:
            self.add(m)

    def add(self, module):
        self.modules.append(module)
        return self

    def modules_list(self):
        return self.modules

    def __len__(self):
        return len(self.modules)

    def get(self, i):
        """1-based access to a child (reference ``modules(i - 1)``)."""
        return self.modules[i - 1]

    # parameters ---------------------------------------------------------------------------------
    def parameters(self):
        ws, gs = [], []
        for m in self.modules:
            p = m.parameters()
            if p is not None:
                ws.extend(p[0])
                gs.extend(p[1])
        return (ws, gs) if ws else None

    def _rebind_into(self, it):
        for m in self.modules:
            m._rebind_into(it)

    def _attach16(self, it, flat16):
        for m in self.modules:
            m._attach16(it, flat16)

    def getParametersTable(self):
        t = Table()
        for m in self.modules:
            for k, v in m.getParametersTable().items():
                t[k] = v
        return t

    def getExtraParameter(self):
        out = []
        for m in self.modules:
            e = m.getExtraParameter()
            if e:
                out.extend(e)
        return out or None

    def setExtraParameter(self, tensors):
        tensors = list(tensors)
        off = 0
        for m in self.modules:
            e = m.getExtraParameter()
            if e:
                m.setExtraParameter(tensors[off:off + len(e)])
                off += len(e)
        return self

    def zeroGradParameters(self):
        for m in self.modules:
            m.zeroGradParameters()

    def training(self):
        super().training()
        for m in self.modules:
            m.training()
        return self

    def evaluate(self, *args, **kw):
        if args or kw:
            return super().evaluate(*args, **kw)
        super().evaluate()
        for m in self.modules:
            m.evaluate()
        return self

    def freeze(self, *names):
        if not names:
            for m in self.modules:
                m.freeze()
            self._frozen = True
        else:
            for m in self.flattened_layers():
                if m.hasName() and m.getName() in names:
                    m.freeze()
        return self

    def unFreeze(self, *names):
        for m in self.flattened_layers():
            if not names or (m.hasName() and m.getName() in names):
                m._frozen = False
        return self

    def to(self, device, memory_format=None):
        super().to(device)
        for m in self.modules:
            m.to(device)
        return self

    def getTimes(self):
        self._resolve_times()
        out = [(self, self.forward_time, self.backward_time)]
        for m in self.modules:
            out.extend(m.getTimes())
        return out

    def resetTimes(self):
        super().resetTimes()
        for m in self.modules:
            m.resetTimes()

    def clearState(self):
        super().clearState()
        for m in self.modules:
            m.clearState()
        return self

    def reset(self):
        for m in self.modules:
            m.reset()

    def __repr__(self):
        inner = "\n".join("  " + repr(m).replace("\n", "\n  ") for m in self.modules)
        return f"{type(self).__name__}{{\n{inner}\n}}"


class Sequential(Container):
    _residual_plan = None   # set by nn.fusion for ResNet blocks on the GPU engine

    def updateOutput(self, input):
        if self._residual_plan is not None:
            from .fusion import residual_forward

            return residual_forward(self, input)
        x = input
        for m in self.modules:
            x = m.forward(x)
        return x

    def backward(self, input, gradOutput):
        t0 = _t_begin(gradOutput)
        if self._residual_plan is not None:
            from .fusion import residual_backward

            self.gradInput = residual_backward(self, input, gradOutput)
            _t_end(self, t0, "backward_time")
            return self.gradInput
        g = gradOutput
        for i in range(len(self.modules) - 1, -1, -1):
            inp = self.modules[i - 1].output if i > 0 else input
            g = self.modules[i].backward(inp, g)
        self.gradInput = g
        _t_end(self, t0, "backward_time")
        return g

    def updateGradInput(self, input, gradOutput):
        g = gradOutput
        for i in range(len(self.modules) - 1, -1, -1):
            inp = self.modules[i - 1].output if i > 0 else input
            g = self.modules[i].updateGradInput(inp, g)
        return g

    def accGradParameters(self, input, gradOutput):
        g = gradOutput
        for i in range(len(self.modules) - 1, -1, -1):
            inp = self.modules[i - 1].output if i > 0 else input
            self.modules[i].accGradParameters(inp, g)
            g = self.modules[i].gradInput


class ConcatTable(Container):
    """Applies every child to the same input; output is a Table (reference ConcatTable.scala:36)."""

    def updateOutput(self, input):
        out = Table()
        for i, m in enumerate(self.modules):
            out[i + 1] = m.forward(input)
        return out

    def backward(self, input, gradOutput):
        gi = None
        for i, m in enumerate(self.modules):
            gi = add_activity(gi, m.backward(input, gradOutput[i + 1]))
        self.gradInput = gi
        return gi

    def updateGradInput(self, input, gradOutput):
        gi = None
        for i, m in enumerate(self.modules):
            gi = add_activity(gi, m.updateGradInput(input, gradOutput[i + 1]))
        return gi

    def accGradParameters(self, input, gradOutput):
        for i, m in enumerate(self.modules):
            m.accGradParameters(input, gradOutput[i + 1])


class Concat(Container):
    """Applies every child to the input and concatenates outputs along 1-based ``dimension``."""

    def __init__(self, dimension, *modules):
        super().__init__(*modules)
        self.dimension = dimension

    def updateOutput(self, input):
        outs = [m.forward(input) for m in self.modules]
        self._sizes = [o.shape[self.dimension - 1] for o in outs]
        out = torch.cat(outs, dim=self.dimension - 1)
        if outs[0].dim() == 4 and outs[0].is_cuda:
            out = out.contiguous(memory_format=torch.channels_last)
        return out

    def _split(self, g):
        return torch.split(g, self._sizes, dim=self.dimension - 1)

    def backward(self, input, gradOutput):
        gi = None
        for m, g in zip(self.modules, self._split(gradOutput)):
            gi = add_activity(gi, m.backward(input, _fmt_like(g)))
        self.gradInput = gi
        return gi

    def updateGradInput(self, input, gradOutput):
        gi = None
        for m, g in zip(self.modules, self._split(gradOutput)):
            gi = add_activity(gi, m.updateGradInput(input, _fmt_like(g)))
        return gi

    def accGradParameters(self, input, gradOutput):
        for m, g in zip(self.modules, self._split(gradOutput)):
            m.accGradParameters(input, _fmt_like(g))


def _fmt_like(g):
    if g.dim() == 4 and g.is_cuda:
        return g.contiguous(memory_format=torch.channels_last)
    return g.contiguous()


class ParallelTable(Container):
    """i-th child applied to the i-th element of the input table."""

    def updateOutput(self, input):
        out = Table()
        for i, m in enumerate(self.modules):
            out[i + 1] = m.forward(input[i + 1])
        return out

    def backward(self, input, gradOutput):
        gi = Table()
        for i, m in enumerate(self.modules):
            gi[i + 1] = m.backward(input[i + 1], gradOutput[i + 1])
        self.gradInput = gi
        return gi

    def updateGradInput(self, input, gradOutput):
        gi = Table()
        for i, m in enumerate(self.modules):
            gi[i + 1] = m.updateGradInput(input[i + 1], gradOutput[i + 1])
        return gi

    def accGradParameters(self, input, gradOutput):
        for i, m in enumerate(self.modules):
            m.accGradParameters(input[i + 1], gradOutput[i + 1])


class MapTable(Container):
    """Applies one module (weights shared across clones) to every element of the input table."""

    def __init__(self, module=None):
        super().__init__()
        if module is not None:
            self.add(module)
        self._clones = []

    def _ensure(self, n):
        base = self.modules[0]
        while len(self._clones) < n:
            c = copy.deepcopy(base) if self._clones else base
            if c is not base:
                _share_params(base, c)
            self._clones.append(c)

    def updateOutput(self, input):
        n = input.length()
        self._ensure(n)
        out = Table()
        for i in range(n):
            out[i + 1] = self._clones[i].forward(input[i + 1])
        return out

    def backward(self, input, gradOutput):
        gi = Table()
        for i in range(input.length()):
            gi[i + 1] = self._clones[i].backward(input[i + 1], gradOutput[i + 1])
        self.gradInput = gi
        return gi

    def updateGradInput(self, input, gradOutput):
        gi = Table()
        for i in range(input.length()):
            gi[i + 1] = self._clones[i].updateGradInput(input[i + 1], gradOutput[i + 1])
        return gi

    def accGradParameters(self, input, gradOutput):
        for i in range(input.length()):
            self._clones[i].accGradParameters(input[i + 1], gradOutput[i + 1])


def _share_params(src, dst):
    for a, b in zip(src.flattened_layers(), dst.flattened_layers()):
        for w, g in a._params:
            setattr(b, w, getattr(a, w))
            setattr(b, g, getattr(a, g))


class Bottle(Container):
    """Applies a module expecting ``nInputDim`` dims to an input with extra leading dims."""

    def __init__(self, module, nInputDim=2, nOutputDim1=None):
        super().__init__(module)
        self.nInputDim = nInputDim
        self.nOutputDim1 = nOutputDim1 if nOutputDim1 is not None else nInputDim

    def updateOutput(self, input):
        self._ishape = input.shape
        lead = input.shape[: input.dim() - self.nInputDim + 1]
        x = input.reshape((-1,) + tuple(input.shape[input.dim() - self.nInputDim + 1:]))
        y = self.modules[0].forward(x)
        self._x = x
        return y.reshape(tuple(lead) + tuple(y.shape[1:]))

    def backward(self, input, gradOutput):
        g = gradOutput.reshape((-1,) + tuple(gradOutput.shape[input.dim() - self.nInputDim + 1:]))
        gi = self.modules[0].backward(self._x, g)
        self.gradInput = gi.reshape(self._ishape)
        return self.gradInput

    def updateGradInput(self, input, gradOutput):
        g = gradOutput.reshape((-1,) + tuple(gradOutput.shape[input.dim() - self.nInputDim + 1:]))
        return self.modules[0].updateGradInput(self._x, g).reshape(self._ishape)

    def accGradParameters(self, input, gradOutput):
        g = gradOutput.reshape((-1,) + tuple(gradOutput.shape[input.dim() - self.nInputDim + 1:]))
        self.modules[0].accGradParameters(self._x, g)


class DynamicContainer(Container):
    pass


__all__ = ["Container", "Sequential", "ConcatTable", "Concat", "ParallelTable", "MapTable", "Bottle",
           "DynamicContainer", "add_activity", "activity_apply"]
