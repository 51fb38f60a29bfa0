"""TensorFlow-graph modules: constants, control flow, state, TensorArray/Stack data flow, parsing and image
decode ops, and the gradient ops a TF training graph contains.

Reference: S/nn/tf/ControlOps.scala:33-330 (SwitchOps, MergeOps, Enter, Exit, NextIteration, LoopCondition,
ControlNodes.switch/merge/whileLoop), ControlDependency.scala, ArrayOps.scala (Const, InvertPermutation,
ConcatOffset, Fill, BroadcastGradientArgs), Assert.scala, NoOp.scala, StateOps.scala (Variable, Assign,
AssignGrad), DataFlowOps.scala (TensorArray*, Stack*), ParsingOps.scala (ParseExample, ParseSingleExample),
ImageOps.scala (DecodeJpeg/Png/Bmp/Gif/Raw), MathOps.scala / NNOps.scala (Sqrt/Rsqrt/activation/pool/LRN/BN/
BiasAdd/conv gradient ops), SplitAndSelect.scala, TensorModuleWrapper.scala, BiasAdd.scala, Log1p.scala.

Control-flow semantics follow the reference: a Switch outputs ``Table(data, None)`` when its condition is false
and ``Table(None, data)`` when true; successors hang off slot 1 (false edge) or slot 2 (true edge) and only the
taken side is scheduled (nn/scheduler.py). ``ControlNodes.whileLoop`` exits when the condition is TRUE, like the
reference builder (the loop runs while ``condition`` is false).
"""
import io
import math

import torch
import torch.nn.functional as F

from ..utils.table import Table
from .abstractnn import AbstractModule, AutogradModule, TensorModule
from .ops import Operation


def is_random(m):
    """Modules that must re-run even when fed only by constants (reference Scheduler RandomNode)."""
    return bool(getattr(m, "_random_node", False))


# ---------------------------------------------------------------------------------------------- constants
class Const(Operation):
    """A constant tensor with no inputs (ArrayOps.scala Const)."""

    def __init__(self, value):
        super().__init__()
        self.value = value if isinstance(value, torch.Tensor) else torch.as_tensor(value)
        self._buffers = ["value"]

    def updateOutput(self, input):
        return self.value


class Fill(Operation):
    """Table(shape, scalar) -> tensor of ``shape`` filled with ``scalar``."""

    def updateOutput(self, input):
        shape, v = input[1], input[2]
        return torch.full([int(s) for s in shape.reshape(-1).tolist()], v.reshape(-1)[0].item(), dtype=v.dtype,
                          device=v.device)


class InvertPermutation(Operation):
    def updateOutput(self, input):
        p = input.reshape(-1).long()
        out = torch.empty_like(p)
        out[p] = torch.arange(p.numel(), device=p.device)
        return out.to(input.dtype)


class ConcatOffset(Operation):
    """Table(axis, shape1, shape2, ...) -> Table of the offsets of each input inside the concatenation."""

    def updateOutput(self, input):
        axis = int(input[1].reshape(-1)[0])
        shapes = [input[i] for i in range(2, input.length() + 1)]
        out, off = Table(), 0
        for i, s in enumerate(shapes):
            o = torch.zeros_like(s)
            o[axis] = off
            off += int(s[axis])
            out[i + 1] = o
        return out


class BroadcastGradientArgs(Operation):
    """Table(shape0, shape1) -> Table(reduction axes for grad0, for grad1) under numpy broadcasting."""

    def updateOutput(self, input):
        s0 = [int(v) for v in input[1].reshape(-1).tolist()]
        s1 = [int(v) for v in input[2].reshape(-1).tolist()]
        n = max(len(s0), len(s1))
        a = [1] * (n - len(s0)) + s0
        b = [1] * (n - len(s1)) + s1
        r0 = [i for i in range(n) if a[i] == 1 and b[i] != 1]
        r1 = [i for i in range(n) if b[i] == 1 and a[i] != 1]
        return Table(torch.tensor(r0, dtype=torch.int32), torch.tensor(r1, dtype=torch.int32))


class Shape(Operation):
    def updateOutput(self, input):
        return torch.tensor(list(input.shape), dtype=torch.int32)


class NoOp(Operation):
    def updateOutput(self, input):
        return Table()


class Assert(Operation):
    """Table(condition, data...) -> raises with ``message`` (or the data) when the condition is false."""

    def __init__(self, message=""):
        super().__init__()
        self.message = message

    def updateOutput(self, input):
        cond = input[1] if isinstance(input, Table) else input
        if not bool(torch.as_tensor(cond).reshape(-1)[0]):
            data = [input[i] for i in range(2, input.length() + 1)] if isinstance(input, Table) else []
            raise AssertionError(self.message or f"assertion failed: {data}")
        return Table()


class ControlDependency(Operation):
    """Ordering-only edge holder; the scheduler routes it without executing (ControlDependency.scala)."""

    def updateOutput(self, input):
        return Table()


# ---------------------------------------------------------------------------------------------- control flow
class ControlOps(Operation):
    def updateGradInput(self, input, gradOutput):
        raise RuntimeError(f"{type(self).__name__}: control-flow ops have no backward")


class IdentityControl(ControlOps):
    def updateOutput(self, input):
        return input


class SwitchOps(ControlOps):
    """Table(data, condition) -> Table(data, None) if condition is false else Table(None, data)."""

    def updateOutput(self, input):
        data, cond = input[1], input[2]
        t = Table()
        if bool(torch.as_tensor(cond).reshape(-1)[0]):
            t[1], t[2] = None, data
        else:
            t[1], t[2] = data, None
        return t


class MergeOps(ControlOps):
    """Forwards the input that arrived (the scheduler sets which one with ``setSwitch``)."""

    def __init__(self, switch=1):
        super().__init__()
        self.switch = switch

    def setSwitch(self, s):
        self.switch = s
        return self

    def updateOutput(self, input):
        return input[self.switch] if isinstance(input, Table) else input


class Enter(IdentityControl):
    def __init__(self, frame):
        super().__init__()
        self.frame = frame


class Exit(IdentityControl):
    pass


class NextIteration(ControlOps):
    def updateOutput(self, input):
        return input.clone() if isinstance(input, torch.Tensor) else input


class LoopCondition(IdentityControl):
    def continue_(self):
        t = self.output
        if not isinstance(t, torch.Tensor) or t.numel() != 1:
            raise RuntimeError("loop condition result should be a one-element boolean tensor")
        return bool(t.reshape(-1)[0])


class ControlNodes:
    """Graph builders for control flow (ControlOps.scala:235-330)."""

    @staticmethod
    def switch(data, condition):
        """Switch node; route with ``(node, 2)`` (true edge) / ``(node, 1)`` (false edge) in ``inputs``.
        The reference's argument naming is kept: ``condition`` supplies slot 1 (the routed data) and
        ``data`` slot 2 (the predicate)."""
        node = SwitchOps().inputs()
        condition.add_next(node)
        data.add_next(node)
        return node

    @staticmethod
    def merge(*nodes):
        node = MergeOps().inputs()
        for n in nodes:
            if isinstance(n, tuple):
                n[0].add_next(node, n[1])
            else:
                n.add_next(node)
        return node

    @staticmethod
    def whileLoop(condition, body, loopVars, name=None):
        """``condition = (cond_inputs, cond_output)``, ``body = [(body_input, body_output), ...]``,
        ``loopVars`` = initial-value nodes. Returns the Exit nodes, one per loop variable."""
        cond_inputs, cond_out = condition
        lc = LoopCondition().inputs(cond_out)
        if name:
            lc.element.setName(f"{name}/loopCondition")
        exits = []
        for i, ((inp, cin), (bin_, bout)) in enumerate(zip(zip(loopVars, cond_inputs), body), start=1):
            enter = Enter("test_frame").inputs(inp)
            merge = ControlNodes.merge(enter)
            merge.add_next(cin)
            sw = ControlNodes.switch(lc, merge)
            ex = Exit().inputs((sw, 2))
            ident = _identity().inputs((sw, 1))
            ident.add_next(bin_)
            nxt = NextIteration().inputs(bout)
            nxt.add_next(merge)
            if name:
                for n, tag in ((enter, "enter"), (merge, "merge"), (sw, "switch"), (ex, "exit"),
                               (ident, "switchFalse"), (nxt, "nextIteration")):
                    n.element.setName(f"{name}/{tag}{i}")
            exits.append(ex)
        return exits


def _identity():
    from .activation import Identity
    return Identity()


# ---------------------------------------------------------------------------------------------- state
class Variable(AbstractModule):
    """A trainable tensor produced by a graph node (StateOps.scala Variable): forward outputs the value,
    backward accumulates gradOutput into its gradient."""

    def __init__(self, variableValue, variableGradient=None):
        super().__init__()
        self.register_parameter("weight", "gradWeight", variableValue)
        if variableGradient is not None:
            self.gradWeight = variableGradient

    def updateOutput(self, input):
        return self.weight

    def updateGradInput(self, input, gradOutput):
        return None

    def accGradParameters(self, input, gradOutput):
        self.gradWeight.add_(gradOutput.to(self.gradWeight.dtype))


class Assign(Operation):
    """Table(ref, value) -> ref after copying value into it (shape change allowed unless validateShape)."""

    def __init__(self, validateShape=True, useLocking=True):
        super().__init__()
        self.validateShape = validateShape

    def updateOutput(self, input):
        ref, value = input[1], input[2]
        if self.validateShape and tuple(ref.shape) != tuple(value.shape):
            raise ValueError(f"Assign: shape mismatch {tuple(ref.shape)} vs {tuple(value.shape)}")
        if tuple(ref.shape) != tuple(value.shape):
            ref.resize_(value.shape)
        with torch.no_grad():
            ref.copy_(value)
        return ref


class AssignGrad(Operation):
    """Writes its input into a gradient buffer (StateOps.scala AssignGrad)."""

    def __init__(self, buffer):
        super().__init__()
        self.buffer = buffer

    def updateOutput(self, input):
        with torch.no_grad():
            self.buffer.copy_(input)
        return Table()


# ---------------------------------------------------------------------------------------------- TensorArray / Stack
_RESOURCES = {}


def _handle(t):
    return t if isinstance(t, str) else (t.item() if isinstance(t, torch.Tensor) and t.numel() == 1 else str(t))


class _TensorArray:
    def __init__(self, size, dynamic, clear_after_read, element_shape=None):
        self.items = [None] * size
        self.dynamic = dynamic
        self.clear_after_read = clear_after_read
        self.element_shape = element_shape

    def write(self, i, t):
        if i >= len(self.items):
            if not self.dynamic:
                raise IndexError(f"TensorArray index {i} out of range {len(self.items)}")
            self.items.extend([None] * (i + 1 - len(self.items)))
        self.items[i] = t

    def read(self, i):
        t = self.items[i]
        if t is None:
            raise RuntimeError(f"TensorArray element {i} was not written")
        if self.clear_after_read:
            self.items[i] = None
        return t


class TensorArrayCreator(Operation):
    """size tensor -> Table(handle, flow). ``handle`` names the array in the resource registry."""

    _counter = 0

    def __init__(self, dynamicSize=False, clearAfterRead=True, identicalElementShapes=False, tensorArrayName=""):
        super().__init__()
        self.dynamicSize = dynamicSize
        self.clearAfterRead = clearAfterRead
        self.tensorArrayName = tensorArrayName

    def updateOutput(self, input):
        TensorArrayCreator._counter += 1
        name = f"{self.tensorArrayName or self.getName()}#{TensorArrayCreator._counter}"
        _RESOURCES[name] = _TensorArray(int(input.reshape(-1)[0]), self.dynamicSize, self.clearAfterRead)
        return Table(name, torch.zeros(1))

    def release(self):
        for k in [k for k in _RESOURCES if k.startswith(f"{self.tensorArrayName or self.getName()}#")]:
            del _RESOURCES[k]


class TensorArrayGrad(Operation):
    def __init__(self, source):
        super().__init__()
        self.source = source

    def updateOutput(self, input):
        h = _handle(input[1])
        g = f"{h}@grad:{self.source}"
        if g not in _RESOURCES:
            ta = _RESOURCES[h]
            _RESOURCES[g] = _TensorArray(len(ta.items), True, True)
        return Table(g, torch.zeros(1))


class TensorArrayWrite(Operation):
    """Table(handle, index, value, flow) -> flow."""

    def updateOutput(self, input):
        _RESOURCES[_handle(input[1])].write(int(input[2].reshape(-1)[0]), input[3])
        return input[4] if input.length() >= 4 else torch.zeros(1)


class TensorArrayRead(Operation):
    """Table(handle, index, flow) -> element."""

    def updateOutput(self, input):
        return _RESOURCES[_handle(input[1])].read(int(input[2].reshape(-1)[0]))


class TensorArrayGather(Operation):
    """Table(handle, indices, flow) -> stacked elements."""

    def updateOutput(self, input):
        ta = _RESOURCES[_handle(input[1])]
        return torch.stack([ta.read(int(i)) for i in input[2].reshape(-1).tolist()])


class TensorArrayScatter(Operation):
    """Table(handle, indices, value, flow) -> flow."""

    def updateOutput(self, input):
        ta = _RESOURCES[_handle(input[1])]
        for k, i in enumerate(input[2].reshape(-1).tolist()):
            ta.write(int(i), input[3][k])
        return input[4] if input.length() >= 4 else torch.zeros(1)


class TensorArrayConcat(Operation):
    """Table(handle, flow) -> Table(concatenation along dim 0, lengths)."""

    def updateOutput(self, input):
        ta = _RESOURCES[_handle(input[1])]
        items = [ta.read(i) for i in range(len(ta.items))]
        return Table(torch.cat(items, 0), torch.tensor([t.shape[0] for t in items], dtype=torch.int64))


class TensorArraySplit(Operation):
    """Table(handle, value, lengths, flow) -> flow."""

    def updateOutput(self, input):
        ta = _RESOURCES[_handle(input[1])]
        for i, piece in enumerate(torch.split(input[2], [int(v) for v in input[3].reshape(-1).tolist()], 0)):
            ta.write(i, piece)
        return input[4] if input.length() >= 4 else torch.zeros(1)


class TensorArraySize(Operation):
    def updateOutput(self, input):
        return torch.tensor(len(_RESOURCES[_handle(input[1])].items), dtype=torch.int32)


class TensorArrayClose(Operation):
    def updateOutput(self, input):
        _RESOURCES.pop(_handle(input[1] if isinstance(input, Table) else input), None)
        return Table()


class StackCreator(Operation):
    _counter = 0

    def __init__(self, elemType=None, stackName=""):
        super().__init__()
        self.stackName = stackName

    def updateOutput(self, input):
        StackCreator._counter += 1
        name = f"{self.stackName or self.getName()}#stack{StackCreator._counter}"
        _RESOURCES[name] = []
        return name


class StackPush(Operation):
    """Table(handle, value) -> value."""

    def __init__(self, swapMemory=False):
        super().__init__()

    def updateOutput(self, input):
        _RESOURCES[_handle(input[1])].append(input[2])
        return input[2]


class StackPop(Operation):
    def updateOutput(self, input):
        return _RESOURCES[_handle(input)].pop()


Stack = StackCreator


# ---------------------------------------------------------------------------------------------- parsing
def _unpack_varints(b):
    from ..utils import pbwire

    out, pos = [], 0
    while pos < len(b):
        v, pos = pbwire.read_varint(b, pos)
        out.append(v - (1 << 64) if v >= 1 << 63 else v)
    return out


def _parse_example_proto(buf):
    """tf.train.Example bytes -> {key: ('bytes'|'float'|'int64', list)} (Example{features=1}; Features{map<string,
    Feature> feature=1}; Feature{bytes_list=1, float_list=2, int64_list=3}; each list's values are field 1)."""
    import struct

    from ..utils import pbwire

    out = {}
    for feats in pbwire.Msg(buf).raw(1):
        for entry in pbwire.Msg(feats).raw(1):
            em = pbwire.Msg(entry)
            key = em.str(1)
            fm = pbwire.Msg(em.raw(2)[-1] if em.has(2) else b"")
            for kind in (1, 2, 3):
                if not fm.has(kind):
                    continue
                vals = []
                for wire, v in pbwire.parse(fm.raw(kind)[-1]).get(1, []):
                    if kind == 1:
                        vals.append(v)
                    elif kind == 2:
                        vals.extend(struct.unpack(f"<{len(v) // 4}f", v))
                    elif wire == pbwire.VARINT:
                        vals.append(v - (1 << 64) if v >= 1 << 63 else v)
                    else:
                        vals.extend(_unpack_varints(v))
                out[key] = ({1: "bytes", 2: "float", 3: "int64"}[kind], vals)
    return out


def encode_example(features):
    """{key: list[float] | list[int] | list[bytes]} -> tf.train.Example bytes (test helper / TFRecord writers)."""
    from ..utils import pbwire

    fmap = b""
    for k, vals in features.items():
        if vals and isinstance(vals[0], (bytes, bytearray)):
            feat = pbwire.f_bytes(1, b"".join(pbwire.f_bytes(1, bytes(v)) for v in vals))
        elif vals and isinstance(vals[0], float):
            feat = pbwire.f_bytes(2, pbwire.f_packed_floats(1, vals))
        else:
            feat = pbwire.f_bytes(3, pbwire.f_packed_varints(1, vals))
        fmap += pbwire.f_bytes(1, pbwire.f_bytes(1, k) + pbwire.f_bytes(2, feat))
    return pbwire.f_bytes(1, fmap)


_KIND_DTYPE = {"float": torch.float32, "int64": torch.int64}


class ParseExample(Operation):
    """Table(serialized[batch], names, dense_keys..., dense_defaults...) -> Table of dense tensors
    ``[batch, *shape]`` (ParsingOps.scala ParseExample; dense features only, like the reference)."""

    def __init__(self, nDense, tDense, denseShape):
        super().__init__()
        self.nDense = nDense
        self.tDense = list(tDense)
        self.denseShape = [list(s) for s in denseShape]

    def updateOutput(self, input):
        serialized = input[1]
        records = list(serialized) if isinstance(serialized, (list, tuple)) else [serialized]
        keys = [input[3 + i] for i in range(self.nDense)]
        keys = [k if isinstance(k, str) else bytes(k).decode() for k in keys]
        defaults = [input[3 + self.nDense + i] if input.length() >= 3 + self.nDense + i else None
                    for i in range(self.nDense)]
        parsed = [_parse_example_proto(r) for r in records]
        out = Table()
        for i, k in enumerate(keys):
            rows = []
            for p in parsed:
                if k in p:
                    kind, vals = p[k]
                    rows.append(torch.tensor(vals, dtype=_KIND_DTYPE.get(kind, torch.float32)) if kind != "bytes"
                                else vals)
                elif defaults[i] is not None:
                    rows.append(defaults[i])
                else:
                    raise KeyError(f"ParseExample: feature {k} missing and no default")
            if rows and isinstance(rows[0], list):
                out[i + 1] = rows
            else:
                dt = self.tDense[i] if isinstance(self.tDense[i], torch.dtype) else rows[0].dtype
                out[i + 1] = torch.stack([r.to(dt).reshape(self.denseShape[i]) for r in rows])
        return out


class ParseSingleExample(ParseExample):
    """One serialized Example -> Table of dense tensors shaped ``denseShape`` (no batch dim)."""

    def updateOutput(self, input):
        out = super().updateOutput(input)
        for i in range(1, out.length() + 1):
            if isinstance(out[i], torch.Tensor):
                out[i] = out[i][0]
        return out


# ---------------------------------------------------------------------------------------------- images
class DecodeImage(Operation):
    """Encoded image bytes -> uint8 HWC tensor (ImageOps.scala; PIL replaces the JVM ImageIO decoders)."""

    def __init__(self, channels=3):
        super().__init__()
        self.channels = channels

    def _decode(self, data):
        from PIL import Image

        img = Image.open(io.BytesIO(bytes(data)))
        mode = {1: "L", 3: "RGB", 4: "RGBA"}.get(self.channels)
        if mode is not None:
            img = img.convert(mode)
        import numpy as np

        a = torch.from_numpy(np.asarray(img).copy())
        return a.unsqueeze(-1) if a.dim() == 2 else a

    def updateOutput(self, input):
        data = input if isinstance(input, (bytes, bytearray)) else bytes(input.to(torch.uint8).tolist()) \
            if isinstance(input, torch.Tensor) else input
        return self._decode(data)


class DecodeJpeg(DecodeImage):
    def __init__(self, channels=3, ratio=1):
        super().__init__(channels)
        self.ratio = ratio

    def _decode(self, data):
        t = super()._decode(data)
        if self.ratio > 1:
            t = t[::self.ratio, ::self.ratio]
        return t


class DecodePng(DecodeImage):
    pass


class DecodeBmp(DecodeImage):
    pass


class DecodeGif(DecodeImage):
    """GIF -> uint8 [frames, H, W, 3]."""

    def _decode(self, data):
        from PIL import Image, ImageSequence
        import numpy as np

        img = Image.open(io.BytesIO(bytes(data)))
        frames = [torch.from_numpy(np.asarray(f.convert("RGB")).copy()) for f in ImageSequence.Iterator(img)]
        return torch.stack(frames)


class DecodeRaw(Operation):
    """Raw bytes -> 1-D tensor of ``outType`` (little endian unless ``littleEndian=False``)."""

    def __init__(self, outType=torch.uint8, littleEndian=True):
        super().__init__()
        self.outType = outType
        self.littleEndian = littleEndian

    def updateOutput(self, input):
        import numpy as np

        data = bytes(input) if not isinstance(input, torch.Tensor) else bytes(input.to(torch.uint8).tolist())
        np_dt = np.dtype(torch.empty(0, dtype=self.outType).numpy().dtype).newbyteorder("<" if self.littleEndian else ">")
        return torch.from_numpy(np.frombuffer(data, dtype=np_dt).astype(np_dt.newbyteorder("=")).copy())


# ---------------------------------------------------------------------------------------------- misc modules
class BiasAdd(AutogradModule):
    """Table(value, bias) -> value + bias over the last dim (nn/tf/BiasAdd.scala)."""

    def fn(self, x):
        return x[1] + x[2]


class Log1p(AutogradModule):
    def fn(self, x):
        return torch.log1p(x)


class SplitAndSelect(AutogradModule):
    """Split ``dimension`` (1-based) into ``numSplit`` equal parts and output part ``index`` (1-based)."""

    def __init__(self, dimension, index, numSplit):
        super().__init__()
        self.dimension, self.index, self.numSplit = dimension, index, numSplit

    def fn(self, x):
        return torch.chunk(x, self.numSplit, self.dimension - 1)[self.index - 1]


class StridedSlice(AutogradModule):
    """Static strided slice: ``sliceSpecs`` = [(dim(1-based), begin(1-based), end(exclusive), stride)]."""

    def __init__(self, sliceSpecs):
        super().__init__()
        self.sliceSpecs = [tuple(s) for s in sliceSpecs]

    def fn(self, x):
        idx = [slice(None)] * x.dim()
        for d, b, e, s in self.sliceSpecs:
            idx[d - 1] = slice(b - 1, e - 1, s)
        return x[tuple(idx)]


class TensorModuleWrapper(Operation):
    """Runs a TensorModule as a forward-only operation (TensorModuleWrapper.scala)."""

    def __init__(self, module):
        super().__init__()
        self.module = module

    def updateOutput(self, input):
        return self.module.forward(input)


# ---------------------------------------------------------------------------------------------- gradient ops
def _autograd_grad(fn, x, dy):
    x = x.detach().requires_grad_(True)
    with torch.enable_grad():
        y = fn(x)
        (g,) = torch.autograd.grad(y, x, dy)
    return g


class UnaryGrad(Operation):
    """Table(y or x, dy) -> dx for an element-wise op, as the TF *Grad ops define it."""

    def grad(self, a, dy):
        raise NotImplementedError

    def updateOutput(self, input):
        return self.grad(input[1], input[2])


class SqrtGrad(UnaryGrad):       # a = y = sqrt(x)
    def grad(self, y, dy):
        return dy * 0.5 / y


class RsqrtGrad(UnaryGrad):      # a = y = rsqrt(x)
    def grad(self, y, dy):
        return dy * -0.5 * y * y * y


class TanhGrad(UnaryGrad):       # a = y
    def grad(self, y, dy):
        return dy * (1 - y * y)


class SigmoidGrad(UnaryGrad):    # a = y
    def grad(self, y, dy):
        return dy * y * (1 - y)


class ReluGrad(UnaryGrad):       # TF order: (gradients, features)
    def updateOutput(self, input):
        return input[1] * (input[2] > 0).to(input[1].dtype)


class Relu6Grad(UnaryGrad):
    def updateOutput(self, input):
        x = input[2]
        return input[1] * ((x > 0) & (x < 6)).to(input[1].dtype)


class EluGrad(UnaryGrad):        # (gradients, outputs)
    def updateOutput(self, input):
        dy, y = input[1], input[2]
        return torch.where(y > 0, dy, dy * (y + 1))


class SoftplusGrad(UnaryGrad):   # (gradients, features)
    def updateOutput(self, input):
        return input[1] * torch.sigmoid(input[2])


class SoftsignGrad(UnaryGrad):
    def updateOutput(self, input):
        x = input[2]
        return input[1] / (1 + x.abs()) ** 2


class BiasAddGrad(Operation):
    def __init__(self, dataFormat="NHWC"):
        super().__init__()
        self.dataFormat = dataFormat

    def updateOutput(self, input):
        if self.dataFormat == "NCHW" and input.dim() >= 3:
            return input.sum(dim=[d for d in range(input.dim()) if d != 1])
        return input.reshape(-1, input.shape[-1]).sum(0)


def _nchw(x, fmt):
    return x.permute(0, 3, 1, 2) if fmt == "NHWC" else x


def _back(x, fmt):
    return x.permute(0, 2, 3, 1) if fmt == "NHWC" else x


def _tf_pads(n, k, s, same):
    if not same:
        return 0, 0
    out = -(-n // s)
    tot = max((out - 1) * s + k - n, 0)
    return tot // 2, tot - tot // 2


class MaxPoolGrad(Operation):
    """Table(orig_input, orig_output, grad) -> grad wrt orig_input."""

    def __init__(self, kH, kW, strideH, strideW, padding="VALID", dataFormat="NHWC"):
        super().__init__()
        self.k, self.s, self.same, self.fmt = (kH, kW), (strideH, strideW), padding == "SAME", dataFormat

    def updateOutput(self, input):
        x = _nchw(input[1], self.fmt)
        ph = _tf_pads(x.shape[2], self.k[0], self.s[0], self.same)
        pw = _tf_pads(x.shape[3], self.k[1], self.s[1], self.same)

        def f(t):
            if t.is_cuda:
                from .tf_ops import tf_pool2d

                return tf_pool2d(t, "max", self.k, self.s, self.same)
            t = F.pad(t, (pw[0], pw[1], ph[0], ph[1]), value=-math.inf)
            return F.max_pool2d(t, self.k, self.s)
        return _back(_autograd_grad(f, x.float(), _nchw(input[3], self.fmt).float()), self.fmt)


class AvgPoolGrad(Operation):
    """Table(orig_input_shape, grad) -> grad wrt the input (VALID/SAME, count excludes padding like TF)."""

    def __init__(self, kH, kW, strideH, strideW, padding="VALID", dataFormat="NHWC"):
        super().__init__()
        self.k, self.s, self.same, self.fmt = (kH, kW), (strideH, strideW), padding == "SAME", dataFormat

    def updateOutput(self, input):
        shape = [int(v) for v in input[1].reshape(-1).tolist()]
        x = _nchw(torch.zeros(shape, device=input[2].device), self.fmt)
        ph = _tf_pads(x.shape[2], self.k[0], self.s[0], self.same)
        pw = _tf_pads(x.shape[3], self.k[1], self.s[1], self.same)

        def f(t):
            if t.is_cuda:
                from .tf_ops import tf_pool2d

                return tf_pool2d(t, "avg", self.k, self.s, self.same)
            ones = F.pad(torch.ones_like(t), (pw[0], pw[1], ph[0], ph[1]))
            t = F.pad(t, (pw[0], pw[1], ph[0], ph[1]))
            return F.avg_pool2d(t, self.k, self.s) / F.avg_pool2d(ones, self.k, self.s)
        return _back(_autograd_grad(f, x, _nchw(input[2], self.fmt).float()), self.fmt)


class LRNGrad(Operation):
    """Table(grad, orig_input, orig_output) -> grad wrt input (TF LRN over the last (channel) dim, NHWC)."""

    def __init__(self, depthRadius=5, bias=1.0, alpha=1.0, beta=0.5):
        super().__init__()
        self.r, self.bias, self.alpha, self.beta = depthRadius, bias, alpha, beta

    def updateOutput(self, input):
        r, bias, alpha, beta = self.r, self.bias, self.alpha, self.beta

        def f(x):
            sq = F.pad((x * x).unsqueeze(1), (r, r)).squeeze(1)
            win = sq.unfold(-1, 2 * r + 1, 1).sum(-1)
            return x / (bias + alpha * win) ** beta
        return _autograd_grad(f, input[2].float(), input[1].float())


class FusedBatchNormGrad(Operation):
    """Table(dy, x, scale, saved_mean, saved_var) -> Table(dx, dscale, doffset) (training mode, NHWC/NCHW)."""

    def __init__(self, epsilon=1e-4, dataFormat="NHWC", isTraining=True):
        super().__init__()
        self.eps, self.fmt, self.isTraining = epsilon, dataFormat, isTraining

    def updateOutput(self, input):
        dy, x, scale, mean, var = (input[i].float() for i in range(1, 6))
        cdim = x.dim() - 1 if self.fmt == "NHWC" else 1
        red = [d for d in range(x.dim()) if d != cdim]
        shp = [1] * x.dim()
        shp[cdim] = -1
        inv = torch.rsqrt(var + self.eps).reshape(shp)
        xhat = (x - mean.reshape(shp)) * inv
        doffset = dy.sum(red)
        dscale = (dy * xhat).sum(red)
        if self.isTraining:
            m = x.numel() // x.shape[cdim]
            dx = scale.reshape(shp) * inv / m * (m * dy - doffset.reshape(shp) - xhat * dscale.reshape(shp))
        else:
            dx = dy * scale.reshape(shp) * inv
        return Table(dx, dscale, doffset)


class FusedBatchNorm(Operation):
    """Table(x, scale, offset, mean, var) -> Table(y, batch_mean, batch_var, saved_mean, saved_var)."""

    def __init__(self, epsilon=1e-4, dataFormat="NHWC", isTraining=True):
        super().__init__()
        self.eps, self.fmt, self.isTraining = epsilon, dataFormat, isTraining

    def updateOutput(self, input):
        from .tf_ops import run_op
        r = run_op("FusedBatchNorm", [input[i] for i in range(1, 6)],
                   {"epsilon": self.eps, "data_format": self.fmt, "is_training": self.isTraining})
        return Table(*r)


class Conv2DBackFilter(Operation):
    """Table(input, filter_sizes, grad) -> filter gradient (HWIO), TF Conv2DBackpropFilter."""

    def __init__(self, strideW, strideH, padW, padH, dataFormat="NHWC"):
        super().__init__()
        self.s, self.same, self.fmt = (strideH, strideW), padW == -1, dataFormat

    def updateOutput(self, input):
        x = _nchw(input[1].float(), self.fmt)
        fs = [int(v) for v in input[2].reshape(-1).tolist()]          # H W I O
        w = torch.zeros(fs[3], fs[2], fs[0], fs[1])
        ph = _tf_pads(x.shape[2], fs[0], self.s[0], self.same)
        pw = _tf_pads(x.shape[3], fs[1], self.s[1], self.same)
        xp = F.pad(x, (pw[0], pw[1], ph[0], ph[1]))
        from ..ops import conv_fn

        w = w.to(xp.device)
        g = _autograd_grad(lambda wt: conv_fn.conv2d(xp, wt, None, self.s), w, _nchw(input[3].float(), self.fmt))
        return g.permute(2, 3, 1, 0).contiguous()


class Conv2DTranspose(Operation):
    """Table(input_sizes, filter, grad) -> data gradient (TF Conv2DBackpropInput)."""

    def __init__(self, strideW, strideH, padW=-1, padH=-1, dataFormat="NHWC"):
        super().__init__()
        self.attrs = {"strides": [1, strideH, strideW, 1] if dataFormat == "NHWC" else [1, 1, strideH, strideW],
                      "padding": "SAME" if padW == -1 else "VALID", "data_format": dataFormat}

    def updateOutput(self, input):
        from .tf_ops import run_op
        return run_op("Conv2DBackpropInput", [input[1], input[2], input[3]], self.attrs)


class Conv2D(Operation):
    """Table(input, filter(HWIO)) -> conv2d, TF semantics."""

    def __init__(self, strideH, strideW, padH=-1, padW=-1, dataFormat="NHWC"):
        super().__init__()
        self.attrs = {"strides": [1, strideH, strideW, 1] if dataFormat == "NHWC" else [1, 1, strideH, strideW],
                      "padding": "SAME" if padW == -1 else "VALID", "data_format": dataFormat}

    def updateOutput(self, input):
        from .tf_ops import run_op
        return run_op("Conv2D", [input[1], input[2]], self.attrs)


def _conv3d(x, w, strides, same, fmt):
    """x NDHWC / NCDHW, w DHWIO -> y in the same format."""
    if fmt == "NDHWC":
        x = x.permute(0, 4, 1, 2, 3)
    wt = w.permute(4, 3, 0, 1, 2)
    pads = []
    for i in (2, 1, 0):
        pads += list(_tf_pads(x.shape[2 + i], wt.shape[2 + i], strides[i], same))
    from ..ops import conv_fn

    y = conv_fn.conv3d(F.pad(x, pads).float(), wt.float(), None, tuple(strides)).to(x.dtype)   # GPU: native
    return y.permute(0, 2, 3, 4, 1) if fmt == "NDHWC" else y


class Conv3D(Operation):
    """Table(input, filter(DHWIO)) -> conv3d."""

    def __init__(self, dT, dH, dW, padding="SAME", dataFormat="NDHWC"):
        super().__init__()
        self.strides, self.same, self.fmt = (dT, dH, dW), padding == "SAME", dataFormat

    def updateOutput(self, input):
        return _conv3d(input[1].float(), input[2].float(), self.strides, self.same, self.fmt)


class Conv3DBackpropFilter(Conv3D):
    """Table(input, filter, grad) -> filter gradient (filter given as a tensor of the right shape)."""

    def _filter(self, input):
        return input[2]

    def updateOutput(self, input):
        x, dy = input[1].float(), input[3].float()
        w = self._filter(input).float()
        return _autograd_grad(lambda wt: _conv3d(x, wt, self.strides, self.same, self.fmt), w, dy)


class Conv3DBackpropFilterV2(Conv3DBackpropFilter):
    """Table(input, filter_sizes, grad)."""

    def _filter(self, input):
        return torch.zeros([int(v) for v in input[2].reshape(-1).tolist()])


class Conv3DBackpropInput(Conv3D):
    """Table(input, filter, grad) -> input gradient."""

    def _input(self, input):
        return input[1]

    def updateOutput(self, input):
        x, w, dy = self._input(input).float(), input[2].float(), input[3].float()
        return _autograd_grad(lambda t: _conv3d(t, w, self.strides, self.same, self.fmt), x, dy)


class Conv3DBackpropInputV2(Conv3DBackpropInput):
    """Table(input_sizes, filter, grad)."""

    def _input(self, input):
        return torch.zeros([int(v) for v in input[1].reshape(-1).tolist()])


__all__ = [n for n in dir() if not n.startswith("_") and isinstance(globals()[n], type)
           and issubclass(globals()[n], AbstractModule)] + ["ControlNodes", "is_random", "encode_example",
                                                              "TensorModule"]
