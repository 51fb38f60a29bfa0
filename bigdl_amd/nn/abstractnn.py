"""Module / criterion base classes.

Reference: S/nn/abstractnn/AbstractModule.scala:59-1201 (forward :255-270, backward :282-289,
updateOutput :306, updateGradInput :316, accGradParameters :327, zeroGradParameters :333, parameters :347,
getExtraParameter :358, getParametersTable :414, training/evaluate :439-457, freeze :204-233, cloneModule
:480-505, save/load :533-611, predict :637-690, evaluate :856-918, quantize :920, inputs :796-826, toGraph
:828, getTimes :168, setScaleW/B :95-106, getParameters :988), AbstractCriterion
(S/nn/abstractnn/AbstractCriterion.scala:50).

Activities are ``torch.Tensor`` or :class:`~bigdl_amd.utils.table.Table`. Tensors keep BigDL's logical
layout (NCHW for images); on the GPU engine 4-D activations are bf16 with ``channels_last`` strides (the
MFMA-friendly NHWC physical layout) and the hot layers dispatch to the gfx950 HIP kernels in
``bigdl_amd.ops``. On CPU every layer computes in fp32 with torch reference math.
"""
import copy
import itertools
import os
import time

import torch

from ..ops import side_stream as _side
from ..utils.table import Table

_REGISTRY = {}


def module_key(cls):
    """Registry / serialization key of a module class. Keras-style layers share names with torch-style ones
    (Dense vs Linear is fine, but LSTM, Sequential, Reshape, ... collide), so they are namespaced."""
    mod = cls.__module__
    if mod.startswith("bigdl_amd.keras"):
        return "keras." + cls.__name__
    if mod == "bigdl_amd.nn.tf_ops":
        return "ops." + cls.__name__
    if mod in ("bigdl_amd.nn.ops", "bigdl_amd.nn.tf", "bigdl_amd.nn.onnx", "bigdl_amd.nn.mkldnn"):
        return mod[len("bigdl_amd."):] + "." + cls.__name__
    return cls.__name__


def register(cls):
    _REGISTRY[module_key(cls)] = cls
    return cls


def module_class(name):
    return _REGISTRY[name]


def all_module_classes():
    return dict(_REGISTRY)


def _detach_nonleaf(v):
    if isinstance(v, torch.Tensor):
        return v.detach() if v.grad_fn is not None else v
    if isinstance(v, Table):
        if not any(isinstance(x, (torch.Tensor, Table)) and _has_nonleaf(x) for _, x in v.items()):
            return v
        t = Table()
        for k, x in v.items():
            t[k] = _detach_nonleaf(x)
        return t
    if isinstance(v, (list, tuple)) and any(_has_nonleaf(x) for x in v):
        return type(v)(_detach_nonleaf(x) for x in v) if isinstance(v, list) else tuple(_detach_nonleaf(x) for x in v)
    return v


def _has_nonleaf(v):
    if isinstance(v, torch.Tensor):
        return v.grad_fn is not None
    if isinstance(v, Table):
        return any(_has_nonleaf(x) for _, x in v.items())
    if isinstance(v, (list, tuple)):
        return any(_has_nonleaf(x) for x in v)
    return False


_NAME_SEQ = itertools.count(1)

class _RecordInit(type):
    """Records the constructor arguments of every module (used by the serializer and cloneModule)."""

    def __call__(cls, *args, **kw):
        obj = cls.__new__(cls)
        obj._init_args = (args, kw)
        obj.__init__(*args, **kw)
        return obj

    def __init__(cls, name, bases, ns):
        super().__init__(name, bases, ns)
        if getattr(cls, "_SYNC_HOOKS", False):
            for kind in ("forward", "backward"):
                if kind in ns:
                    setattr(cls, kind, _sync_wrap(kind, ns[kind]))
        if not name.startswith("_"):
            _REGISTRY[module_key(cls)] = cls


class StragglerTimeout(RuntimeError):
    """Raised at a module boundary once the straggler deadline of the current iteration has passed (reference
    DistriOptimizer.scala:241-278 cancels the late model replicas with invokeAndWait2(..., timeout))."""


# [deadline in time.perf_counter() seconds, 0 = none]: checked by every module forward / backward (one float
# compare), set by the Optimizer loop while a straggler threshold is active
STRAGGLER_DEADLINE = [0.0]
# the DevicePacer of the current iteration on a GPU rank (None: the deadline is checked against the host clock only)
STRAGGLER_PACER = [None]
_BWD_DEPTH = [0]


class DevicePacer:
    """Device-time straggler detection (reference: the replica's measured compute time, S/optim/DistriOptimizer.scala:
    241-278). Kernel launches are asynchronous, so on a GPU the host clock at a module boundary says nothing about
    how far the device got. The pacer records an event at every module boundary and keeps the host at most ``lag``
    boundaries ahead of the device: while it waits for the device it checks the deadline, so a rank whose GPU is
    slow raises ``StragglerTimeout`` within one boundary's worth of device work of the deadline, with at most
    ``lag`` boundaries of kernels still queued behind it. ``drain`` waits for everything enqueued (end of backward)
    under the same deadline."""

    def __init__(self, lag=8, poll_s=50e-6):
        import collections

        self.lag, self.poll_s = lag, poll_s
        self.q = collections.deque()

    def _wait(self, ev, deadline, where):
        while not ev.query():
            if time.perf_counter() > deadline:
                raise StragglerTimeout(where)
            time.sleep(self.poll_s)

    def boundary(self, deadline, where):
        ev = torch.cuda.Event()
        ev.record()
        self.q.append(ev)
        while len(self.q) > self.lag:
            self._wait(self.q[0], deadline, where)
            self.q.popleft()
        if time.perf_counter() > deadline:
            raise StragglerTimeout(where)

    def drain(self, deadline, where="end of backward"):
        ev = torch.cuda.Event()
        ev.record()
        self._wait(ev, deadline, where)
        self.q.clear()


def _deadline_check(m):
    dl = STRAGGLER_DEADLINE[0]
    p = STRAGGLER_PACER[0]
    if p is not None:
        p.boundary(dl, m.getPrintName())
    elif time.perf_counter() > dl:
        raise StragglerTimeout(m.getPrintName())


def _sync_wrap(kind, f):
    """Per-module synchroniser hooks (reference AbstractModule.scala:282-297 / 1184-1199): every module class's
    own ``forward`` / ``backward`` — including overrides in containers, Graph, BN, recurrent layers — calls
    ``self._sync.before_forward(self)`` before its forward and ``self._sync.after_backward(self)`` after its
    backward when a synchroniser is installed (ParallelOptimizer, parallel/bucketed.py). A depth counter makes an
    override that calls ``super().forward/backward`` fire once."""
    if getattr(f, "_sync_wrapped", False):
        return f
    key = "_sync_fd" if kind == "forward" else "_sync_bd"

    if kind == "forward":
        def wrapped(self, *args, **kw):
            if STRAGGLER_DEADLINE[0]:
                _deadline_check(self)
            s = self.__dict__.get("_sync")
            if s is None:
                return f(self, *args, **kw)
            d = self.__dict__.get(key, 0)
            self.__dict__[key] = d + 1
            try:
                if d == 0:
                    s.before_forward(self)
                return f(self, *args, **kw)
            finally:
                self.__dict__[key] = d
    else:
        def wrapped(self, *args, **kw):
            if STRAGGLER_DEADLINE[0]:
                _deadline_check(self)
            _BWD_DEPTH[0] += 1
            try:
                s = self.__dict__.get("_sync")
                if s is None:
                    return f(self, *args, **kw)
                d = self.__dict__.get(key, 0)
                self.__dict__[key] = d + 1
                try:
                    out = f(self, *args, **kw)
                finally:
                    self.__dict__[key] = d
                if d == 0:
                    s.after_backward(self)
                return out
            finally:
                _BWD_DEPTH[0] -= 1
                if _BWD_DEPTH[0] == 0 and _side.pending():
                    _side.join()     # gradients final when the outermost backward returns (ops/side_stream.py)
    wrapped.__name__, wrapped.__qualname__, wrapped.__doc__ = f.__name__, f.__qualname__, f.__doc__
    wrapped.__wrapped__ = f
    wrapped._sync_wrapped = True
    return wrapped


def to_device_tensor(t, device):
    return t.to(device) if isinstance(t, torch.Tensor) else t


def activity_apply(a, fn):
    if isinstance(a, torch.Tensor):
        return fn(a)
    if isinstance(a, Table):
        out = Table()
        for k, v in a.items():
            out[k] = activity_apply(v, fn)
        return out
    if isinstance(a, (list, tuple)):
        return type(a)(activity_apply(v, fn) for v in a)
    return a


class MklInt8Convertible:
    """Int8 calibration state carried by every module (reference S/nn/MklInt8Convertible.scala:53-423):
    ``calcScales`` records activation ranges over a sample batch, dim masks pick the scale granularity and the
    scale getters / setters expose what a later ``quantize()`` consumes. Ranges are max-abs values; the int8
    kernels use one input scale per tensor (mask 0) and one weight scale per output channel (mask 1)."""

    def calcScales(self, sample):
        from ..quantized.quantizer import calibrate

        calibrate(self, sample)
        return self

    def _scales(self, key):
        return self.__dict__.setdefault(key, [])

    def getInputScales(self):
        amax = self.__dict__.get("_calib_amax")
        if amax is not None and not self._scales("_input_scales"):
            return [[float(amax)]]
        return self._scales("_input_scales")

    def setInputScales(self, scales):
        self._input_scales = [list(map(float, s)) for s in scales]
        if self._input_scales and len(self._input_scales[0]) == 1:
            self._calib_amax = self._input_scales[0][0]
        return self

    def getOutputScales(self):
        return self._scales("_output_scales")

    def setOutputScales(self, scales):
        self._output_scales = [list(map(float, s)) for s in scales]
        return self

    def getWeightScales(self):
        if not self._scales("_weight_scales"):
            w = self.__dict__.get("weight")
            if torch.is_tensor(w) and w.dim() >= 2:
                return [w.detach().float().abs().reshape(w.shape[0], -1).amax(1).tolist()]
        return self._scales("_weight_scales")

    def setWeightScales(self, scales):
        self._weight_scales = [list(map(float, s)) for s in scales]
        return self

    def getInputDimMask(self):
        return self.__dict__.get("_input_dim_mask", 0)

    def setInputDimMask(self, mask):
        self._input_dim_mask = mask
        return self

    def getOutputDimMask(self):
        return self.__dict__.get("_output_dim_mask", 0)

    def setOutputDimMask(self, mask):
        self._output_dim_mask = mask
        return self

    def getWeightDimMask(self):
        return self.__dict__.get("_weight_dim_mask", 1)

    def setWeightDimMask(self, mask):
        self._weight_dim_mask = mask
        return self


# Module timing (reference AbstractModule.scala:168-196 getTimes: forward / backward time per module, nanoseconds).
# Host timing around an asynchronous GPU launch measures only the enqueue, so with device timing on
# (``AbstractModule.setDeviceTiming(True)``, ``bigdl.module.deviceTiming`` or BIGDL_DEVICE_TIMES=1) a GPU call records
# a pair of HIP timing events on the current stream instead, and getTimes() resolves the pending pairs into device
# nanoseconds (elapsed time between the events: the module's own kernels plus whatever else that stream ran in
# between; work the module forks onto the weight-gradient side stream is not included). Inside a HIP-graph capture
# no events are recorded (the host time is kept).
DEVICE_TIMING = [os.environ.get("BIGDL_DEVICE_TIMES", "0") not in ("0", "")]


def _on_cuda(x):
    if isinstance(x, torch.Tensor):
        return x.is_cuda
    if isinstance(x, (list, tuple)):
        return any(_on_cuda(v) for v in x)
    if hasattr(x, "values") and callable(x.values):
        try:
            return any(_on_cuda(v) for v in x.values())
        except Exception:
            return False
    return False


def _t_begin(x):
    """Start token of a timed module call: a recorded HIP event (device timing on, GPU input, not capturing) or the
    host clock."""
    if DEVICE_TIMING[0] and _on_cuda(x) and not torch.cuda.is_current_stream_capturing():
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev
    return time.perf_counter_ns()


def _t_end(m, tok, attr):
    """Close a timed call started by _t_begin: host time is added to ``attr`` now, an event pair is queued on the module
    and resolved by getTimes()."""
    if isinstance(tok, int):
        setattr(m, attr, getattr(m, attr) + time.perf_counter_ns() - tok)
        return
    end = torch.cuda.Event(enable_timing=True)
    end.record()
    pend = m.__dict__.setdefault("_dev_times", [])
    pend.append((attr, tok, end))


class AbstractModule(MklInt8Convertible, metaclass=_RecordInit):
    """Base of every layer and container."""

    _SYNC_HOOKS = True

    def __init__(self):
        self.output = None
        self.gradInput = None
        self.train = True
        self._name = None
        self.forward_time = 0
        self.backward_time = 0
        self.scaleW = 1.0
        self.scaleB = 1.0
        self._frozen = False
        self._params = []        # list of (weight_attr, grad_attr)
        self._buffers = []       # extra state (running stats) names
        self.wRegularizer = None
        self.bRegularizer = None
        self._w16 = {}           # bf16 compute shadows of parameters (GPU engine)
        self._w16_managed = False
        self._line_id = None
        self.weightInitMethod = None
        self.biasInitMethod = None
        self._device = torch.device("cpu")
        self._sync = None        # per-layer gradient synchronizer hook (ParallelOptimizer)

    # ------------------------------------------------------------------ naming / printing
    def setName(self, name):
        self._name = name
        return self

    def getName(self):
        if self._name is None:
            # unique per process (the reference appends a random 32-bit hex): an object-id-derived suffix collides
            # inside large models and breaks name-matched weight loading (Caffe / TF / serializer)
            self._name = f"{type(self).__name__}{next(_NAME_SEQ):08x}"
        return self._name

    def hasName(self):
        return self._name is not None

    def getPrintName(self):
        return f"{type(self).__name__}[{self.getName()}]"

    def __repr__(self):
        return self.getPrintName()

    def toString(self):
        return repr(self)

    # ------------------------------------------------------------------ forward / backward
    def forward(self, input):
        t0 = _t_begin(input)
        if getattr(input, "_is_bigdl_tensor", False):     # bigdl_amd.tensor.Tensor -> its torch tensor
            input = input._t
        try:
            self.output = self.updateOutput(input)
        except Exception as e:  # reference wraps errors with the module path (AbstractModule.scala:260-266)
            if not getattr(e, "_bigdl_wrapped", False):
                try:
                    e.args = (f"{self.getPrintName()}: {e.args[0] if e.args else ''}",) + tuple(e.args[1:])
                    e._bigdl_wrapped = True
                except Exception:
                    pass
            raise
        _t_end(self, t0, "forward_time")
        return self.output

    def backward(self, input, gradOutput):
        t0 = _t_begin(gradOutput)
        if getattr(input, "_is_bigdl_tensor", False):
            input = input._t
        if getattr(gradOutput, "_is_bigdl_tensor", False):
            gradOutput = gradOutput._t
        self.gradInput = self.updateGradInput(input, gradOutput)
        if not self._frozen:
            self.accGradParameters(input, gradOutput)
            self._apply_regularizers()
        _t_end(self, t0, "backward_time")
        return self.gradInput

    def __call__(self, *nodes):
        """Graph building: ``layer(node1, node2)`` == ``layer.inputs(node1, node2)``."""
        return self.inputs(*nodes)

    def updateOutput(self, input):
        raise NotImplementedError(type(self).__name__)

    def updateGradInput(self, input, gradOutput):
        raise NotImplementedError(type(self).__name__)

    def accGradParameters(self, input, gradOutput):
        pass

    def _apply_regularizers(self):
        if (self.wRegularizer is None and self.bRegularizer is None) or getattr(self, "_reg_folded", False):
            return
        for (w, g) in self._params:
            reg = self.bRegularizer if w == "bias" else self.wRegularizer
            wt, gt = getattr(self, w, None), getattr(self, g, None)
            if reg is not None and wt is not None and gt is not None:
                reg.accRegularization(wt, gt, self.scaleB if w == "bias" else self.scaleW)

    # ------------------------------------------------------------------ parameters
    def register_parameter(self, wname, gname, weight):
        setattr(self, wname, weight)
        setattr(self, gname, torch.zeros_like(weight) if weight is not None else None)
        self._params.append((wname, gname))

    def parameters(self):
        """(weights, grads) lists, or None for parameter-free modules (reference contract)."""
        ws, gs = [], []
        for w, g in self._params:
            wt = getattr(self, w, None)
            if wt is not None:
                ws.append(wt)
                gs.append(getattr(self, g))
        if not ws:
            return None
        return ws, gs

    def _all_params(self):
        p = self.parameters()
        return ([], []) if p is None else p

    def getParametersTable(self):
        t = Table()
        sub = Table()
        for w, g in self._params:
            if getattr(self, w, None) is not None:
                sub[w] = getattr(self, w)
                sub[g] = getattr(self, g)
        t[self.getName()] = sub
        return t

    def getExtraParameter(self):
        """Non-trainable state (e.g. BN running mean/var): list of tensors or None."""
        ext = [getattr(self, b) for b in self._buffers if getattr(self, b, None) is not None]
        return ext or None

    def setExtraParameter(self, tensors):
        it = iter(tensors)
        for b in self._buffers:
            if getattr(self, b, None) is not None:
                getattr(self, b).copy_(next(it))
        return self

    def zeroGradParameters(self):
        for g in self._all_params()[1]:
            g.zero_()

    def getParameters(self, pad_multiple=1):
        """Compact every weight (and gradient) into ONE contiguous fp32 storage and return 1-D views of it.

        Reference: AbstractModule.getParameters (AbstractModule.scala:988) + Module.flatten
        (S/nn/Module.scala:113-141). Each parameter tensor becomes a view of the flat buffer that keeps its
        own strides (conv weights stay channels_last = KRSC on the GPU engine). The flat layout is what the
        fused optimizer kernels and the RCCL bucketed all-reduce / reduce-scatter operate on.
        """
        ws, gs = self.parameters() or ([], [])
        if not ws:
            return torch.zeros(0), torch.zeros(0)
        dev = ws[0].device
        if getattr(self, "_flat", None) is not None and self._flat_ok(ws, gs):
            return self._flat
        total = sum(w.numel() for w in ws)
        padded = -(-total // pad_multiple) * pad_multiple
        fw = torch.zeros(padded, dtype=torch.float32, device=dev)
        fg = torch.zeros(padded, dtype=torch.float32, device=dev)
        views = []
        off = 0
        for w, g in zip(ws, gs):
            n = w.numel()
            stride = _dense_strides(w)
            vw = fw[off:off + n].as_strided(w.shape, stride)
            vg = fg[off:off + n].as_strided(w.shape, stride)
            vw.copy_(w.detach())
            vg.copy_(g.detach())
            views.append((vw, vg, off, n, stride))
            off += n
        self._rebind_params(views)
        self._flat_total = total
        self._flat = (fw, fg)
        self._flat_views = views
        return fw, fg

    def _flat_ok(self, ws, gs):
        fw, fg = self._flat
        return all(w.untyped_storage().data_ptr() == fw.untyped_storage().data_ptr() for w in ws)

    def _rebind_params(self, views):
        it = iter(views)
        self._rebind_into(it)

    def _rebind_into(self, it):
        for w, g in self._params:
            if getattr(self, w, None) is not None:
                vw, vg, _, _, _ = next(it)
                setattr(self, w, vw)
                setattr(self, g, vg)

    def attach_bf16_shadow(self, flat16):
        """Point every parameter's bf16 compute copy at a view of ``flat16`` (written by the optimizer)."""
        views = self._flat_views
        it = iter(views)
        self._attach16(it, flat16)

    def _attach16(self, it, flat16):
        for w, _ in self._params:
            if getattr(self, w, None) is not None:
                _, _, off, n, stride = next(it)
                self._w16[w] = flat16[off:off + n].as_strided(getattr(self, w).shape, stride)
                self._w16_managed = True

    def w16(self, name):
        """bf16 compute copy of parameter ``name`` (GPU engine). Training steps publish it from the optimizer kernel
        (``_w16_managed``); in evaluation mode the cast is cached until the parameter changes (its version counter,
        which torch in-place ops and the native TensorMath backend bump), so inference casts each weight once."""
        if self._w16_managed and name in self._w16:
            return self._w16[name]
        w = getattr(self, name)
        key = None
        if not self.train and w.is_cuda:
            key = (w.data_ptr(), w._version, tuple(w.shape), w.stride(), w.dtype)
            hit = self.__dict__.get("_w16_cache", {}).get(name)
            if hit is not None and hit[0] == key:
                return hit[1]
        from .. import ops

        if w.dim() == 4 and w.is_contiguous(memory_format=torch.channels_last):
            out = torch.empty_like(w, dtype=torch.bfloat16)
            ops.native.get().cast_f32_bf16(w.permute(0, 2, 3, 1).contiguous().view(-1),
                                           out.permute(0, 2, 3, 1).view(-1))
        else:
            out = ops.to_bf16(w)
        if key is not None:
            self.__dict__.setdefault("_w16_cache", {})[name] = (key, out)
        return out

    def mark_w16_dirty(self):
        pass

    # ------------------------------------------------------------------ modes
    def training(self):
        self.train = True
        self.__dict__.pop("_w16_cache", None)
        return self

    def evaluate(self, *args, **kw):
        if args or kw:
            from ..optim.evaluator import evaluate_module

            return evaluate_module(self, *args, **kw)
        self.train = False
        return self

    def isTraining(self):
        return self.train

    def freeze(self, *names):
        self._frozen = True
        return self

    def unFreeze(self, *names):
        self._frozen = False
        return self

    def setScaleW(self, w):
        self.scaleW = w
        return self

    def setScaleB(self, b):
        self.scaleB = b
        return self

    def getScaleW(self):
        return self.scaleW

    def getScaleB(self):
        return self.scaleB

    # ------------------------------------------------------------------ timing
    @staticmethod
    def setDeviceTiming(on=True):
        """GPU modules report device time (HIP events) in getTimes instead of host enqueue time."""
        DEVICE_TIMING[0] = bool(on)

    def _resolve_times(self):
        pend = self.__dict__.get("_dev_times")
        if not pend:
            return
        for attr, a, b in pend:
            b.synchronize()
            setattr(self, attr, getattr(self, attr) + int(a.elapsed_time(b) * 1e6))
        pend.clear()

    def getTimes(self):
        self._resolve_times()
        return [(self, self.forward_time, self.backward_time)]

    def getTimesGroupByModuleType(self):
        agg = {}
        for m, f, b in self.getTimes():
            k = type(m).__name__
            fa, ba = agg.get(k, (0, 0))
            agg[k] = (fa + f, ba + b)
        return [(k, f, b) for k, (f, b) in agg.items()]

    def resetTimes(self):
        self.__dict__.pop("_dev_times", None)
        self.forward_time = 0
        self.backward_time = 0

    # ------------------------------------------------------------------ init methods
    def setInitMethod(self, weightInitMethod=None, biasInitMethod=None):
        if weightInitMethod is not None:
            self.weightInitMethod = weightInitMethod
        if biasInitMethod is not None:
            self.biasInitMethod = biasInitMethod
        self.reset()
        return self

    def reset(self):
        pass

    # ------------------------------------------------------------------ devices
    def to(self, device, memory_format=None):
        device = torch.device(device)
        self._device = device
        for w, g in self._params:
            for a in (w, g):
                t = getattr(self, a, None)
                if t is not None:
                    setattr(self, a, self._place(a, t.to(device)))
        for b in self._buffers:
            t = getattr(self, b, None)
            if t is not None:
                setattr(self, b, t.to(device))
        self._w16 = {}
        self._w16_managed = False
        self._flat = None
        self.output = None
        self.gradInput = None
        self._on_device_change()
        return self

    def _place(self, attr, t):
        return t

    def _on_device_change(self):
        pass

    def cuda(self, idx=None):
        return self.to(torch.device("cuda", idx) if idx is not None else "cuda")

    def cpu(self):
        return self.to("cpu")

    @property
    def device(self):
        return self._device

    # ------------------------------------------------------------------ cloning / structure
    def cloneModule(self):
        # graphs of a few hundred nodes (imported Caffe / TF models) are linked node -> node, which a recursive
        # deepcopy walks depth-first: give it room instead of failing at Python's default depth
        import sys

        old = sys.getrecursionlimit()
        sys.setrecursionlimit(max(old, 100000))
        try:
            return copy.deepcopy(self)
        finally:
            sys.setrecursionlimit(old)

    def clone(self):
        return self.cloneModule()

    def modules_list(self):
        return []

    def apply_modules(self, fn):
        fn(self)
        for m in self.modules_list():
            m.apply_modules(fn)

    def flattened_layers(self):
        out = []
        self.apply_modules(lambda m: out.append(m))
        return out

    def findModules(self, typename):
        return [m for m in self.flattened_layers() if type(m).__name__ == typename]

    def apply1(self, name):
        for m in self.flattened_layers():
            if m.hasName() and m.getName() == name:
                return m
        return None

    def __getitem__(self, name):
        return self.apply1(name)

    def clearState(self):
        self.output = None
        self.gradInput = None
        return self

    def __deepcopy__(self, memo):
        cls = type(self)
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            if k in ("output", "gradInput", "_flat", "_flat_views", "_w16", "_sync", "_sync_fd", "_sync_bd"):
                setattr(new, k, {} if k == "_w16" else (0 if k in ("_sync_fd", "_sync_bd") else None))
            elif isinstance(v, torch.Tensor):
                setattr(new, k, v.detach().clone(memory_format=torch.preserve_format))
            else:   # cached autograd activations (non-leaf tensors) are copied as plain data
                setattr(new, k, copy.deepcopy(_detach_nonleaf(v), memo))
        new._w16_managed = False
        return new

    # ------------------------------------------------------------------ graph building
    def inputs(self, *nodes):
        from .graph import Node

        node = Node(self)
        for n in nodes:
            if isinstance(n, tuple) and len(n) == 2 and isinstance(n[1], int):   # (node, fromIndex) edge
                n[0].add_next(node, n[1])
            elif isinstance(n, (list, tuple)):
                for x in n:
                    if isinstance(x, tuple):
                        x[0].add_next(node, x[1])
                    else:
                        x.add_next(node)
            elif n is not None:
                n.add_next(node)
        return node

    def toGraph(self, *startNodes):
        """Graph over this module's leaf layers (containers flattened; reference Sequential/DynamicContainer
        .toGraph). The layers are shared with this module, not copied."""
        from .graph import Graph, Input

        if getattr(self, "modules", None):
            from ..utils.intermediate import BlasToIR

            return BlasToIR.convert(self).build("blas", share=True)
        inp = Input()
        out = self.inputs(inp)
        return Graph([inp], [out])

    # ------------------------------------------------------------------ persistence / inference
    def saveModule(self, path, weightPath=None, overWrite=False, format=None):
        from ..utils.serializer import save_module

        save_module(self, path, weightPath, overWrite, format)
        return self

    def saveBigDL(self, path, weightPath=None, overWrite=False):
        """Write the reference's bigdl.proto ``BigDLModule`` format (utils/bigdl_proto.py)."""
        return self.saveModule(path, weightPath, overWrite, format="bigdl")

    def save(self, path, overWrite=False):
        return self.saveModule(path, overWrite=overWrite)

    def saveCaffe(self, prototxtPath, modelPath, useV2=True, overwrite=False):
        from ..interop.caffe import save_caffe

        save_caffe(self, prototxtPath, modelPath, overwrite)
        return self

    def saveTF(self, inputs, path, byteOrder=None, dataFormat="NHWC"):
        from ..interop.tensorflow import save_tf

        return save_tf(self, inputs, path, byteOrder, dataFormat)

    def saveTorch(self, path, overWrite=False):
        from ..interop.torchfile import save_torch

        save_torch(self, path, overWrite)
        return self

    def predict(self, dataset, batchSize=-1, shareBuffer=False):
        from ..optim.predictor import Predictor

        return Predictor(self, batchSize).predict(dataset)

    def predictClass(self, dataset, batchSize=-1):
        from ..optim.predictor import Predictor

        return Predictor(self, batchSize).predictClass(dataset)

    def quantize(self):
        from ..quantized.quantizer import quantize

        return quantize(self)

    def setOptimMethod(self, m):
        self._optim_method = m
        return self

    def release(self):
        return self


def _dense_strides(t):
    """Dense strides with the same dimension ordering as ``t`` (preserves channels_last)."""
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last) and not t.is_contiguous():
        N, C, H, W = t.shape
        return (H * W * C, 1, W * C, C)
    st = []
    acc = 1
    for d in reversed(t.shape):
        st.append(acc)
        acc *= d
    return tuple(reversed(st))


class TensorModule(AbstractModule):
    """Tensor → Tensor module (reference TensorModule, AbstractModule.scala:48)."""


class AutogradModule(TensorModule):
    """A module whose backward is derived with torch autograd from a functional forward.

    Used for the long tail of element-wise / shape / reduction layers. The hot layers (conv, BN, ReLU,
    pooling, linear, residual add, cross-entropy, LSTM) have explicit native backward implementations.
    Subclasses implement ``fn(self, x)`` using torch ops on the parameters returned by ``_fn_params``.
    """

    def fn(self, x):
        raise NotImplementedError

    def updateOutput(self, input):
        if not torch.is_grad_enabled() and not self.train:
            self._ag = None
            return self.fn(input)
        xin = activity_apply(input, lambda t: t.detach().requires_grad_(t.is_floating_point()))
        params = self._ag_params()
        with torch.enable_grad():
            out = self.fn_with(xin, params)
        self._ag = (xin, params, out)
        return activity_apply(out, lambda t: t.detach())

    def _ag_params(self):
        ws = self._all_params()[0]
        return [w.detach().requires_grad_(True) for w in ws]

    def fn_with(self, x, params):
        saved = []
        names = [w for w, _ in self._params if getattr(self, w, None) is not None]
        for n, p in zip(names, params):
            saved.append(getattr(self, n))
            object.__setattr__(self, n, p)
        try:
            return self.fn(x)
        finally:
            for n, s in zip(names, saved):
                object.__setattr__(self, n, s)

    def _grads(self, gradOutput):
        if getattr(self, "_ag", None) is None:
            raise RuntimeError(f"{type(self).__name__}: backward called without a training forward")
        xin, params, out = self._ag
        outs = _flatten(out)
        gouts = _flatten(gradOutput)
        pairs = [(o, g) for o, g in zip(outs, gouts) if o.requires_grad and g is not None]
        ins = [t for t in _flatten(xin) if t.requires_grad]
        targets = ins + params
        if not pairs or not targets:
            gi = [None] * len(ins)
            return gi, [None] * len(params)
        grads = torch.autograd.grad([o for o, _ in pairs], targets,
                                    [g.to(o.dtype) for o, g in pairs], allow_unused=True, retain_graph=True)
        return list(grads[:len(ins)]), list(grads[len(ins):])

    def updateGradInput(self, input, gradOutput):
        gi, gp = self._grads(gradOutput)
        self._pending_param_grads = gp
        xin = self._ag[0]
        it = iter(gi)

        def fill(t):
            if t.requires_grad:
                g = next(it)
                return torch.zeros_like(t) if g is None else g
            return torch.zeros_like(t)

        return activity_apply(xin, fill)

    def accGradParameters(self, input, gradOutput):
        gp = getattr(self, "_pending_param_grads", None)
        if gp is None:
            return
        for (w, g), pg in zip([p for p in self._params if getattr(self, p[0], None) is not None], gp):
            if pg is not None:
                scale = self.scaleB if w == "bias" else self.scaleW
                getattr(self, g).add_(pg.to(getattr(self, g).dtype), alpha=scale)
        self._pending_param_grads = None


def _flatten(a):
    if isinstance(a, torch.Tensor):
        return [a]
    if isinstance(a, Table):
        out = []
        for v in a.toSeq() if a.length() == len(a.keys()) else a.values():
            out.extend(_flatten(v))
        return out
    if isinstance(a, (list, tuple)):
        out = []
        for v in a:
            out.extend(_flatten(v))
        return out
    return []


class AbstractCriterion(metaclass=_RecordInit):
    """Loss function (reference S/nn/abstractnn/AbstractCriterion.scala:50)."""

    def __init__(self, sizeAverage=True):
        self.output = 0.0
        self.gradInput = None
        self.sizeAverage = sizeAverage
        self._device = torch.device("cpu")

    def forward(self, input, target):
        input = input._t if getattr(input, "_is_bigdl_tensor", False) else input
        target = target._t if getattr(target, "_is_bigdl_tensor", False) else target
        self.output = self.updateOutput(input, target)
        return self.output

    def backward(self, input, target):
        input = input._t if getattr(input, "_is_bigdl_tensor", False) else input
        target = target._t if getattr(target, "_is_bigdl_tensor", False) else target
        self.gradInput = self.updateGradInput(input, target)
        return self.gradInput

    def updateOutput(self, input, target):
        raise NotImplementedError

    def updateGradInput(self, input, target):
        raise NotImplementedError

    def cloneCriterion(self):
        return copy.deepcopy(self)

    def to(self, device):
        self._device = torch.device(device)
        return self

    def __repr__(self):
        return type(self).__name__


class TensorCriterion(AbstractCriterion):
    pass


class AutogradCriterion(AbstractCriterion):
    """Criterion with autograd-derived gradient. Subclasses implement ``loss(input, target)``."""

    def loss(self, input, target):
        raise NotImplementedError

    def updateOutput(self, input, target):
        xin = activity_apply(input, lambda t: t.detach().float().requires_grad_(True))
        tgt = activity_apply(target, lambda t: t.detach())
        with torch.enable_grad():
            out = self.loss(xin, tgt)
        self._ag = (xin, out)
        return out.detach()

    def updateGradInput(self, input, target):
        if getattr(self, "_ag", None) is None or self._ag[0] is None:
            self.updateOutput(input, target)
        xin, out = self._ag
        ins = _flatten(xin)
        grads = torch.autograd.grad(out, ins, allow_unused=True)
        it = iter(grads)

        def fill(t):
            g = next(it)
            return torch.zeros_like(t) if g is None else g

        gi = activity_apply(xin, fill)
        dt = input.dtype if isinstance(input, torch.Tensor) else None
        if dt is not None and dt != torch.float32:
            gi = gi.to(dt)
        return gi
