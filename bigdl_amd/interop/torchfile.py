"""Lua Torch7 ``.t7`` binary format: reader and writer for tensors, tables and ``nn.*`` modules.

Reference: S/utils/TorchFile.scala:42-1102 (``load`` :79, ``save`` :95; type tags nil/number/string/table/
torch-object/boolean; object references; supported modules :150-169 — Sequential, Concat, ConcatTable,
Linear, SpatialConvolution(MM), SpatialMaxPooling, SpatialAveragePooling, ReLU, Threshold, Tanh, Sigmoid,
View, Reshape, Dropout, SpatialBatchNormalization, BatchNormalization, LogSoftMax, SoftMax, CAddTable,
SpatialZeroPadding, Identity, ...). Only data is read: no Lua code is ever executed (function tags are refused).
"""
import os
import struct

import torch

from .. import nn

TYPE_NIL, TYPE_NUMBER, TYPE_STRING, TYPE_TABLE, TYPE_TORCH, TYPE_BOOLEAN = 0, 1, 2, 3, 4, 5
TYPE_FUNCTION, TYPE_RECUR_FUNCTION, LEGACY_TYPE_RECUR_FUNCTION = 6, 7, 8

_STORAGE_DTYPES = {"torch.FloatStorage": ("f", 4, torch.float32), "torch.DoubleStorage": ("d", 8, torch.float64),
                   "torch.LongStorage": ("q", 8, torch.int64), "torch.IntStorage": ("i", 4, torch.int32),
                   "torch.ShortStorage": ("h", 2, torch.int16), "torch.ByteStorage": ("B", 1, torch.uint8),
                   "torch.CharStorage": ("b", 1, torch.int8), "torch.CudaStorage": ("f", 4, torch.float32)}
_TENSOR_TO_STORAGE = {k.replace("Storage", "Tensor"): k for k in _STORAGE_DTYPES}


class TorchObject(dict):
    """A non-tensor torch object (e.g. an ``nn.*`` module): its class name plus its field table."""

    def __init__(self, typename, fields):
        super().__init__(fields or {})
        self.typename = typename


class _Reader:
    def __init__(self, data):
        self.d = data
        self.p = 0
        self.refs = {}

    def _u(self, fmt, n):
        v = struct.unpack_from("<" + fmt, self.d, self.p)
        self.p += n
        return v

    def int(self):
        return self._u("i", 4)[0]

    def long(self):
        return self._u("q", 8)[0]

    def double(self):
        return self._u("d", 8)[0]

    def string(self):
        n = self.int()
        s = self.d[self.p:self.p + n]
        self.p += n
        return s.decode("latin-1")

    def read(self):
        t = self.int()
        if t == TYPE_NIL:
            return None
        if t == TYPE_NUMBER:
            v = self.double()
            return int(v) if v.is_integer() and abs(v) < 2 ** 53 else v
        if t == TYPE_STRING:
            return self.string()
        if t == TYPE_BOOLEAN:
            return self.int() == 1
        if t == TYPE_TABLE:
            idx = self.int()
            if idx in self.refs:
                return self.refs[idx]
            tbl = {}
            self.refs[idx] = tbl
            n = self.int()
            for _ in range(n):
                k = self.read()
                tbl[k] = self.read()
            return tbl
        if t == TYPE_TORCH:
            idx = self.int()
            if idx in self.refs:
                return self.refs[idx]
            version = self.string()
            if version.startswith("V "):
                cls = self.string()
            else:
                cls = version
            if cls in _STORAGE_DTYPES:
                fmt, sz, dt = _STORAGE_DTYPES[cls]
                n = self.long()
                arr = torch.frombuffer(bytearray(self.d[self.p:self.p + n * sz]), dtype=dt).clone() if n else \
                    torch.empty(0, dtype=dt)
                self.p += n * sz
                self.refs[idx] = arr
                return arr
            if cls in _TENSOR_TO_STORAGE:
                nd = self.int()
                sizes = [self.long() for _ in range(nd)]
                strides = [self.long() for _ in range(nd)]
                off = self.long() - 1
                storage = self.read()
                if nd == 0 or storage is None:
                    ten = torch.empty(0, dtype=_STORAGE_DTYPES[_TENSOR_TO_STORAGE[cls]][2])
                else:
                    ten = torch.as_strided(storage, sizes, strides, off).clone()
                self.refs[idx] = ten
                return ten
            obj = TorchObject(cls, None)
            self.refs[idx] = obj
            fields = self.read()
            if isinstance(fields, dict):
                obj.update(fields)
            return obj
        if t in (TYPE_FUNCTION, TYPE_RECUR_FUNCTION, LEGACY_TYPE_RECUR_FUNCTION):
            raise ValueError("t7 file contains a serialized Lua function; refusing to load code")
        raise ValueError(f"unknown t7 type tag {t} at offset {self.p - 4}")


def read_t7(path):
    with open(path, "rb") as f:
        return _Reader(f.read()).read()


class _Writer:
    def __init__(self):
        self.buf = bytearray()
        self.idx = 0
        self.seen = {}

    def int(self, v):
        self.buf += struct.pack("<i", v)

    def long(self, v):
        self.buf += struct.pack("<q", v)

    def string(self, s):
        b = s.encode("latin-1")
        self.int(len(b))
        self.buf += b

    def _next(self):
        self.idx += 1
        return self.idx

    def write(self, v):
        if v is None:
            self.int(TYPE_NIL)
        elif isinstance(v, bool):
            self.int(TYPE_BOOLEAN)
            self.int(1 if v else 0)
        elif isinstance(v, (int, float)):
            self.int(TYPE_NUMBER)
            self.buf += struct.pack("<d", float(v))
        elif isinstance(v, str):
            self.int(TYPE_STRING)
            self.string(v)
        elif isinstance(v, torch.Tensor):
            self._tensor(v)
        elif isinstance(v, TorchObject):
            self.int(TYPE_TORCH)
            self.int(self._next())
            self.string("V 1")
            self.string(v.typename)
            self.write(dict(v))
        elif isinstance(v, (dict, list, tuple)):
            d = v if isinstance(v, dict) else {i + 1: x for i, x in enumerate(v)}
            self.int(TYPE_TABLE)
            self.int(self._next())
            self.int(len(d))
            for k, x in d.items():
                self.write(k)
                self.write(x)
        else:
            raise TypeError(f"cannot write {type(v).__name__} to t7")

    def _tensor(self, t):
        t = t.detach().cpu().contiguous()
        name = {torch.float32: "torch.FloatTensor", torch.float64: "torch.DoubleTensor",
                torch.int64: "torch.LongTensor", torch.int32: "torch.IntTensor", torch.uint8: "torch.ByteTensor",
                torch.int16: "torch.ShortTensor", torch.int8: "torch.CharTensor"}.get(t.dtype)
        if name is None:
            t, name = t.float(), "torch.FloatTensor"
        self.int(TYPE_TORCH)
        self.int(self._next())
        self.string("V 1")
        self.string(name)
        self.int(t.dim())
        for s in t.shape:
            self.long(s)
        for s in t.stride():
            self.long(s)
        self.long(1)
        self.int(TYPE_TORCH)
        self.int(self._next())
        self.string("V 1")
        sname = _TENSOR_TO_STORAGE[name]
        self.string(sname)
        self.long(t.numel())
        self.buf += t.numpy().tobytes()


def write_t7(path, obj):
    w = _Writer()
    w.write(obj)
    with open(path, "wb") as f:
        f.write(bytes(w.buf))


# ---------------------------------------------------------------------------------------------- nn modules
def _f(o, k, d=None):
    v = o.get(k, d)
    return v


def _copy(dst, src):
    if src is not None and dst is not None and src.numel() == dst.numel():
        dst.data.copy_(src.reshape(dst.shape).to(dst.dtype))


def to_module(o):
    """Convert a t7 ``nn.*`` TorchObject into a bigdl_amd module (TorchFile.scala read* methods)."""
    if not isinstance(o, TorchObject):
        raise ValueError(f"not a torch object: {type(o).__name__}")
    c = o.typename
    train = _f(o, "train", True)
    if c in ("nn.Sequential", "nn.Concat", "nn.ConcatTable", "nn.ParallelTable"):
        m = {"nn.Sequential": nn.Sequential, "nn.ConcatTable": nn.ConcatTable, "nn.ParallelTable": nn.ParallelTable}[c]() \
            if c != "nn.Concat" else nn.Concat(int(_f(o, "dimension", 1)))
        mods = _f(o, "modules", {})
        for k in sorted(mods):
            m.add(to_module(mods[k]))
    elif c == "nn.Linear":
        w = o["weight"]
        m = nn.Linear(w.shape[1], w.shape[0], withBias=_f(o, "bias") is not None)
        _copy(m.weight, w)
        _copy(m.bias, _f(o, "bias"))
    elif c in ("nn.SpatialConvolution", "nn.SpatialConvolutionMM"):
        m = nn.SpatialConvolution(int(o["nInputPlane"]), int(o["nOutputPlane"]), int(o["kW"]), int(o["kH"]),
                                  int(_f(o, "dW", 1)), int(_f(o, "dH", 1)), int(_f(o, "padW", _f(o, "padding", 0))),
                                  int(_f(o, "padH", _f(o, "padding", 0))), withBias=_f(o, "bias") is not None)
        _copy(m.weight, o["weight"])
        _copy(m.bias, _f(o, "bias"))
    elif c == "nn.SpatialMaxPooling":
        m = nn.SpatialMaxPooling(int(o["kW"]), int(o["kH"]), int(o["dW"]), int(o["dH"]), int(_f(o, "padW", 0)),
                                 int(_f(o, "padH", 0)))
        if _f(o, "ceil_mode", False):
            m.ceil()
    elif c == "nn.SpatialAveragePooling":
        m = nn.SpatialAveragePooling(int(o["kW"]), int(o["kH"]), int(o["dW"]), int(o["dH"]), int(_f(o, "padW", 0)),
                                     int(_f(o, "padH", 0)), ceilMode=bool(_f(o, "ceil_mode", False)),
                                     countIncludePad=bool(_f(o, "count_include_pad", True)))
    elif c in ("nn.BatchNormalization", "nn.SpatialBatchNormalization"):
        rm = o["running_mean"]
        cls = nn.SpatialBatchNormalization if c == "nn.SpatialBatchNormalization" else nn.BatchNormalization
        m = cls(rm.numel(), float(_f(o, "eps", 1e-5)), float(_f(o, "momentum", 0.1)),
                affine=_f(o, "weight") is not None)
        _copy(m.runningMean, rm)
        _copy(m.runningVar, _f(o, "running_var", _f(o, "running_std")))
        if m.affine:
            _copy(m.weight, o["weight"])
            _copy(m.bias, o["bias"])
    elif c == "nn.ReLU":
        m = nn.ReLU(bool(_f(o, "inplace", False)))
    elif c == "nn.Threshold":
        m = nn.Threshold(float(_f(o, "threshold", 1e-6)), float(_f(o, "val", 0.0)))
    elif c == "nn.Tanh":
        m = nn.Tanh()
    elif c == "nn.Sigmoid":
        m = nn.Sigmoid()
    elif c == "nn.LogSoftMax":
        m = nn.LogSoftMax()
    elif c == "nn.SoftMax":
        m = nn.SoftMax()
    elif c == "nn.Dropout":
        m = nn.Dropout(float(_f(o, "p", 0.5)))
    elif c == "nn.View":
        size = _f(o, "size")
        dims = [int(x) for x in size.tolist()] if isinstance(size, torch.Tensor) else [int(size)]
        m = nn.View(*dims)
        if _f(o, "numInputDims") is not None:
            m.setNumInputDims(int(o["numInputDims"]))
    elif c == "nn.Reshape":
        size = _f(o, "size")
        m = nn.Reshape([int(x) for x in size.tolist()] if isinstance(size, torch.Tensor) else [int(size)])
    elif c == "nn.CAddTable":
        m = nn.CAddTable()
    elif c == "nn.Identity":
        m = nn.Identity()
    elif c == "nn.SpatialZeroPadding":
        m = nn.SpatialZeroPadding(int(o["pad_l"]), int(o["pad_r"]), int(o["pad_t"]), int(o["pad_b"]))
    elif c == "nn.SpatialCrossMapLRN":
        m = nn.SpatialCrossMapLRN(int(o["size"]), float(o["alpha"]), float(o["beta"]), float(_f(o, "k", 1.0)))
    elif c == "nn.Mean":
        m = nn.Mean(int(_f(o, "dimension", 1)))
    elif c == "nn.Squeeze":
        m = nn.Squeeze(int(o["dim"])) if _f(o, "dim") is not None else nn.Squeeze()
    else:
        raise ValueError(f"unsupported t7 module {c}")
    if train is False:
        m.evaluate()
    return m


def load_torch(path):
    """Load a t7 file: tensors come back as tensors, ``nn`` objects as bigdl_amd modules, tables as dicts."""
    obj = read_t7(path)
    if isinstance(obj, TorchObject) and obj.typename.startswith("nn."):
        return to_module(obj)
    return obj


def from_module(m):
    """bigdl_amd module -> TorchObject for saving (TorchFile.scala write* methods)."""
    def base(cls, **kw):
        d = {"train": m.train, "output": torch.zeros(0), "gradInput": torch.zeros(0)}
        d.update(kw)
        return TorchObject(cls, d)

    if isinstance(m, (nn.Sequential, nn.ConcatTable, nn.Concat, nn.ParallelTable)):
        cls = {nn.Sequential: "nn.Sequential", nn.ConcatTable: "nn.ConcatTable", nn.Concat: "nn.Concat",
               nn.ParallelTable: "nn.ParallelTable"}[type(m)]
        kids = list(m.modules)
        if isinstance(m, nn.Sequential):
            kids = _static_flattens(kids)
        o = base(cls, modules={i + 1: from_module(c) for i, c in enumerate(kids)})
        if isinstance(m, nn.Concat):
            o["dimension"] = m.dimension
        return o
    if isinstance(m, nn.Linear):
        return base("nn.Linear", weight=m.weight.detach().float().cpu(),
                    bias=m.bias.detach().float().cpu() if m.bias is not None else None)
    if isinstance(m, nn.SpatialConvolution):
        return base("nn.SpatialConvolution", nInputPlane=m.nInputPlane, nOutputPlane=m.nOutputPlane, kW=m.kernelW,
                    kH=m.kernelH, dW=m.strideW, dH=m.strideH, padW=m.padW, padH=m.padH,
                    weight=m.weight.detach().float().cpu().contiguous(),
                    bias=m.bias.detach().float().cpu() if m.bias is not None else None)
    if isinstance(m, nn.SpatialMaxPooling):
        return base("nn.SpatialMaxPooling", kW=m.kW, kH=m.kH, dW=m.dW, dH=m.dH, padW=m.padW, padH=m.padH,
                    ceil_mode=bool(m.ceilMode))
    if isinstance(m, nn.SpatialAveragePooling):
        return base("nn.SpatialAveragePooling", kW=m.kW, kH=m.kH, dW=m.dW, dH=m.dH, padW=m.padW, padH=m.padH,
                    ceil_mode=bool(m.ceilMode), count_include_pad=bool(m.countIncludePad))
    if isinstance(m, nn.BatchNormalization):
        cls = "nn.SpatialBatchNormalization" if isinstance(m, nn.SpatialBatchNormalization) else \
            "nn.BatchNormalization"
        return base(cls, eps=m.eps, momentum=m.momentum, running_mean=m.runningMean.detach().float().cpu(),
                    running_var=m.runningVar.detach().float().cpu(),
                    weight=m.weight.detach().float().cpu() if m.affine else None,
                    bias=m.bias.detach().float().cpu() if m.affine else None, affine=m.affine)
    simple = {nn.ReLU: "nn.ReLU", nn.Tanh: "nn.Tanh", nn.Sigmoid: "nn.Sigmoid", nn.LogSoftMax: "nn.LogSoftMax",
              nn.SoftMax: "nn.SoftMax", nn.CAddTable: "nn.CAddTable", nn.Identity: "nn.Identity"}
    if type(m) in simple:
        return base(simple[type(m)])
    if isinstance(m, nn.Dropout):
        return base("nn.Dropout", p=float(m.p))
    if isinstance(m, nn.View):
        return base("nn.View", size=torch.tensor(list(m.sizes), dtype=torch.int64),
                    numInputDims=getattr(m, "numInputDims", None))
    if isinstance(m, nn.Reshape):
        return base("nn.Reshape", size=torch.tensor(list(m.size), dtype=torch.int64))
    if isinstance(m, nn.InferReshape) and tuple(m.size) in ((0, -1), (-1,)) and (tuple(m.size) == (0, -1) or
                                                                                 m.batchMode):
        # Caffe Flatten of a [N, C, H, W] blob: per-sample flatten = nn.View(-1) over 3 input dims
        return base("nn.View", size=torch.tensor([-1], dtype=torch.int64), numInputDims=3)
    raise ValueError(f"cannot save {type(m).__name__} to t7")


def _first_linear(m):
    while True:
        if isinstance(m, nn.Linear):
            return m
        mods = getattr(m, "modules", None)
        if not mods or isinstance(m, (nn.ConcatTable, nn.Concat, nn.ParallelTable)):
            return None
        m = mods[0]


def _static_flattens(mods):
    """Torch7 nn has no shape-inferring flatten: an InferReshape(0, -1) (Caffe Flatten / InnerProduct input)
    whose consumer is a Linear becomes nn.Reshape(inputSize), which Torch7 applies per sample."""
    out = list(mods)
    for i, m in enumerate(out):
        if isinstance(m, nn.InferReshape) and tuple(m.size) == (0, -1) and i + 1 < len(out):
            lin = _first_linear(out[i + 1])
            if lin is not None:
                out[i] = nn.Reshape([lin.inputSize])
    return out


def _chain_to_sequential(g):
    """A Graph that is a single chain (e.g. an imported Caffe net without branches) as a Sequential; Torch7 nn
    has no graph container."""
    seq = nn.Sequential()
    for n in g.order:
        if len(n.prevs) > 1 or len(n.nexts) > 1:
            raise ValueError("cannot save a branching Graph to t7 (Torch7 nn has no graph container)")
        if n in g.inputs_nodes and not n.prevs:
            continue
        seq.add(n.element)
    return seq


def save_torch(obj, path, overWrite=False):
    if os.path.exists(path) and not overWrite:
        raise FileExistsError(path)
    if isinstance(obj, nn.Graph):
        obj = _chain_to_sequential(obj)
    if isinstance(obj, nn.AbstractModule):
        obj = from_module(obj)
    write_t7(path, obj)
