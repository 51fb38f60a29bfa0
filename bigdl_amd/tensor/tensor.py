"""BigDL ``Tensor`` API: a Torch7-style, 1-based, mutable-by-default tensor over a ``torch.Tensor``.

Reference: S/tensor/Tensor.scala:37-1400 (API + factory object :853), TensorMath.scala:38-829 (~150 math ops),
DenseTensor.scala:33 (semantics: ops write into ``this`` and return it), Storage.scala:26 / ArrayStorage.scala:25,
SparseTensor.scala:55, DenseTensorConv.scala:24-253 (conv2 / xcorr2).

Design: the compute data lives in a ``torch.Tensor`` (host or HBM), so every op dispatches to PyTorch-ROCm kernels
on the device the tensor lives on; this class only supplies BigDL's calling conventions:
  * dimensions and indices are 1-based (``narrow(1, 2, 3)``, ``select``, ``valueAt``, ``max(dim)`` indices,
    ``gather`` / ``scatter`` / ``index`` / ``topk`` index tensors);
  * most math methods are in place on ``self`` and return ``self`` (``x.add(y)`` is ``x += y``,
    ``x.addmm(a, b)`` is ``x = x + a @ b``; overloads with a source tensor write the result into ``self``);
  * views (``narrow``, ``select``, ``transpose``, ``view``, ``set(storage, ...)``) share storage like the reference.
Modules accept a ``Tensor`` wherever they accept a ``torch.Tensor`` (``AbstractModule.forward`` unwraps it);
``t.torch()`` / ``Tensor.of(torch_tensor)`` convert without copies.
"""
import math
import numbers

import numpy as np
import torch

from ..ops import tensor_math as _tm

_DTYPES = {"float": torch.float32, "double": torch.float64, "int": torch.int32, "long": torch.int64,
           "short": torch.int16, "byte": torch.uint8, "char": torch.int8, "boolean": torch.bool,
           "bfloat16": torch.bfloat16, "half": torch.float16}


def _d(dim):
    """1-based dimension -> 0-based."""
    return dim - 1


def _g32(*ts):
    """Every operand an fp32 GPU tensor: the native TensorMath backend (ops/tensor_math.py, csrc/tensor_math.hip)
    runs the op; other dtypes and the CPU engine use torch."""
    return all(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 for t in ts)


# torch element functions the native backend implements (csrc/tensor_math.hip op names)
_NATIVE_UNARY = {"abs": "ABS", "exp": "EXP", "log": "LOG", "log1p": "LOG1P", "sqrt": "SQRT", "square": "SQUARE",
                 "tanh": "TANH", "floor": "FLOOR", "ceil": "CEIL", "sign": "SIGN"}


def _same(*ts):
    return all(tuple(t.shape) == tuple(ts[0].shape) for t in ts)


def _raw(x):
    return x._t if isinstance(x, Tensor) else x


def _sizes(args):
    if len(args) == 1 and isinstance(args[0], (list, tuple, torch.Size)):
        return [int(s) for s in args[0]]
    if len(args) == 1 and isinstance(args[0], Tensor):
        return [int(s) for s in args[0]._t.reshape(-1).tolist()]
    return [int(s) for s in args]


class Storage:
    """Flat 1-based storage (reference ArrayStorage.scala:25). Backed by a 1-D torch tensor."""

    def __init__(self, data=None, dtype=torch.float32, device=None):
        if data is None:
            self._s = torch.empty(0, dtype=dtype, device=device)
        elif isinstance(data, int):
            self._s = torch.zeros(data, dtype=dtype, device=device)
        elif isinstance(data, torch.Tensor):
            self._s = data.reshape(-1)
        else:
            self._s = torch.as_tensor(np.asarray(data), dtype=dtype, device=device).reshape(-1)

    def __len__(self):
        return self._s.numel()

    def length(self):
        return self._s.numel()

    size = length

    def __call__(self, i):
        return self._s[i - 1].item()

    apply = __call__

    def update(self, i, v):
        self._s[i - 1] = v
        return self

    def array(self):
        return self._s.cpu().numpy()

    def fill(self, v, offset=1, length=None):
        n = self._s.numel() - offset + 1 if length is None else length
        self._s[offset - 1: offset - 1 + n] = v
        return self

    def copy(self, src, srcOffset=1, dstOffset=1, length=None):
        src = src._s if isinstance(src, Storage) else torch.as_tensor(src).reshape(-1)
        n = src.numel() - srcOffset + 1 if length is None else length
        self._s[dstOffset - 1: dstOffset - 1 + n] = src[srcOffset - 1: srcOffset - 1 + n]
        return self

    def resize(self, n):
        if n != self._s.numel():
            new = torch.zeros(n, dtype=self._s.dtype, device=self._s.device)
            k = min(n, self._s.numel())
            new[:k] = self._s[:k]
            self._s = new
        return self

    def __iter__(self):
        return iter(self._s.tolist())

    def __eq__(self, other):
        return isinstance(other, Storage) and torch.equal(self._s, other._s)

    def __repr__(self):
        return f"Storage({self._s.tolist()})"


class Tensor:
    """1-based Torch7-style tensor (reference Tensor.scala:37)."""
    __slots__ = ("_t", "_storage")
    _is_bigdl_tensor = True

    # ------------------------------------------------------------------ construction
    def __init__(self, *args, dtype=torch.float32, device=None):
        self._storage = None
        if not args:
            self._t = torch.empty(0, dtype=dtype, device=device)
        elif len(args) == 1 and isinstance(args[0], torch.Tensor):
            self._t = args[0]
        elif len(args) == 1 and isinstance(args[0], Tensor):
            self._t = args[0]._t
        elif len(args) == 1 and isinstance(args[0], Storage):
            self._t = args[0]._s
            self._storage = args[0]
        elif len(args) >= 1 and isinstance(args[0], Storage):
            st = args[0]
            off = args[1] if len(args) > 1 else 1
            sizes = args[2] if len(args) > 2 else [st.length() - off + 1]
            strides = args[3] if len(args) > 3 else None
            self._storage = st
            self._t = st._s.as_strided(list(sizes), list(strides) if strides else _contig_strides(sizes), off - 1)
        elif len(args) == 1 and isinstance(args[0], (list, tuple, np.ndarray)) and len(args[0]) and \
                not all(isinstance(v, numbers.Integral) for v in np.asarray(args[0]).reshape(-1)[:1]):
            self._t = torch.as_tensor(np.asarray(args[0]), dtype=dtype, device=device)
        elif len(args) == 1 and isinstance(args[0], np.ndarray):
            self._t = torch.as_tensor(args[0], device=device)
        elif len(args) == 2 and isinstance(args[0], (list, tuple, np.ndarray)) and \
                isinstance(args[1], (list, tuple, torch.Size)):      # Tensor(data, shape)
            self._t = torch.as_tensor(np.asarray(args[0]), dtype=dtype, device=device).reshape(list(args[1]))
        else:
            self._t = torch.zeros(_sizes(args), dtype=dtype, device=device)

    @staticmethod
    def of(t):
        return Tensor(t)

    def torch(self):
        return self._t

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):   # lets torch functions accept a Tensor
        def unwrap(a):
            if isinstance(a, Tensor):
                return a._t
            if isinstance(a, (list, tuple)):
                return type(a)(unwrap(x) for x in a)
            return a
        return func(*unwrap(args), **{k: unwrap(v) for k, v in (kwargs or {}).items()})

    def _wrap(self, t):
        return Tensor(t)

    def _set_t(self, t):
        self._t = t
        self._storage = None
        return self

    # ------------------------------------------------------------------ shape / metadata
    def dim(self):
        return self._t.dim()

    nDimension = dim

    def nElement(self):
        return self._t.numel()

    def size(self, dim=None):
        return list(self._t.shape) if dim is None else self._t.shape[_d(dim)]

    def stride(self, dim=None):
        return list(self._t.stride()) if dim is None else self._t.stride(_d(dim))

    def isEmpty(self):
        return self._t.numel() == 0

    def isScalar(self):
        return self._t.dim() == 0

    def isContiguous(self):
        return self._t.is_contiguous()

    def isSameSizeAs(self, other):
        return list(self._t.shape) == list(_raw(other).shape)

    def getType(self):
        return {v: k for k, v in _DTYPES.items()}.get(self._t.dtype, str(self._t.dtype))

    def getTensorType(self):
        return "SparseType" if self._t.is_sparse else "DenseType"

    def storage(self):
        if self._storage is None:
            base = self._t
            try:
                flat = torch.as_strided(base, (base.untyped_storage().nbytes() // base.element_size(),), (1,), 0)
            except RuntimeError:
                flat = base.reshape(-1)
            self._storage = Storage(flat)
        return self._storage

    def storageOffset(self):
        return self._t.storage_offset() + 1

    @property
    def device(self):
        return self._t.device

    @property
    def shape(self):
        return self._t.shape

    def __len__(self):
        return self._t.shape[0]

    # ------------------------------------------------------------------ element access
    def __call__(self, index):
        return self.select(1, index) if self._t.dim() > 1 else self._t[index - 1].item()

    def apply(self, index):
        return self(index)

    def valueAt(self, *idx):
        return self._t[tuple(i - 1 for i in idx)].item()

    def value(self):
        return self._t.reshape(-1)[0].item() if self._t.numel() == 1 else self._t.item()

    def setValue(self, *args):
        *idx, v = args
        self._t[tuple(i - 1 for i in idx)] = v
        return self

    def update(self, index, value):
        if isinstance(value, Tensor):
            self._t[index - 1].copy_(value._t)
        else:
            self._t[index - 1] = value
        return self

    def toArray(self):
        return self._t.detach().cpu().reshape(-1).numpy()

    def numpy(self):
        return self._t.detach().cpu().numpy()

    def tolist(self):
        return self._t.tolist()

    # ------------------------------------------------------------------ views
    def narrow(self, dim, index, size):
        return self._wrap(self._t.narrow(_d(dim), index - 1, size))

    def select(self, dim, index):
        return self._wrap(self._t.select(_d(dim), index - 1))

    def transpose(self, dim1, dim2):
        return self._wrap(self._t.transpose(_d(dim1), _d(dim2)))

    def t(self):
        assert self._t.dim() == 2, "t() expects a 2D tensor"
        return self._wrap(self._t.t())

    def view(self, *sizes):
        return self._wrap(self._t.view(_sizes(sizes)))

    def reshape(self, *sizes):
        return self._wrap(self._t.reshape(_sizes(sizes)).clone())

    def expand(self, *sizes):
        return self._wrap(self._t.expand(_sizes(sizes)))

    def expandAs(self, template):
        return self._wrap(self._t.expand_as(_raw(template)))

    def unfold(self, dim, size, step):
        return self._wrap(self._t.unfold(_d(dim), size, step))

    def contiguous(self):
        return self if self._t.is_contiguous() else self._wrap(self._t.contiguous())

    def squeeze(self, dim=None):
        return self._set_t(self._t.squeeze() if dim is None else self._t.squeeze(_d(dim)))

    def squeezeNewTensor(self):
        return self._wrap(self._t.squeeze())

    def addSingletonDimension(self, t=None, dim=1):
        src = self._t if t is None else _raw(t)
        return self._set_t(src.unsqueeze(_d(dim)))

    def addMultiDimension(self, t=None, dims=(1,)):
        src = self._t if t is None else _raw(t)
        for d in sorted(dims):
            src = src.unsqueeze(_d(d))
        return self._set_t(src)

    def split(self, size, dim=1):
        if isinstance(size, int) and dim is not None:
            return [self._wrap(x) for x in torch.split(self._t, size, _d(dim))]
        return [self._wrap(x) for x in torch.split(self._t, 1, _d(size))]

    def repeatTensor(self, *sizes):
        return self._wrap(self._t.repeat(_sizes(sizes)))

    def shallowClone(self):
        return self._wrap(self._t)

    def clone(self):
        return self._wrap(self._t.clone())

    def emptyInstance(self):
        return Tensor(torch.empty(0, dtype=self._t.dtype, device=self._t.device))

    def cast(self, castTensor):
        dst = _raw(castTensor)
        res = self._t.to(dst.dtype)
        castTensor._set_t(res.clone() if res is self._t else res)
        return castTensor

    def to(self, *a, **kw):
        return self._wrap(self._t.to(*a, **kw))

    def cuda(self):
        return self._wrap(self._t.cuda())

    def cpu(self):
        return self._wrap(self._t.cpu())

    # ------------------------------------------------------------------ mutation of shape / content
    def resize(self, *sizes):
        sz = _sizes(sizes)
        if list(self._t.shape) == sz:
            return self
        n = int(np.prod(sz)) if sz else 1
        if self._t.is_contiguous() and self._t.numel() == n:
            return self._set_t(self._t.view(sz))
        try:
            self._t.resize_(sz)
            self._storage = None
        except RuntimeError:
            self._set_t(torch.zeros(sz, dtype=self._t.dtype, device=self._t.device))
        return self

    def resizeAs(self, src):
        return self.resize(list(_raw(src).shape))

    def set(self, *args):
        if not args:
            return self._set_t(torch.empty(0, dtype=self._t.dtype, device=self._t.device))
        if isinstance(args[0], Tensor):
            self._t = args[0]._t
            self._storage = args[0]._storage
            return self
        st = args[0]
        off = args[1] if len(args) > 1 else 1
        sizes = list(args[2]) if len(args) > 2 else [st.length() - off + 1]
        strides = list(args[3]) if len(args) > 3 else _contig_strides(sizes)
        self._t = st._s.as_strided(sizes, strides, off - 1)
        self._storage = st
        return self

    def copy(self, other):
        src = _raw(other)
        if src.numel() != self._t.numel():
            raise ValueError(f"copy: element count mismatch {src.numel()} vs {self._t.numel()}")
        src = src.reshape(self._t.shape) if src.shape != self._t.shape else src
        if _g32(self._t, src) and _tm.apply(_tm.COPY, self._t, src):
            return self
        self._t.copy_(src)
        return self

    def fill(self, v):
        if _g32(self._t) and _tm.apply(_tm.FILL, self._t, s0=v):
            return self
        self._t.fill_(v)
        return self

    forceFill = fill

    def zero(self):
        if _g32(self._t) and _tm.apply(_tm.FILL, self._t, s0=0.0):
            return self
        self._t.zero_()
        return self

    def rand(self, lowerBound=0.0, upperBound=1.0):
        from ..utils.random_generator import RNG
        self._t.copy_(RNG.uniform(lowerBound, upperBound, tuple(self._t.shape)).to(self._t))
        return self

    def randn(self, mean=0.0, stdv=1.0):
        from ..utils.random_generator import RNG
        self._t.copy_(RNG.normal(mean, stdv, tuple(self._t.shape)).to(self._t))
        return self

    def uniform(self, a=0.0, b=1.0):
        from ..utils.random_generator import RNG
        return RNG.uniform(a, b)

    def bernoulli(self, p):
        from ..utils.random_generator import RNG
        self._t.copy_(RNG.bernoulli(p, tuple(self._t.shape)).to(self._t))
        return self

    def apply1(self, func):
        flat = self._t.reshape(-1)
        vals = [func(v) for v in flat.tolist()]
        self._t.copy_(torch.tensor(vals, dtype=self._t.dtype).reshape(self._t.shape))
        return self

    def map(self, other, func):
        a, b = self._t.reshape(-1).tolist(), _raw(other).reshape(-1).tolist()
        self._t.copy_(torch.tensor([func(x, y) for x, y in zip(a, b)], dtype=self._t.dtype).reshape(self._t.shape))
        return self

    def zipWith(self, t1, t2, func):
        a, b = _raw(t1).reshape(-1).tolist(), _raw(t2).reshape(-1).tolist()
        self.resizeAs(t1)
        self._t.copy_(torch.tensor([func(x, y) for x, y in zip(a, b)], dtype=self._t.dtype).reshape(self._t.shape))
        return self

    # ------------------------------------------------------------------ arithmetic (in place on self)
    def _assign(self, res):
        if list(res.shape) != list(self._t.shape):
            self.resize(list(res.shape))
        self._t.copy_(res)
        return self

    def add(self, *args):
        """add(value) | add(y) | add(value, y) | add(x, y) | add(x, value, y) (TensorMath.scala:65-108)."""
        if self._native_axpy(_tm.ADD, _tm.ADDS, args):
            return self
        if len(args) == 1:
            a = args[0]
            self._t.add_(_raw(a))
        elif len(args) == 2:
            a, b = args
            if isinstance(a, numbers.Number):
                self._t.add_(_raw(b), alpha=a)
            else:
                return self._assign(_raw(a) + _raw(b))
        else:
            x, v, y = args
            return self._assign(_raw(x) + v * _raw(y))
        return self

    def sub(self, *args):
        if self._native_axpy(_tm.SUB, None, args):
            return self
        if len(args) == 1:
            self._t.sub_(_raw(args[0]))
        elif len(args) == 2:
            a, b = args
            if isinstance(a, numbers.Number):
                self._t.sub_(_raw(b), alpha=a)
            else:
                return self._assign(_raw(a) - _raw(b))
        else:
            x, v, y = args
            return self._assign(_raw(x) - v * _raw(y))
        return self

    def _native_axpy(self, op, op_scalar, args):
        """add / sub on the native backend: (value) | (y) | (value, y) | (x, y) | (x, value, y), same shapes."""
        t = self._t
        if not _g32(t):
            return False
        if len(args) == 1:
            a = args[0]
            if isinstance(a, numbers.Number):
                return op_scalar is not None and _tm.apply(op_scalar, t, t, s0=a)
            y = _raw(a)
            return _g32(y) and _same(t, y) and _tm.apply(op, t, t, y, s0=1.0)
        if len(args) == 2:
            a, b = args
            if isinstance(a, numbers.Number):
                y = _raw(b)
                return _g32(y) and _same(t, y) and _tm.apply(op, t, t, y, s0=a)
            x, y = _raw(a), _raw(b)
            return _g32(x, y) and _same(t, x, y) and _tm.apply(op, t, x, y, s0=1.0)
        x, v, y = _raw(args[0]), args[1], _raw(args[2])
        return _g32(x, y) and _same(t, x, y) and _tm.apply(op, t, x, y, s0=v)

    def _native_ew(self, op, a, b=None, c=None, s0=0.0, s1=0.0):
        """self = op(a, b, c) on the native backend when every tensor is fp32 on the GPU with self's shape."""
        ts = [x for x in (a, b, c) if x is not None]
        return (_g32(self._t, *ts) and _same(self._t, *ts)
                and _tm.apply(op, self._t, a, b, c, s0=s0, s1=s1))

    def mul(self, *args):
        if len(args) == 1:
            if isinstance(args[0], numbers.Number) and self._native_ew(_tm.MULS, self._t, s0=args[0]):
                return self
            self._t.mul_(args[0])
            return self
        x, v = args
        if isinstance(v, numbers.Number) and self._native_ew(_tm.MULS, _raw(x), s0=v):
            return self
        return self._assign(_raw(x) * v)

    def div(self, *args):
        if len(args) == 1:
            a = args[0]
            if isinstance(a, numbers.Number):
                if self._native_ew(_tm.DIVS, self._t, s0=a):
                    return self
            elif self._native_ew(_tm.DIV, self._t, _raw(a)):
                return self
            self._t.div_(_raw(a))
            return self
        x, v = args
        if not isinstance(v, numbers.Number) and self._native_ew(_tm.DIV, _raw(x), _raw(v)):
            return self
        return self._assign(_raw(x) / _raw(v))

    def cmul(self, *args):
        if len(args) == 1:
            if self._native_ew(_tm.MUL, self._t, _raw(args[0])):
                return self
            self._t.mul_(_raw(args[0]))
            return self
        if self._native_ew(_tm.MUL, _raw(args[0]), _raw(args[1])):
            return self
        return self._assign(_raw(args[0]) * _raw(args[1]))

    def cdiv(self, *args):
        if len(args) == 1:
            if self._native_ew(_tm.DIV, self._t, _raw(args[0])):
                return self
            self._t.div_(_raw(args[0]))
            return self
        if self._native_ew(_tm.DIV, _raw(args[0]), _raw(args[1])):
            return self
        return self._assign(_raw(args[0]) / _raw(args[1]))

    def cmax(self, *args):
        if len(args) == 1 and isinstance(args[0], numbers.Number):
            if self._native_ew(_tm.CLAMP, self._t, s0=args[0], s1=math.inf):
                return self
        elif len(args) == 1:
            if self._native_ew(_tm.MAX, self._t, _raw(args[0])):
                return self
        elif self._native_ew(_tm.MAX, _raw(args[0]), _raw(args[1])):
            return self
        if len(args) == 1:
            o = args[0]
            res = torch.clamp(self._t, min=o) if isinstance(o, numbers.Number) else torch.maximum(self._t, _raw(o))
            return self._assign(res)
        return self._assign(torch.maximum(_raw(args[0]), _raw(args[1])))

    def cmin(self, *args):
        if len(args) == 1 and isinstance(args[0], numbers.Number):
            if self._native_ew(_tm.CLAMP, self._t, s0=-math.inf, s1=args[0]):
                return self
        elif len(args) == 1:
            if self._native_ew(_tm.MIN, self._t, _raw(args[0])):
                return self
        elif self._native_ew(_tm.MIN, _raw(args[0]), _raw(args[1])):
            return self
        if len(args) == 1:
            o = args[0]
            res = torch.clamp(self._t, max=o) if isinstance(o, numbers.Number) else torch.minimum(self._t, _raw(o))
            return self._assign(res)
        return self._assign(torch.minimum(_raw(args[0]), _raw(args[1])))

    def addcmul(self, *args):
        """addcmul(value, t1, t2) | addcmul(t1, t2): self += value * t1 * t2."""
        v, t1, t2 = args if len(args) == 3 else (1.0, *args)
        if self._native_ew(_tm.ADDCMUL, self._t, _raw(t1), _raw(t2), s0=v):
            return self
        self._t.addcmul_(_raw(t1), _raw(t2), value=v)
        return self

    def addcdiv(self, *args):
        v, t1, t2 = args if len(args) == 3 else (1.0, *args)
        if self._native_ew(_tm.ADDCDIV, self._t, _raw(t1), _raw(t2), s0=v):
            return self
        self._t.addcdiv_(_raw(t1), _raw(t2), value=v)
        return self

    def negative(self, x=None):
        if self._native_ew(_tm.NEG, self._t if x is None else _raw(x)):
            return self
        return self._assign(-(self._t if x is None else _raw(x)))

    def inv(self):
        if self._native_ew(_tm.RECIP, self._t):
            return self
        self._t.reciprocal_()
        return self

    def clamp(self, minValue, maxValue):
        if self._native_ew(_tm.CLAMP, self._t, s0=minValue, s1=maxValue):
            return self
        self._t.clamp_(minValue, maxValue)
        return self

    def _unary(self, fn, x=None):
        """``fn``: a torch function, or the name of one the native backend implements (looked up at call time)."""
        src = self._t if x is None else _raw(x)
        name = _NATIVE_UNARY.get(fn) if isinstance(fn, str) else None
        if name is not None and self._native_ew(getattr(_tm, name), src):
            return self
        return self._assign((getattr(torch, fn) if isinstance(fn, str) else fn)(src))

    def abs(self, x=None):
        return self._unary("abs", x)

    def exp(self, x=None):
        return self._unary("exp", x)

    def log(self, x=None):
        return self._unary("log", x)

    def log1p(self, x=None):
        return self._unary("log1p", x)

    def sqrt(self, x=None):
        return self._unary("sqrt", x)

    def square(self, x=None):
        return self._unary("square", x)

    def tanh(self, x=None):
        return self._unary("tanh", x)

    def floor(self, x=None):
        return self._unary("floor", x)

    def ceil(self, x=None):
        return self._unary("ceil", x)

    def sign(self, x=None):
        return self._unary("sign", x)

    def erf(self, x=None):
        return self._unary(torch.erf, x)

    def erfc(self, x=None):
        return self._unary(torch.erfc, x)

    def logGamma(self, x=None):
        return self._unary(torch.lgamma, x)

    def digamma(self, x=None):
        return self._unary(torch.digamma, x)

    def pow(self, *args):
        if len(args) == 1:
            if isinstance(args[0], numbers.Number) and self._native_ew(_tm.POWS, self._t, s0=args[0]):
                return self
            self._t.pow_(args[0])
            return self
        if isinstance(args[1], numbers.Number) and self._native_ew(_tm.POWS, _raw(args[0]), s0=args[1]):
            return self
        return self._assign(torch.pow(_raw(args[0]), args[1]))

    # ------------------------------------------------------------------ BLAS
    def addmm(self, *args):
        """addmm(v1, M, v2, a, b) | addmm(M, a, b) | addmm(a, b) | addmm(v2, a, b) | addmm(v1, v2, a, b)."""
        if len(args) == 5:
            v1, M, v2, a, b = args
        elif len(args) == 4:
            v1, v2, a, b = args
            M = self._t
        elif len(args) == 3 and isinstance(args[0], numbers.Number):
            v1, M, v2, (a, b) = 1.0, self._t, args[0], args[1:]
        elif len(args) == 3:
            v1, M, v2, a, b = 1.0, args[0], 1.0, args[1], args[2]
        else:
            v1, M, v2, (a, b) = 1.0, self._t, 1.0, args
        if self._native_gemm(_raw(M), _raw(a), _raw(b), v1, v2):
            return self
        return self._assign(torch.addmm(_raw(M), _raw(a), _raw(b), beta=v1, alpha=v2))

    def _native_gemm(self, M, a, b, beta, alpha):
        """self = beta * M + alpha * a @ b (2-D, or 3-D batched) on the fp32 MFMA GEMM (ops/tensor_math.py)."""
        if not (_g32(a, b) and (M is None or _g32(M)) and a.dim() == b.dim() and a.dim() in (2, 3)):
            return False
        shape = tuple(a.shape[:-1]) + (b.shape[-1],)
        if a.shape[-1] != b.shape[-2] or (a.dim() == 3 and a.shape[0] != b.shape[0]):
            return False
        if M is not None and tuple(M.shape) != shape:
            try:
                M = M.expand(shape)
            except RuntimeError:
                return False
        t = self._t
        alias = lambda x: x.untyped_storage().data_ptr() == t.untyped_storage().data_ptr()  # noqa: E731
        if tuple(t.shape) != shape or not t.is_cuda or t.dtype != torch.float32 or alias(a) or alias(b) or (
                M is not None and alias(M) and (M.data_ptr() != t.data_ptr() or M.stride() != t.stride())):
            out = torch.empty(shape, device=a.device, dtype=torch.float32)
            _tm.gemm(out, a, b, M, alpha, beta)
            self.resize(list(shape))
            return self._native_ew(_tm.COPY, out) or bool(self._t.copy_(out) is not None)
        _tm.gemm(t, a, b, M, alpha, beta)
        return True

    def mm(self, a, b):
        if self._native_gemm(None, _raw(a), _raw(b), 0.0, 1.0):
            return self
        return self._assign(_raw(a) @ _raw(b))

    def addmv(self, *args):
        if len(args) == 5:
            v1, M, v2, a, b = args
        elif len(args) == 4:
            v1, v2, a, b = args
            M = self._t
        elif len(args) == 3:
            v2, a, b = args
            v1, M = 1.0, self._t
        else:
            v1, M, v2, (a, b) = 1.0, self._t, 1.0, args
        if self._native_gemv(_raw(M), _raw(a), _raw(b), v1, v2):
            return self
        return self._assign(torch.addmv(_raw(M), _raw(a), _raw(b), beta=v1, alpha=v2))

    def _native_gemv(self, M, a, x, beta, alpha):
        if not (_g32(a, x) and (M is None or _g32(M)) and a.dim() == 2 and x.dim() == 1 and a.shape[1] == x.shape[0]):
            return False
        m = a.shape[0]
        t = self._t
        if M is not None and tuple(M.shape) != (m,):
            return False
        alias = lambda y: y.untyped_storage().data_ptr() == t.untyped_storage().data_ptr()  # noqa: E731
        if tuple(t.shape) != (m,) or not _g32(t) or alias(a) or alias(x) or (
                M is not None and alias(M) and (M.data_ptr() != t.data_ptr() or M.stride() != t.stride())):
            out = torch.empty(m, device=a.device, dtype=torch.float32)
            _tm.gemv(out, a, x, M, alpha, beta)
            self.resize([m])
            return self._native_ew(_tm.COPY, out) or bool(self._t.copy_(out) is not None)
        _tm.gemv(t, a, x, M, alpha, beta)
        return True

    def mv(self, a, b):
        if self._native_gemv(None, _raw(a), _raw(b), 0.0, 1.0):
            return self
        return self._assign(_raw(a) @ _raw(b))

    def addr(self, *args):
        if len(args) == 5:
            v1, M, v2, x, y = args
        elif len(args) == 3:
            v2, x, y = args
            v1, M = 1.0, self._t
        else:
            v1, M, v2, (x, y) = 1.0, self._t, 1.0, args
        M, x, y = _raw(M), _raw(x), _raw(y)
        if (_g32(M, x, y) and x.dim() == 1 and y.dim() == 1 and tuple(M.shape) == (x.shape[0], y.shape[0])
                and tuple(self._t.shape) == tuple(M.shape)):
            m, n = M.shape
            if _tm.apply(_tm.AXPBYZ, self._t, M, x.view(m, 1).expand(m, n), y.view(1, n).expand(m, n), s0=v2, s1=v1):
                return self
        return self._assign(torch.addr(M, x, y, beta=v1, alpha=v2))

    def baddbmm(self, *args):
        if len(args) == 5:
            v1, M, v2, a, b = args
        elif len(args) == 4:
            v1, v2, a, b = args
            M = self._t
        else:
            v1, M, v2, (a, b) = 1.0, self._t, 1.0, args
        if self._native_gemm(_raw(M), _raw(a), _raw(b), v1, v2):
            return self
        return self._assign(torch.baddbmm(_raw(M), _raw(a), _raw(b), beta=v1, alpha=v2))

    def bmm(self, a, b):
        if self._native_gemm(None, _raw(a), _raw(b), 0.0, 1.0):
            return self
        return self._assign(torch.bmm(_raw(a), _raw(b)))

    def dot(self, y):
        yr = _raw(y)
        if _g32(self._t, yr) and self._t.numel() == yr.numel():
            prod = torch.empty(self._t.shape, device=self._t.device)
            if _tm.apply(_tm.MUL, prod, self._t, yr.reshape(self._t.shape)):
                return float(_tm.reduce(prod, _tm.R_SUM)[0])
        return float((self._t.reshape(-1).double() * yr.reshape(-1).double()).sum())

    # ------------------------------------------------------------------ reductions
    def _reduce_dim(self, fn, args):
        if not args:
            return fn(self._t, None)
        if isinstance(args[0], Tensor):
            x, dim = args
            return self._assign(fn(_raw(x), _d(dim)))
        return self._wrap(fn(self._t, _d(args[0])))

    @staticmethod
    def _nred(op, mean=False, fallback=None):
        """Reduction fn(t, d) on the native backend for fp32 GPU tensors (ops/tensor_math.reduce), else ``fallback``."""
        def fn(t, d):
            if _g32(t) and t.numel() > 0:
                v, _ = _tm.reduce(t, op, d, mean=mean)
                return float(v) if d is None else v
            return fallback(t, d)
        return fn

    def sum(self, *args):
        return self._reduce_dim(self._nred(_tm.R_SUM, fallback=lambda t, d: t.sum().item() if d is None
                                           else t.sum(d, keepdim=True)), args)

    def mean(self, *args):
        return self._reduce_dim(self._nred(_tm.R_SUM, True, lambda t, d: t.float().mean().item() if d is None
                                           else t.mean(d, keepdim=True)), args)

    def prod(self, *args):
        return self._reduce_dim(self._nred(_tm.R_PROD, fallback=lambda t, d: t.prod().item() if d is None
                                           else t.prod(d, keepdim=True)), args)

    def sumSquare(self):
        if _g32(self._t) and self._t.numel() > 0:
            return float(_tm.reduce(self._t, _tm.R_SUMSQ)[0])
        return float((self._t.double() ** 2).sum())

    def norm(self, *args):
        """norm(p) -> scalar | norm(y, p, dim) -> self = p-norm of y along dim."""
        if len(args) <= 1:
            p = args[0] if args else 2
            return float(torch.linalg.vector_norm(self._t.double().reshape(-1), ord=p))
        y, p, dim = args
        return self._assign(torch.linalg.vector_norm(_raw(y), ord=p, dim=_d(dim), keepdim=True))

    def dist(self, y, norm=2):
        return float(torch.linalg.vector_norm((self._t - _raw(y)).double().reshape(-1), ord=norm))

    def _minmax(self, fn, args):
        if not args:
            return fn(self._t).item()
        dim = args[0]
        vals, idx = (fn(self._t, _d(dim), keepdim=True) if not isinstance(dim, Tensor) else (None, None))
        # T-typed 1-based indices (the reference's representation), the same as the native fp32 GPU path
        return self._wrap(vals), self._wrap((idx + 1).to(self._t.dtype) if self._t.is_floating_point() else idx + 1)

    def _native_minmax(self, op, args):
        if not (_g32(self._t) and self._t.numel() > 0):
            return None
        if not args:
            return float(_tm.reduce(self._t, op)[0])
        if len(args) == 3:
            values, indices, dim = args
            v, i = _tm.reduce(self._t, op, _d(dim), want_index=True)
            values._assign(v)
            indices._assign(i.to(indices._t.dtype))
            return values, indices
        if isinstance(args[0], Tensor):
            return None
        v, i = _tm.reduce(self._t, op, _d(args[0]), want_index=True)
        return self._wrap(v), self._wrap(i)

    def max(self, *args):
        r = self._native_minmax(_tm.R_MAX, args)
        if r is not None:
            return r
        if len(args) == 3:     # max(values, indices, dim) on self
            values, indices, dim = args
            v, i = self._t.max(_d(dim), keepdim=True)
            values._assign(v)
            indices._assign((i + 1).to(indices._t.dtype))
            return values, indices
        return self._minmax(torch.max, args)

    def min(self, *args):
        r = self._native_minmax(_tm.R_MIN, args)
        if r is not None:
            return r
        if len(args) == 3:
            values, indices, dim = args
            v, i = self._t.min(_d(dim), keepdim=True)
            values._assign(v)
            indices._assign((i + 1).to(indices._t.dtype))
            return values, indices
        return self._minmax(torch.min, args)

    def topk(self, k, dim=-1, increase=True, result=None, indices=None, sortedResult=True):
        """k smallest (``increase=True``, the Torch7 default) or largest values along ``dim``; 1-based indices."""
        d = self._t.dim() - 1 if dim == -1 else _d(dim)
        r = _tm.topk(self._t, k, d, not increase)      # native in-LDS sort (always sorted) for fp32 GPU rows <= 8192
        if r is not None:
            v, i1 = r
        else:
            v, i = torch.topk(self._t, k, dim=d, largest=not increase, sorted=sortedResult)
            v, i1 = v.clone(), (i + 1).to(self._t.dtype)
        result = Tensor() if result is None else result
        indices = Tensor() if indices is None else indices
        result._set_t(v)
        indices._set_t(i1)
        return result, indices

    def numNonZeroByRow(self):
        return (self._t != 0).sum(dim=1).tolist()

    # ------------------------------------------------------------------ comparison / masking (results 1 / 0)
    def _cmp(self, fn, x, v):
        return self._assign(fn(_raw(x), _raw(v)).to(self._t.dtype))

    def gt(self, x, v):
        return self._cmp(torch.gt, x, v)

    def lt(self, x, v):
        return self._cmp(torch.lt, x, v)

    def le(self, x, v):
        return self._cmp(torch.le, x, v)

    def ge(self, x, v):
        return self._cmp(torch.ge, x, v)

    def eq(self, x, v):
        return self._cmp(torch.eq, x, v)

    def notEqualValue(self, v):
        return bool((self._t != v).any())

    def maskedFill(self, mask, e):
        if _tm.masked_fill(self._t, _raw(mask), e) is None:
            self._t.masked_fill_(_raw(mask).bool(), e)
        return self

    def maskedCopy(self, mask, y):
        if _tm.masked_copy(self._t, _raw(mask), _raw(y)) is None:
            m = _raw(mask).bool()
            self._t[m] = _raw(y).reshape(-1)[: int(m.sum())].to(self._t.dtype)
        return self

    def maskedSelect(self, mask, y):
        r = _tm.masked_select(self._t, _raw(mask))
        return y._set_t(r if r is not None else self._t[_raw(mask).bool()].clone())

    # ------------------------------------------------------------------ indexing (1-based index tensors)
    def index(self, dim, index, y):
        """self = y.index_select(dim, index) (TensorMath.scala index)."""
        r = _tm.index_select(_raw(y), _d(dim), _raw(index))
        if r is None:
            r = _raw(y).index_select(_d(dim), _raw(index).long().reshape(-1) - 1)
        return self._assign(r)

    def indexAdd(self, dim, index, y):
        if _tm.index_add(self._t, _d(dim), _raw(index), _raw(y)) is None:
            self._t.index_add_(_d(dim), _raw(index).long().reshape(-1) - 1, _raw(y))
        return self

    def gather(self, dim, index, src):
        r = _tm.gather(_raw(src), _d(dim), _raw(index))
        if r is None:
            r = torch.gather(_raw(src), _d(dim), _raw(index).long() - 1)
        return self._assign(r)

    def scatter(self, dim, index, src):
        if _tm.scatter(self._t, _d(dim), _raw(index), _raw(src)) is None:
            self._t.scatter_(_d(dim), _raw(index).long() - 1, _raw(src))
        return self

    # ------------------------------------------------------------------ conv
    def conv2(self, kernel, vf="V"):
        """2-D full ('F') or valid ('V') convolution (kernel flipped) — DenseTensorConv.scala:24."""
        return self._conv(kernel, vf, flip=True)

    def xcorr2(self, kernel, vf="V"):
        return self._conv(kernel, vf, flip=False)

    def _conv(self, kernel, vf, flip):
        x, k = self._t.double(), _raw(kernel).double()
        if flip:
            k = torch.flip(k, dims=(-2, -1))
        kh, kw = k.shape[-2:]
        pad = (kh - 1, kw - 1) if vf.upper() == "F" else (0, 0)
        y = torch.nn.functional.conv2d(x.reshape(1, 1, *x.shape[-2:]), k.reshape(1, 1, kh, kw), padding=pad)
        return self._wrap(y.reshape(y.shape[-2:]).to(self._t.dtype))

    # ------------------------------------------------------------------ misc
    def diff(self, other, count=1, reverse=False):
        """True when the tensors differ; prints up to ``count`` differing positions (Tensor.diff)."""
        a, b = self._t.reshape(-1), _raw(other).reshape(-1)
        d = (a != b).nonzero().reshape(-1)
        if reverse:
            d = d.flip(0)
        for i in d[:count].tolist():
            print(f"diff at {i + 1}: {a[i].item()} vs {b[i].item()}")
        return bool(d.numel())

    def almostEqual(self, other, delta):
        o = _raw(other)
        return list(o.shape) == list(self._t.shape) and bool(((self._t.double() - o.double()).abs() <= delta).all())

    def toBreezeMatrix(self):
        return self._t.detach().cpu().numpy()

    toBreezeVector = toMLlibMatrix = toMLlibVector = toBreezeMatrix

    def save(self, path, overWrite=False):
        import os
        if os.path.exists(path) and not overWrite:
            raise FileExistsError(path)
        torch.save(self._t.detach().cpu(), path)
        return self

    @staticmethod
    def load(path):
        return Tensor(torch.load(path, weights_only=True))

    # ------------------------------------------------------------------ python protocol
    def __getitem__(self, idx):
        r = self._t[idx]
        return r.item() if r.dim() == 0 else self._wrap(r)

    def __setitem__(self, idx, v):
        self._t[idx] = _raw(v)

    def __add__(self, o):
        return self._wrap(self._t + _raw(o))

    __radd__ = __add__

    def __sub__(self, o):
        return self._wrap(self._t - _raw(o))

    def __rsub__(self, o):
        return self._wrap(_raw(o) - self._t)

    def __mul__(self, o):
        return self._wrap(self._t * _raw(o))

    __rmul__ = __mul__

    def __truediv__(self, o):
        return self._wrap(self._t / _raw(o))

    def __neg__(self):
        return self._wrap(-self._t)

    def __eq__(self, other):
        if isinstance(other, (Tensor, torch.Tensor)):
            o = _raw(other)
            return list(o.shape) == list(self._t.shape) and bool(torch.equal(self._t, o.to(self._t.dtype)))
        return NotImplemented

    def __hash__(self):
        return id(self)

    def __iter__(self):
        for i in range(self._t.shape[0]):
            r = self._t[i]
            yield r.item() if r.dim() == 0 else self._wrap(r)

    def __repr__(self):
        return f"{self._t!r}\n[bigdl Tensor of size {'x'.join(map(str, self._t.shape))}]"


def _contig_strides(sizes):
    st, acc = [], 1
    for s in reversed(list(sizes)):
        st.append(acc)
        acc *= int(s)
    return list(reversed(st))


# ---------------------------------------------------------------------- factory (Tensor object, Tensor.scala:853)
def ones(*sizes, dtype=torch.float32):
    return Tensor(torch.ones(_sizes(sizes), dtype=dtype))


def zeros(*sizes, dtype=torch.float32):
    return Tensor(torch.zeros(_sizes(sizes), dtype=dtype))


def range_(xmin, xmax, step=1, dtype=torch.float32):
    """Inclusive range (Tensor.range)."""
    n = int(math.floor((xmax - xmin) / step)) + 1
    return Tensor(xmin + step * torch.arange(n, dtype=torch.float64).to(dtype))


def randperm(n, dtype=torch.float32):
    from ..utils.random_generator import RNG
    return Tensor((RNG.randperm(n) + 1).to(dtype))


def scalar(v, dtype=torch.float32):
    return Tensor(torch.tensor(v, dtype=dtype))


def gaussian1D(size=3, sigma=0.25, amplitude=1.0, normalize=False, mean=0.5, tensor=None):
    """1-D gaussian kernel (Tensor.gaussian1D, used by SpatialContrastiveNormalization)."""
    center = mean * size + 0.5
    i = torch.arange(1, size + 1, dtype=torch.float64)
    g = amplitude * torch.exp(-(((i - center) / (sigma * size)) ** 2) / 2)
    if normalize:
        g = g / g.sum()
    t = Tensor(g.float())
    if tensor is not None:
        tensor._set_t(t._t)
        return tensor
    return t


def unique(tensor, distinctTensor=None, indexTensor=None):
    """(distinct values in first-seen order, 1-based position of every element in the distinct list)."""
    vals = _raw(tensor).reshape(-1).tolist()
    seen = {}
    order, idx = [], []
    for v in vals:
        if v not in seen:
            seen[v] = len(order) + 1
            order.append(v)
        idx.append(seen[v])
    d = Tensor(torch.tensor(order, dtype=_raw(tensor).dtype))
    ix = Tensor(torch.tensor(idx, dtype=torch.int32))
    if distinctTensor is not None:
        distinctTensor._set_t(d._t)
        d = distinctTensor
    if indexTensor is not None:
        indexTensor._set_t(ix._t)
        ix = indexTensor
    return d, ix


def dense(sparse_t):
    return Tensor(_raw(sparse_t).to_dense())


def sparse(*args, dtype=torch.float32):
    """sparse(denseTensor) | sparse(indices (1-based, [nDim, nnz]), values, shape) -> COO SparseTensor."""
    if len(args) == 1:
        return SparseTensor(_raw(args[0]).to_sparse())
    indices, values, shape = args
    idx = torch.as_tensor(np.asarray(_raw(indices))).long() - 1
    return SparseTensor(torch.sparse_coo_tensor(idx, torch.as_tensor(_raw(values), dtype=dtype), list(shape)).coalesce())


class SparseTensor(Tensor):
    """COO sparse tensor (reference SparseTensor.scala:55; SparseTensorBLAS coomv / coomm)."""
    __slots__ = ()

    def nElement(self):
        return int(self._t._nnz())

    def getTensorType(self):
        return "SparseType"

    def toDense(self):
        return Tensor(self._t.to_dense())

    def indices(self):
        return Tensor(self._t.coalesce().indices() + 1)

    def values(self):
        return Tensor(self._t.coalesce().values())

    def narrow(self, dim, index, size):
        return SparseTensor(self._t.narrow_copy(_d(dim), index - 1, size))

    def mm(self, dense_t):
        return Tensor(torch.sparse.mm(self._t, _raw(dense_t)))


def to_torch(x):
    """Unwrap a bigdl Tensor (recursively through lists/tuples/Tables)."""
    if isinstance(x, Tensor):
        return x._t
    return x
