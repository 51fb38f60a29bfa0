"""``nn.ops``: forward-only operations for TF-style graphs and feature engineering.

Reference: S/nn/ops/*.scala (71 files). ``Operation`` (Operation.scala:32) is a module without a backward;
the element-wise / comparison / reduction / indexing ops reuse the TF-semantics table in ``tf_ops`` so a
graph built from these classes and one imported from a GraphDef run the same code on the GPU engine.
Feature-column ops (BucketizedCol, CategoricalColHashBucket, CategoricalColVocaList, CrossCol, IndicatorCol,
Kv2Tensor, MkString, Substr) operate on string columns, represented here as lists / numpy object arrays of
Python strings (the reference's ``Tensor[String]``); sparse results are ``bigdl_amd.tensor.SparseTensor``-
compatible torch sparse COO tensors (``isSparse=False`` densifies). ``TensorOp`` is the reference's composable
tensor-transform algebra (``TensorOp.sqrt -> TensorOp.add(1) * 2``).
"""
import bisect

import torch

from ..utils.table import Table
from .abstractnn import AbstractModule


class Operation(AbstractModule):
    """Module without a backward pass (reference Operation.scala:32-47)."""

    def updateGradInput(self, input, gradOutput):
        raise RuntimeError(f"{type(self).__name__}: Operation does not support updateGradInput()")

    def backward(self, input, gradOutput):
        raise RuntimeError(f"{type(self).__name__}: Operation does not support backward()")


def _table_inputs(x):
    if isinstance(x, Table):
        return [x[i] for i in range(1, x.length() + 1)]
    return [x]


class TFTableOp(Operation):
    """An op from the ``tf_ops.OPS`` table with fixed attributes; the input is one tensor or a Table."""

    op = None

    def __init__(self, **attrs):
        super().__init__()
        self.attrs = attrs

    def updateOutput(self, input):
        from .tf_ops import run_op

        with torch.no_grad():
            r = run_op(self.op, _table_inputs(input), self.attrs)
        if isinstance(r, (list, tuple)):
            return Table(*r)
        return r


def _op_class(name, op, doc):
    return type(name, (TFTableOp,), {"op": op, "__doc__": doc})


_SIMPLE = {
    # name: (tf op, doc)
    "Abs": "Abs", "Ceil": "Ceil", "Floor": "Floor", "Round": "Round", "Rint": "Rint", "Sign": "Sign",
    "Inv": "Inv", "Erf": "Erf", "Erfc": "Erfc", "Lgamma": "Lgamma", "Digamma": "Digamma", "Expm1": "Expm1",
    "Exp": "Exp", "IsFinite": "IsFinite", "IsInf": "IsInf", "IsNan": "IsNan", "LogicalNot": "LogicalNot",
    "Rank": "Rank", "L2Loss": "L2Loss",
    "Equal": "Equal", "NotEqual": "NotEqual", "Greater": "Greater", "GreaterEqual": "GreaterEqual",
    "Less": "Less", "LessEqual": "LessEqual", "LogicalAnd": "LogicalAnd", "LogicalOr": "LogicalOr",
    "Maximum": "Maximum", "Minimum": "Minimum", "FloorDiv": "FloorDiv", "FloorMod": "FloorMod",
    "TruncateDiv": "TruncateDiv", "Mod": "Mod", "Pow": "Pow", "SquaredDifference": "SquaredDifference",
    "BatchMatMul": "BatchMatMul", "Gather": "GatherV2", "Pad": "Pad", "Slice": "Slice", "Tile": "Tile",
    "Select": "Select", "SegmentSum": "SegmentSum", "RangeOps": "Range",
}
for _n, _op in _SIMPLE.items():
    globals()[_n] = _op_class(_n, _op, f"TF ``{_op}`` (reference nn/ops/{_n}.scala).")


class ApproximateEqual(TFTableOp):
    op = "ApproximateEqual"

    def __init__(self, tolerance=1e-5):
        super().__init__(tolerance=tolerance)


class _Reduce(TFTableOp):
    def __init__(self, keepDims=False, startFromZero=False):
        super().__init__(keep_dims=keepDims)
        self.startFromZero = startFromZero

    def updateOutput(self, input):
        xs = _table_inputs(input)
        if len(xs) > 1 and not self.startFromZero:           # reference axes are 1-based unless startFromZero
            ax = xs[1]
            xs[1] = torch.where(ax > 0, ax - 1, ax)
        from .tf_ops import run_op
        with torch.no_grad():
            return run_op(self.op, xs, self.attrs)


class Sum(_Reduce):
    op = "Sum"


class Prod(_Reduce):
    op = "Prod"


class Max(_Reduce):
    op = "Max"


class All(_Reduce):
    op = "All"


class Any(_Reduce):
    op = "Any"


class ArgMax(TFTableOp):
    """Table(input, dimension(0-based)) -> indices (int32, like the reference)."""

    op = "ArgMax"

    def __init__(self):
        super().__init__(output_type="DT_INT32")


class Cast(Operation):
    def __init__(self, dtype=torch.float32):
        super().__init__()
        self.dtype = dtype

    def updateOutput(self, input):
        return input.to(self.dtype)


class OneHot(TFTableOp):
    """Table(indices, depth, on_value, off_value) -> one-hot along ``axis``."""

    op = "OneHot"

    def __init__(self, axis=-1):
        super().__init__(axis=axis)


class TopK(Operation):
    """Top-k values and 1-based indices along the last dim (``startIndex`` shifts the index base)."""

    def __init__(self, k, sorted=True, startIndex=1):
        super().__init__()
        self.k, self.sorted, self.startIndex = k, sorted, startIndex

    def updateOutput(self, input):
        v, i = torch.topk(input, self.k, dim=-1, sorted=self.sorted)
        return Table(v, (i + self.startIndex).to(torch.int32))


class InTopK(Operation):
    """Table(predictions, targets) -> bool per row: target among the top-k (targets 1-based unless
    ``startFromZero``)."""

    def __init__(self, k, startFromZero=False):
        super().__init__()
        self.k, self.startFromZero = k, startFromZero

    def updateOutput(self, input):
        pred, tgt = input[1], input[2].long().reshape(-1)
        if not self.startFromZero:
            tgt = tgt - 1
        top = torch.topk(pred, self.k, dim=-1).indices
        return (top == tgt.unsqueeze(1)).any(1)


class Compare(Operation):
    """Base of the binary comparison ops: Table(a, b) -> bool tensor."""

    def compare(self, a, b):
        raise NotImplementedError

    def updateOutput(self, input):
        return self.compare(input[1], input[2])


class Dilation2D(TFTableOp):
    op = "Dilation2D"

    def __init__(self, strides, rates, padding):
        super().__init__(strides=list(strides), rates=list(rates), padding=padding)


class ResizeBilinearOps(TFTableOp):
    """Table(images NHWC, size) -> resized (ops/ResizeBilinear.scala)."""

    op = "ResizeBilinear"

    def __init__(self, alignCorner=False):
        super().__init__(align_corners=alignCorner)


class RandomUniform(Operation):
    """shape tensor -> uniform [minVal, maxVal) sample, re-drawn on every forward (never constant-folded)."""

    _random_node = True

    def __init__(self, minVal=0.0, maxVal=1.0, seed=None):
        super().__init__()
        self.minVal, self.maxVal, self.seed = minVal, maxVal, seed

    def updateOutput(self, input):
        from ..utils.random_generator import RNG
        return RNG.uniform(self.minVal, self.maxVal, tuple(int(v) for v in input.reshape(-1).tolist()))


class TruncatedNormal(Operation):
    _random_node = True

    def __init__(self, mean=0.0, stddev=1.0, seed=0):
        super().__init__()
        self.mean, self.stddev = mean, stddev

    def updateOutput(self, input):
        from .tf_ops import run_op
        return run_op("TruncatedNormal", [input], {}) * self.stddev + self.mean


class CrossEntropy(Operation):
    """Table(logits, labels(probabilities)) -> Table(per-row loss, dlogits)."""

    def updateOutput(self, input):
        from .tf_ops import run_op
        return Table(*run_op("SoftmaxCrossEntropyWithLogits", [input[1], input[2]], {}))


class DepthwiseConv2D(TFTableOp):
    """Table(input, filter[H, W, C, mult]) -> depthwise conv (ops/DepthwiseConv2D.scala)."""

    op = "DepthwiseConv2dNative"

    def __init__(self, strideW=1, strideH=1, padW=0, padH=0, dataFormat="NHWC"):
        super().__init__(strides=[1, strideH, strideW, 1] if dataFormat == "NHWC" else [1, 1, strideH, strideW],
                         padding="SAME" if padW == -1 else "VALID", data_format=dataFormat)


class ModuleToOperation(Operation):
    """Runs a module's forward as an operation (ModuleToOperation.scala)."""

    def __init__(self, module):
        super().__init__()
        self.module = module

    def updateOutput(self, input):
        return self.module.forward(input)


# ---------------------------------------------------------------------------------------------- TensorOp algebra
class TensorOp(Operation):
    """Composable tensor transform (TensorOp.scala): ``TensorOp.sqrt() -> TensorOp.add(1.0)`` via ``>>``
    (the reference's ``->``), plus arithmetic operators that append a step."""

    def __init__(self, transformer):
        super().__init__()
        self.transformer = transformer

    def updateOutput(self, input):
        return self.transformer(input.clone())

    def __rshift__(self, nxt):
        f, g = self.transformer, nxt.transformer
        return TensorOp(lambda t: g(f(t)))

    def _then(self, fn):
        return self >> TensorOp(fn)

    def __add__(self, v):
        return self._then(lambda t: t + v)

    def __sub__(self, v):
        return self._then(lambda t: t - v)

    def __mul__(self, v):
        return self._then(lambda t: t * v)

    def __truediv__(self, v):
        return self._then(lambda t: t / v)

    def __pow__(self, n):
        return self._then(lambda t: t ** n)

    def __ge__(self, v):
        return self._then(lambda t: (t >= v).to(t.dtype))

    def eq(self, v):
        return self._then(lambda t: (t == v).to(t.dtype))

    @property
    def t(self):
        return self._then(lambda t: t.t())

    @staticmethod
    def identity():
        return TensorOp(lambda t: t)

    @staticmethod
    def add(v):
        return TensorOp(lambda t: t + v)

    @staticmethod
    def sub(v):
        return TensorOp(lambda t: t - v)

    @staticmethod
    def mul(v):
        return TensorOp(lambda t: t * v)

    @staticmethod
    def div(v):
        return TensorOp(lambda t: t / v)

    @staticmethod
    def pow(n):
        return TensorOp(lambda t: t ** n)

    @staticmethod
    def ge(v):
        return TensorOp(lambda t: (t >= v).to(t.dtype))

    @staticmethod
    def transpose():
        return TensorOp(lambda t: t.t())

    @staticmethod
    def sqrt():
        return TensorOp(torch.sqrt)

    @staticmethod
    def log():
        return TensorOp(torch.log)

    @staticmethod
    def log1p():
        return TensorOp(torch.log1p)

    @staticmethod
    def exp():
        return TensorOp(torch.exp)

    @staticmethod
    def abs():
        return TensorOp(torch.abs)

    @staticmethod
    def floor():
        return TensorOp(torch.floor)

    @staticmethod
    def ceil():
        return TensorOp(torch.ceil)

    @staticmethod
    def negative():
        return TensorOp(torch.neg)

    @staticmethod
    def inv():
        return TensorOp(torch.reciprocal)

    @staticmethod
    def sigmoid():
        return TensorOp(torch.sigmoid)

    @staticmethod
    def tanh():
        return TensorOp(torch.tanh)

    @staticmethod
    def square():
        return TensorOp(torch.square)


# ---------------------------------------------------------------------------------------------- string hashing
def _rotl(x, r):
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF


def _mix_k(k):
    k = (k * 0xCC9E2D51) & 0xFFFFFFFF
    k = _rotl(k, 15)
    return (k * 0x1B873593) & 0xFFFFFFFF


def _mix(h, d):
    h ^= _mix_k(d)
    h = _rotl(h, 13)
    return (h * 5 + 0xE6546B64) & 0xFFFFFFFF


STRING_SEED = 0xF7CA7FD2


def murmur3_string_hash(s, seed=STRING_SEED):
    """Scala ``MurmurHash3.stringHash`` (UTF-16 code units mixed two at a time), as a signed 32-bit int. The
    reference's hashed feature columns (utils/HashFunc.scala) bucket this value, so the same strings land in
    the same buckets here."""
    units = s.encode("utf-16-le")
    cu = [units[i] | (units[i + 1] << 8) for i in range(0, len(units), 2)]
    h = seed & 0xFFFFFFFF
    i = 0
    while i + 1 < len(cu):
        h = _mix(h, ((cu[i] << 16) + cu[i + 1]) & 0xFFFFFFFF)
        i += 2
    if i < len(cu):
        h ^= _mix_k(cu[i])
    h ^= len(cu)
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h - (1 << 32) if h >= 1 << 31 else h


def string_hash_bucket(s, buckets, seed=STRING_SEED):
    """utils/HashFunc.stringHashBucket32: non-negative ``hash % buckets`` (Java remainder semantics)."""
    h = murmur3_string_hash(s, seed)
    v = int(h - buckets * int(h / buckets))      # truncated remainder like the JVM
    return v + buckets if v < 0 else v


def _str_rows(x):
    """String column -> list of Python strings (accepts lists, nested single-element lists, numpy arrays)."""
    import numpy as np

    if isinstance(x, torch.Tensor):
        x = x.reshape(-1).tolist()
    if isinstance(x, np.ndarray):
        x = x.reshape(-1).tolist()
    out = []
    for v in x:
        while isinstance(v, (list, tuple)) and len(v) == 1:
            v = v[0]
        out.append(v if isinstance(v, str) else (v.decode() if isinstance(v, bytes) else str(v)))
    return out


def _sparse(rows, cols, values, shape, dtype=torch.int32):
    idx = torch.tensor([rows, cols], dtype=torch.int64).reshape(2, -1)
    return torch.sparse_coo_tensor(idx, torch.tensor(values, dtype=dtype), tuple(shape)).coalesce()


class BucketizedCol(Operation):
    """Real values -> bucket ids given sorted ``boundaries`` (value == boundary goes to the upper bucket)."""

    def __init__(self, boundaries):
        super().__init__()
        if len(boundaries) < 1:
            raise ValueError("the length of boundaries must be at least 1")
        self.boundaries = [float(b) for b in boundaries]

    def updateOutput(self, input):
        b = torch.tensor(self.boundaries, dtype=torch.float64)
        return torch.bucketize(input.double(), b, right=True).to(torch.int32)


class CategoricalColHashBucket(Operation):
    """Delimited strings -> hash bucket ids [rows, max features] (sparse unless ``isSparse=False``)."""

    def __init__(self, hashBucketSize, strDelimiter=",", isSparse=True):
        super().__init__()
        self.hashBucketSize, self.strDelimiter, self.isSparse = hashBucketSize, strDelimiter, isSparse

    def updateOutput(self, input):
        rows, cols, vals, width = [], [], [], 0
        strs = _str_rows(input)
        for i, s in enumerate(strs):
            parts = s.split(self.strDelimiter)
            width = max(width, len(parts))
            for j, p in enumerate(parts):
                rows.append(i)
                cols.append(j)
                vals.append(string_hash_bucket(p, self.hashBucketSize))
        out = _sparse(rows, cols, vals, (len(strs), width))
        return out if self.isSparse else out.to_dense()


class CategoricalColVocaList(Operation):
    """Delimited strings -> vocabulary ids; out-of-vocabulary strings are dropped, mapped to ``len(vocab)``
    (``isSetDefault``) or hashed into ``numOovBuckets`` extra ids."""

    def __init__(self, vocaList, strDelimiter=",", isSetDefault=False, numOovBuckets=0):
        super().__init__()
        if numOovBuckets < 0:
            raise ValueError("numOovBuckets is negative")
        if isSetDefault and numOovBuckets != 0:
            raise ValueError("defaultValue and numOovBuckets are both specified")
        if not vocaList or len(set(vocaList)) != len(vocaList):
            raise ValueError("the vocabulary list is empty or has duplicates")
        self.vocaList = list(vocaList)
        self.voca = {v: i for i, v in enumerate(self.vocaList)}
        self.strDelimiter, self.isSetDefault, self.numOovBuckets = strDelimiter, isSetDefault, numOovBuckets

    def updateOutput(self, input):
        n = len(self.vocaList)
        width = (n + 1 if self.isSetDefault else n) if self.numOovBuckets == 0 else n + self.numOovBuckets
        rows, cols, vals = [], [], []
        strs = _str_rows(input)
        for i, s in enumerate(strs):
            parts = s.split(self.strDelimiter)
            if not self.isSetDefault and self.numOovBuckets == 0:
                parts = [p for p in parts if p in self.voca]
            for j, p in enumerate(parts):
                if self.numOovBuckets == 0:
                    v = self.voca.get(p, n)
                else:
                    v = self.voca.get(p, string_hash_bucket(p, self.numOovBuckets) + n)
                rows.append(i)
                cols.append(j)
                vals.append(v)
        return _sparse(rows, cols, vals, (len(strs), width))


class CrossCol(Operation):
    """Table of string columns -> hashed crosses of their values, one sparse row per example."""

    def __init__(self, hashBucketSize, strDelimiter=","):
        super().__init__()
        self.hashBucketSize, self.strDelimiter = hashBucketSize, strDelimiter

    @staticmethod
    def _recombine(parts):
        # the reference enumerates combinations with a LIFO stack (last value of each column first)
        stack = [[p] for p in parts[0]]
        out = []
        while stack:
            cur = stack.pop()
            children = [cur + [nxt] for nxt in parts[len(cur)]]
            if len(cur) == len(parts) - 1:
                out.extend(children)
            else:
                stack.extend(children)
        return out

    def _hash(self, combo):
        h = murmur3_string_hash(combo[0])
        for s in combo[1:]:
            h = murmur3_string_hash(s, h & 0xFFFFFFFF)
        b = self.hashBucketSize
        v = int(h - b * int(h / b))
        return v + b if v < 0 else v

    def updateOutput(self, input):
        cols_in = [_str_rows(c) for c in _table_inputs(input)]
        if len(cols_in) < 2:
            raise ValueError("CrossCol needs at least two columns")
        rows, cols, vals, width = [], [], [], 1
        for i in range(len(cols_in[0])):
            parts = [c[i].split(self.strDelimiter) for c in cols_in]
            combos = self._recombine(parts)
            width = max(width, len(combos))
            for m, combo in enumerate(combos):
                rows.append(i)
                cols.append(m)
                vals.append(self._hash(combo))
        return _sparse(rows, cols, vals, (len(cols_in[0]), width))


class IndicatorCol(Operation):
    """Sparse ids [rows, k] -> dense multi-hot (or counts when ``isCount``) [rows, feaLen]."""

    def __init__(self, feaLen, isCount=True, dtype=torch.float32):
        super().__init__()
        self.feaLen, self.isCount, self.dtype = feaLen, isCount, dtype

    def updateOutput(self, input):
        sp = input.coalesce() if input.is_sparse else input.to_sparse().coalesce()
        r, v = sp.indices()[0], sp.values().long()
        if bool((v >= self.feaLen).any()):
            raise ValueError("the parameter feaLen is set too small")
        out = torch.zeros(sp.shape[0], self.feaLen, dtype=self.dtype)
        if self.isCount:
            out.index_put_((r, v), torch.ones(v.numel(), dtype=self.dtype), accumulate=True)
        else:
            out[r, v] = 1
        return out


class Kv2Tensor(Operation):
    """Table(strings "k:v,k:v", feaLen) -> [rows, feaLen] values; ``transType`` 0 dense, 1 sparse."""

    def __init__(self, kvDelimiter=",", itemDelimiter=":", transType=0, dtype=torch.float32):
        super().__init__()
        self.kvDelimiter, self.itemDelimiter, self.transType, self.dtype = kvDelimiter, itemDelimiter, transType, dtype

    def updateOutput(self, input):
        strs = _str_rows(input[1])
        fea_len = int(torch.as_tensor(input[2]).reshape(-1)[0])
        rows, cols, vals = [], [], []
        for i, s in enumerate(strs):
            for kv in s.split(self.kvDelimiter):
                k, v = kv.split(self.itemDelimiter)[:2]
                rows.append(i)
                cols.append(int(k))
                vals.append(float(v))
        sp = _sparse(rows, cols, vals, (len(strs), fea_len), self.dtype)
        return sp.to_dense() if self.transType == 0 else sp


class MkString(Operation):
    """[rows, n] tensor -> list of delimiter-joined strings, one per row."""

    def __init__(self, strDelimiter=","):
        super().__init__()
        self.strDelimiter = strDelimiter

    def updateOutput(self, input):
        if input.is_sparse:
            input = input.to_dense()
        rows = input.reshape(input.shape[0], -1).tolist()
        return [self.strDelimiter.join(_fmt_num(v) for v in r) for r in rows]


def _fmt_num(v):
    return str(int(v)) if float(v).is_integer() and not isinstance(v, float) else str(v)


class Substr(Operation):
    """Table(strings, pos(0-based), len) -> substrings."""

    def updateOutput(self, input):
        strs = _str_rows(input[1])
        pos = int(torch.as_tensor(input[2]).reshape(-1)[0])
        ln = int(torch.as_tensor(input[3]).reshape(-1)[0])
        return [s[pos:pos + ln] for s in strs]


__all__ = ["Operation", "TFTableOp", "TensorOp", "ModuleToOperation", "Compare", "ApproximateEqual", "Sum", "Prod",
           "Max", "All", "Any", "ArgMax", "Cast", "OneHot", "TopK", "InTopK", "Dilation2D", "ResizeBilinearOps",
           "RandomUniform", "TruncatedNormal", "CrossEntropy", "DepthwiseConv2D", "BucketizedCol",
           "CategoricalColHashBucket", "CategoricalColVocaList", "CrossCol", "IndicatorCol", "Kv2Tensor", "MkString",
           "Substr", "murmur3_string_hash", "string_hash_bucket"] + list(_SIMPLE)
