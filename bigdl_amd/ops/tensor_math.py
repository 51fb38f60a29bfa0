"""Native TensorMath backend for fp32 GPU tensors (csrc/tensor_math.hip), used by the 1-based Tensor API.

Reference: S/tensor/DenseTensorApply.scala:19 (strided apply1/2/3), S/tensor/DenseTensorMath.scala (element ops,
dimension reductions) and the MKL BLAS entry points of S/tensor/TensorMath.scala (addmm / addmv / addr / baddbmm /
dot). ``native_ok(*tensors)`` says whether a call can take this path (every tensor fp32 on the GPU); the Tensor API
falls back to torch for other dtypes and for the CPU engine.
"""
import os

import torch
from torch.autograd.graph import increment_version

from . import native

# element ops (csrc/tensor_math.hip enum Op)
COPY, FILL, ADDS, MULS, NEG, ABS, EXP, LOG, LOG1P, SQRT, SQUARE, TANH, FLOOR, CEIL, SIGN, RECIP, POWS, CLAMP, \
    SIGMOID, DIVS = range(20)
ADD, SUB, MUL, DIV, MAX, MIN, POW = range(32, 39)
ADDCMUL, ADDCDIV, AXPBYZ = range(64, 67)
# reductions (enum RedOp)
R_SUM, R_PROD, R_MAX, R_MIN, R_SUMSQ, R_ABSPOW = range(6)


def native_ok(*ts):
    return all(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 for t in ts if t is not None)


def _collapse(shape, strides_list):
    """Drop size-1 dims and merge adjacent dims that are contiguous for EVERY operand."""
    dims = [(s, [st[k] for st in strides_list]) for k, s in enumerate(shape) if s != 1]
    out = []
    for s, sts in dims:
        if out:
            ps, psts = out[-1]
            if all(pst == st * s for pst, st in zip(psts, sts)):
                out[-1] = (ps * s, sts)
                continue
        out.append((s, sts))
    return [s for s, _ in out], [[sts[i] for _, sts in out] for i in range(len(strides_list))]


def apply(op, out, a=None, b=None, c=None, s0=0.0, s1=0.0):
    """out = op(a, b, c) element-wise; a / b / c are broadcast to out's shape (zero strides). Returns False when the
    collapsed geometry exceeds 6 dims or aliasing would make the result order-dependent (caller falls back)."""
    shape = tuple(out.shape)
    ops = [t.expand(shape) if t is not None else None for t in (a, b, c)]
    present = [t for t in ops if t is not None]
    for t in present:       # an input that overlaps the output without being the very same view is unsafe
        if t.data_ptr() != out.data_ptr() and _overlaps(t, out):
            return False
        if t.data_ptr() == out.data_ptr() and t.stride() != out.stride():
            return False
    strides = [list(out.stride())] + [list(t.stride()) for t in present]
    size, sts = _collapse(shape, strides)
    if len(size) > 6:
        return False
    it = iter(sts[1:])
    sa, sb, sc = ([] if t is None else next(it) for t in ops)
    contiguous = out.is_contiguous() and all(t.is_contiguous() for t in present)
    native.get().tensor_apply(out, ops[0], ops[1], ops[2], size, sts[0], sa, sb, sc, int(op), float(s0), float(s1),
                              contiguous)
    increment_version(out)      # written through a raw pointer: keep version-keyed caches (Module.w16) honest
    return True


def _overlaps(t, out):
    if t.numel() == 0 or out.numel() == 0:
        return False
    def span(x):
        lo = x.data_ptr()
        hi = lo + sum((s - 1) * abs(st) for s, st in zip(x.shape, x.stride())) * x.element_size()
        return lo, hi
    a0, a1 = span(t)
    b0, b1 = span(out)
    return t.untyped_storage().data_ptr() == out.untyped_storage().data_ptr() and a0 <= b1 and b0 <= a1


def reduce(x, op, dim=None, p=2.0, mean=False, want_index=False):
    """Reduction of fp32 GPU ``x`` over 0-based ``dim`` (keepdim) or over everything (dim None -> 0-d values).
    Returns (values, 1-based float indices or None)."""
    xc = x if x.is_contiguous() else x.contiguous()
    if dim is None:
        outer, R, inner = 1, xc.numel(), 1
        oshape = ()
    else:
        outer = 1
        for s in xc.shape[:dim]:
            outer *= s
        R = xc.shape[dim]
        inner = 1
        for s in xc.shape[dim + 1:]:
            inner *= s
        oshape = tuple(xc.shape[:dim]) + (1,) + tuple(xc.shape[dim + 1:])
    out = torch.empty(oshape, device=x.device, dtype=torch.float32)
    outi = torch.empty(oshape, device=x.device, dtype=torch.float32) if want_index else None
    rows = outer * inner
    chunks = 1
    if R >= 4096 and rows < 4096:       # long rows over few outputs: spread each row over many workgroups
        chunks = int(min(1024, max(1, R // 2048), max(1, 8192 // max(rows, 1))))
    ws = torch.empty(chunks * rows * 3 + 1, device=x.device, dtype=torch.float32) if chunks > 1 else None
    native.get().tensor_reduce(xc, outer, R, inner, int(op), float(p), out, outi, bool(mean), ws, chunks)
    return out, outi


def gemm(C, A, B, M=None, alpha=1.0, beta=0.0):
    """C = beta * M + alpha * A @ B for 2-D or batched 3-D fp32 GPU operands (any strides, C written in place)."""
    if A.dim() == 2:
        A3, B3, C3 = A.unsqueeze(0), B.unsqueeze(0), C.unsqueeze(0)
        M3 = M.unsqueeze(0) if M is not None else None
    else:
        A3, B3, C3, M3 = A, B, C, M
    bt, m, k = A3.shape
    n = B3.shape[2]
    if M3 is not None:
        M3 = M3.expand(bt, m, n)
    s = [A3.stride(1), A3.stride(2), B3.stride(1), B3.stride(2), C3.stride(1), C3.stride(2),
         M3.stride(1) if M3 is not None else 0, M3.stride(2) if M3 is not None else 0,
         A3.stride(0) if bt > 1 else 0, B3.stride(0) if bt > 1 else 0, C3.stride(0) if bt > 1 else 0,
         M3.stride(0) if (M3 is not None and bt > 1) else 0]
    native.get().gemm_f32(A3, B3, M3, C3, bt, m, n, k, s, float(alpha), float(beta if M3 is not None else 0.0))
    increment_version(C)
    return C


def gemv(y, A, x, M=None, alpha=1.0, beta=0.0):
    m, k = A.shape
    Mv = M.expand(m) if M is not None else None
    s = [A.stride(0), A.stride(1), x.stride(0), Mv.stride(0) if Mv is not None else 0, y.stride(0)]
    native.get().gemv_f32(A, x, Mv, y, m, k, s, float(alpha), float(beta if Mv is not None else 0.0))
    increment_version(y)
    return y


# ------------------------------------------------------------------------------------- index / sort / mask ops
# csrc/index_ops.hip. Every function returns None when the operands do not qualify (non-contiguous in-place
# target, index not a 1-based fp32 / int64 cuda tensor, row too long for the in-LDS sort): the caller uses torch.
_ERR = {}


def _orc(shape, dim):
    outer = 1
    for s in shape[:dim]:
        outer *= s
    inner = 1
    for s in shape[dim + 1:]:
        inner *= s
    return outer, shape[dim], inner


def _idx_ok(idx):
    return isinstance(idx, torch.Tensor) and idx.is_cuda and idx.dtype in (torch.float32, torch.int64)


def _err(dev):
    """None: the kernels report out-of-range indices into the process's host-mapped error word (host_word slot 1)."""
    return None


# BIGDL_INDEX_CHECK: 1 (default) raise IndexError right after the op (one stream synchronisation, the reference's
# DenseTensor 'index out of bound' semantics); 0 = deferred: an error surfaces at the next index op / check_index_errors()
_INDEX_SYNC = os.environ.get("BIGDL_INDEX_CHECK", "1") != "0"


def check_index_errors(sync=True):
    """Raise IndexError if an index kernel met a 1-based index outside its dimension since the last check."""
    if sync:
        torch.cuda.current_stream().synchronize()
    if native.get().host_word(1, True):
        raise IndexError("index out of bound (1-based index outside the indexed dimension)")


def _index_op(*args):
    check_index_errors(sync=False)           # a deferred error of an earlier op surfaces first
    native.get().index_op(*args)
    if _INDEX_SYNC:
        check_index_errors(sync=True)


def _c(t):
    if t.is_contiguous():
        return t
    out = torch.empty(t.shape, dtype=t.dtype, device=t.device)
    if t.dtype == torch.float32 and apply(COPY, out, t):
        return out
    return t.contiguous()


def index_select(src, dim, idx):
    """out = src.index_select(dim, idx - 1) with a 1-based index vector."""
    if not (native_ok(src) and _idx_ok(idx)):
        return None
    idx = _c(idx.reshape(-1))
    src = _c(src)
    outer, R, inner = _orc(tuple(src.shape), dim)
    shape = list(src.shape)
    shape[dim] = idx.numel()
    out = torch.empty(shape, device=src.device, dtype=torch.float32)
    _index_op(0, None, idx, src, out, outer, R, idx.numel(), inner, 0, _err(src.device))
    return out


def index_add(dst, dim, idx, src):
    """dst.index_add_(dim, idx - 1, src) in place (duplicate indices accumulate)."""
    if not (native_ok(dst, src) and _idx_ok(idx) and dst.is_contiguous()):
        return None
    idx = _c(idx.reshape(-1))
    src = _c(src)
    outer, R, inner = _orc(tuple(dst.shape), dim)
    if src.numel() != outer * idx.numel() * inner:
        return None
    _index_op(1, dst, idx, src, None, outer, R, idx.numel(), inner, 0, _err(dst.device))
    increment_version(dst)
    return dst


def gather(src, dim, idx):
    """out[..., j, ...] = src[..., idx[..., j, ...] - 1, ...] (idx shaped like the output; other dims = src's)."""
    if not (native_ok(src) and _idx_ok(idx)) or idx.dim() != src.dim():
        return None
    if any(idx.shape[d] != src.shape[d] for d in range(src.dim()) if d != dim):
        return None
    idx, src = _c(idx), _c(src)
    outer, R, inner = _orc(tuple(src.shape), dim)
    out = torch.empty(idx.shape, device=src.device, dtype=torch.float32)
    _index_op(2, None, idx, src, out, outer, R, idx.shape[dim], inner, 0, _err(src.device))
    return out


def scatter(dst, dim, idx, src):
    """dst[..., idx[..., j, ...] - 1, ...] = src[..., j, ...] in place."""
    if not (native_ok(dst, src) and _idx_ok(idx) and dst.is_contiguous()) or idx.dim() != dst.dim():
        return None
    if any(idx.shape[d] != dst.shape[d] for d in range(dst.dim()) if d != dim) or src.dim() != dst.dim():
        return None
    if any(src.shape[d] != idx.shape[d] for d in range(dst.dim()) if d != dim) or src.shape[dim] < idx.shape[dim]:
        return None
    idx, src = _c(idx), _c(src)
    outer, R, inner = _orc(tuple(dst.shape), dim)
    _index_op(3, dst, idx, src, None, outer, R, idx.shape[dim], inner, src.shape[dim], _err(dst.device))
    increment_version(dst)
    return dst


def masked_fill(x, mask, v):
    if not (native_ok(x, mask) and x.is_contiguous() and mask.numel() == x.numel()):
        return None
    native.get().masked_fill(x, _c(mask).reshape(-1), float(v))
    increment_version(x)
    return x


def _mask_counts(mask):
    C = native.get()
    counts = torch.empty(C.mask_blocks(mask.numel()) + 1, dtype=torch.int32, device=mask.device)
    C.mask_scan(mask, counts)
    return counts


def masked_select(x, mask):
    """1-D tensor of x's elements where mask != 0, in element order (one host read of the count)."""
    if not (native_ok(x, mask) and mask.numel() == x.numel()):
        return None
    x, mask = _c(x), _c(mask)
    counts = _mask_counts(mask)
    n = int(counts.narrow(0, counts.numel() - 1, 1).item())
    out = torch.empty(n, device=x.device, dtype=torch.float32)
    if n:
        native.get().mask_write(False, x, mask, None, out, counts)
    return out


def masked_copy(x, mask, src):
    """x[mask != 0] = the first elements of src, in element order, in place."""
    if not (native_ok(x, mask, src) and x.is_contiguous() and mask.numel() == x.numel()):
        return None
    mask, src = _c(mask), _c(src)
    counts = _mask_counts(mask)
    n = int(counts.narrow(0, counts.numel() - 1, 1).item())
    if src.numel() < n:           # torch masked_scatter_ / the reference's maskedCopy raise here
        raise RuntimeError(f"maskedCopy: source has {src.numel()} elements, the mask selects {n}")
    native.get().mask_write(True, x, mask, src.reshape(-1), None, counts)
    increment_version(x)
    return x


def topk(x, k, dim, largest):
    """(values, 1-based fp32 indices) of the k smallest / largest along ``dim``, sorted; None for rows > 8192."""
    if not native_ok(x) or x.dim() == 0:
        return None
    outer, R, inner = _orc(tuple(x.shape), dim)
    if R > 8192 or k > R or k <= 0:
        return None
    x = _c(x)
    shape = list(x.shape)
    shape[dim] = k
    vals = torch.empty(shape, device=x.device, dtype=torch.float32)
    inds = torch.empty(shape, device=x.device, dtype=torch.float32)
    if not native.get().topk_f32(x, outer, R, inner, k, bool(largest), vals, inds):
        return None
    return vals, inds


__all__ = ["native_ok", "apply", "reduce", "gemm", "gemv", "index_select", "index_add", "gather", "scatter",
           "masked_fill", "masked_select", "masked_copy", "topk"]
