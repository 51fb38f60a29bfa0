"""Native TensorMath backend for fp32 GPU tensors (csrc/tensor_math.hip), used by the 1-based Tensor API.

Reference: S/tensor/DenseTensorApply.scala:19 (strided apply1/2/3), S/tensor/DenseTensorMath.scala (element ops,
dimension reductions) and the MKL BLAS entry points of S/tensor/TensorMath.scala (addmm / addmv / addr / baddbmm /
dot). ``native_ok(*tensors)`` says whether a call can take this path (every tensor fp32 on the GPU); the Tensor API
falls back to torch for other dtypes and for the CPU engine.
"""
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


__all__ = ["native_ok", "apply", "reduce", "gemm", "gemv"]
