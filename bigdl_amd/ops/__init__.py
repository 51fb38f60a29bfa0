"""bigdl_amd.ops — the numeric backend.

Every GPU tensor op here launches a hand-written gfx950 HIP kernel from ``bigdl_amd/_C`` (csrc/*.hip);
CPU tensors use the fp32 torch reference implementation (the "local CPU engine"). This replaces the
reference's MKL / MKL-DNN / BigQuant JNI layer.
"""
import torch

from . import native  # noqa: F401
from . import conv, bn, pool  # noqa: F401

BF16 = torch.bfloat16
CL = torch.channels_last


def zeros(*shape, device=None, dtype=torch.float32, memory_format=None):
    """torch.zeros without the aten fill kernel on the GPU: one native fill kernel (graph-capture safe)."""
    if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
        shape = tuple(shape[0])
    kw = {"memory_format": memory_format} if memory_format is not None else {}
    t = torch.empty(shape, dtype=dtype, device=device, **kw)
    if t.is_cuda:
        native.get().fill_bytes(t, 0)
    else:
        t.zero_()
    return t


def zero_(t):
    """In-place zero without a memset node or aten fill on the GPU (dense tensors); returns t."""
    if t.is_cuda and (t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last))):
        native.get().fill_bytes(t, 0)
    else:
        t.zero_()
    return t


def is_gpu(t):
    return isinstance(t, torch.Tensor) and t.is_cuda


def relu_gpu(x, out=None):
    if out is None:
        out = torch.empty_like(x)
    native.get().relu_fwd(x, out)
    return out


def relu_bwd_gpu(dy, y, out=None):
    if out is None:
        out = torch.empty_like(y)
    if dy.dtype != BF16:
        dy = dy.to(BF16)
    dy = dy.contiguous(memory_format=_fmt(y))
    native.get().relu_bwd(dy, y, out)
    return out


def add_gpu(a, b, out=None):
    if b.stride() != a.stride():
        b = b.contiguous(memory_format=_fmt(a))
    if out is None:
        out = torch.empty_like(a)
    native.get().add_bf16(a, b, out)
    return out


def _fmt(t):
    if t.dim() == 4 and t.is_contiguous(memory_format=CL) and not t.is_contiguous():
        return CL
    return torch.contiguous_format


def to_bf16(x):
    if x.dtype == BF16:
        return x
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=BF16, device=x.device)
    native.get().cast_f32_bf16(x, y)
    return y


def to_f32(x):
    if x.dtype == torch.float32:
        return x
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    native.get().cast_bf16_f32(x, y)
    return y


def softmax_xent_gpu(logits, labels, label_base=1.0, size_average=True, need_grad=True):
    """Fused LogSoftMax + ClassNLL (CrossEntropyCriterion). Returns (loss[1] fp32, dlogits or None)."""
    B = logits.shape[0]
    logits = logits.contiguous()
    labels = labels.to(dtype=torch.float32).contiguous()
    loss = torch.empty(1, dtype=torch.float32, device=logits.device)
    native.get().fill_bytes(loss, 0)
    dl = torch.empty_like(logits) if need_grad else None
    scale = 1.0 / B if size_average else 1.0
    native.get().softmax_xent(logits, labels, loss, dl, float(label_base), float(scale))
    return loss, dl
