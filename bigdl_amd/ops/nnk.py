"""Autograd-aware wrappers of the misc NN kernels (csrc/nn_misc.hip) with the fp32 torch reference for CPU.

GPU tensors always run the native kernel (``native.get()`` raises if the extension is missing); CPU tensors run
the reference formula in torch. Both follow the BigDL semantics:
* LRN across channels: window ``[c - (size-1)//2, c - (size-1)//2 + size - 1]`` (S/nn/SpatialCrossMapLRN.scala:43),
  ``scale = k + alpha/size * sum x^2``, ``y = x * scale^-beta``;
* Dropout keeps with probability ``1-p`` (S/nn/Dropout.scala:44); on the GPU the keep-mask comes from a
  Philox counter stream keyed by a per-call seed and is regenerated in backward (nothing stored);
* ResizeBilinear: TF legacy sampling ``src = dst * in/out`` (``(in-1)/(out-1)`` with align_corners), lower index
  clamped, upper ``min(lower+1, in-1)`` (S/nn/ResizeBilinear.scala:266-280);
* LogSoftMax over the last dim (S/nn/LogSoftMax.scala:49);
* fp32 -> bf16 by truncation (S/parameters/FP16CompressedTensor.scala:271).
"""
import torch

from . import native


def _gpu(t):
    return isinstance(t, torch.Tensor) and t.is_cuda


# ---------------------------------------------------------------------------------------------- LRN
def lrn_cpu(x, size, alpha, beta, k):
    pre = (size - 1) // 2
    sq = (x * x).unsqueeze(1)                                   # N 1 C H W
    sq = torch.nn.functional.pad(sq, (0, 0, 0, 0, pre, size - pre - 1))
    win = torch.nn.functional.avg_pool3d(sq, (size, 1, 1), stride=1).squeeze(1) * size
    return x * (k + alpha / size * win).pow(-beta)


class _LRN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, size, alpha, beta, k):
        x = x.contiguous()
        y = torch.empty_like(x)
        scale = torch.empty_like(x)
        native.get().lrn_fwd(x, y, scale, size, alpha, beta, k)
        ctx.save_for_backward(x, y, scale)
        ctx.p = (size, alpha, beta)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, y, scale = ctx.saved_tensors
        gx = torch.empty_like(x)
        size, alpha, beta = ctx.p
        native.get().lrn_bwd(x, y, scale, gy.contiguous().float(), gx, size, alpha, beta)
        return gx, None, None, None, None


def lrn(x, size, alpha, beta, k):
    """x: [N, C, H, W] (or [C, H, W]) fp32."""
    squeeze = x.dim() == 3
    if squeeze:
        x = x.unsqueeze(0)
    xf = x.float()
    y = _LRN.apply(xf, int(size), float(alpha), float(beta), float(k)) if _gpu(x) else lrn_cpu(xf, size, alpha, beta, k)
    return y.squeeze(0) if squeeze else y


# ---------------------------------------------------------------------------------------------- dropout
_seed_counter = [0x5EED]


def next_seed():
    from ..utils.random_generator import RNG

    _seed_counter[0] += 1
    return ((RNG.random() & 0x7FFFFFFF) << 32) | (_seed_counter[0] & 0xFFFFFFFF)     # deterministic under RNG.setSeed


def dropout_gpu(x, p, scale, seed, out=None):
    """y = x * keep(seed) [/ (1-p)]; call again with the same seed on dy for the backward."""
    x = x.contiguous()
    out = torch.empty_like(x) if out is None else out
    mul = 1.0 / (1.0 - p) if scale else 1.0
    native.get().dropout(x, out, float(p), float(mul), int(seed) & 0x7FFFFFFFFFFFFFFF)
    return out


# ---------------------------------------------------------------------------------------------- embedding
def embedding_fwd_gpu(weight, idx):
    """idx: int64 0-based (negative -> zero row)."""
    idx = idx.contiguous()
    out = torch.empty(tuple(idx.shape) + (weight.shape[1],), device=weight.device, dtype=torch.float32)
    native.get().embedding_fwd(weight.contiguous(), idx, out)
    return out


def embedding_bwd_gpu(grad_weight, idx, gout, scale=1.0):
    native.get().embedding_bwd(gout.contiguous().float(), idx.contiguous(), grad_weight, float(scale))


# ---------------------------------------------------------------------------------------------- bilinear resize
def _scales(H, W, OH, OW, align):
    sh = (H - 1) / (OH - 1) if align and OH > 1 else H / OH
    sw = (W - 1) / (OW - 1) if align and OW > 1 else W / OW
    return sh, sw


def resize_bilinear_cpu(x, OH, OW, align):
    N, C, H, W = x.shape
    sh, sw = _scales(H, W, OH, OW, align)

    def axis(o, n, s):
        src = torch.arange(o, dtype=torch.float32) * s
        lo = src.floor().long().clamp(max=n - 1)
        hi = (lo + 1).clamp(max=n - 1)
        return lo, hi, src - lo.float()

    h0, h1, fh = axis(OH, H, sh)
    w0, w1, fw = axis(OW, W, sw)
    fw = fw.view(1, 1, 1, OW)
    fh = fh.view(1, 1, OH, 1)
    top = x[:, :, h0][..., w0] + (x[:, :, h0][..., w1] - x[:, :, h0][..., w0]) * fw
    bot = x[:, :, h1][..., w0] + (x[:, :, h1][..., w1] - x[:, :, h1][..., w0]) * fw
    return top + (bot - top) * fh


class _Resize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, OH, OW, align):
        x = x.contiguous()
        N, C, H, W = x.shape
        sh, sw = _scales(H, W, OH, OW, align)
        y = torch.empty(N, C, OH, OW, device=x.device, dtype=torch.float32)
        native.get().resize_bilinear_fwd(x, y, sh, sw)
        ctx.geo = (N, C, H, W, sh, sw)
        return y

    @staticmethod
    def backward(ctx, gy):
        N, C, H, W, sh, sw = ctx.geo
        gx = torch.zeros(N, C, H, W, device=gy.device, dtype=torch.float32)
        native.get().resize_bilinear_bwd(gy.contiguous().float(), gx, sh, sw)
        return gx, None, None, None


def resize_bilinear(x, OH, OW, align=False):
    """x: NCHW -> NCHW fp32, BigDL / TF-legacy sampling."""
    xf = x.float()
    return _Resize.apply(xf, int(OH), int(OW), bool(align)) if _gpu(x) else resize_bilinear_cpu(xf, OH, OW, align)


# ---------------------------------------------------------------------------------------------- log-softmax
class _LogSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        y = torch.empty_like(x)
        native.get().log_softmax_fwd(x, y)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        gx = torch.empty_like(y)
        native.get().log_softmax_bwd(y, gy.contiguous().float(), gx)
        return gx


def log_softmax(x):
    """Log-softmax over the last dimension."""
    xf = x.float()
    return _LogSoftmax.apply(xf) if _gpu(x) else torch.log_softmax(xf, -1)


class _Softmax(torch.autograd.Function):
    """softmax = exp(log-softmax) on the native row kernel and the TensorMath backend (ops/tensor_math.py);
    backward gx = y * (gy - sum(gy * y)) as a native reduction and one broadcast element pass."""

    @staticmethod
    def forward(ctx, x):
        from . import tensor_math as tm

        x = x.contiguous()
        y = torch.empty_like(x)
        native.get().log_softmax_fwd(x, y)
        tm.apply(tm.EXP, y, y)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, gy):
        from . import tensor_math as tm

        (y,) = ctx.saved_tensors
        gy = gy.contiguous().float()
        prod = torch.empty_like(y)
        tm.apply(tm.MUL, prod, gy, y)
        s, _ = tm.reduce(prod, tm.R_SUM, y.dim() - 1)           # [..., 1]
        gx = torch.empty_like(y)
        tm.apply(tm.SUB, gx, gy, s.expand(y.shape), s0=1.0)      # gy - sum(gy * y)
        tm.apply(tm.MUL, gx, gx, y)
        return gx


def softmax(x, dim=-1):
    """Softmax over ``dim``; native on the GPU when ``dim`` is the last dimension of an fp32 / bf16 tensor."""
    d = dim if dim >= 0 else x.dim() + dim
    if _gpu(x) and d == x.dim() - 1 and x.numel() > 0:
        return _Softmax.apply(x.float())
    return torch.softmax(x.float(), d)


# ---------------------------------------------------------------------------------------------- bf16 truncation
def f32_to_bf16_rtz(x, out=None):
    x = x.contiguous().float()
    if _gpu(x):
        out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if out is None else out
        native.get().f32_to_bf16_rtz(x, out)
        return out
    bits = x.view(torch.int32) >> 16
    return bits.to(torch.int16).view(torch.bfloat16) if out is None else out.copy_(bits.to(torch.int16).view(torch.bfloat16))


__all__ = ["lrn", "lrn_cpu", "dropout_gpu", "next_seed", "embedding_fwd_gpu", "embedding_bwd_gpu", "resize_bilinear",
           "resize_bilinear_cpu", "log_softmax", "f32_to_bf16_rtz"]
