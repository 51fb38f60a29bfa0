"""Layer normalisation on the native kernels (csrc/layernorm.hip) as an autograd function (reference
S/nn/LayerNormalization.scala); the CPU engine keeps the fp32 torch math."""
import torch
import torch.nn.functional as F

from . import native


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, g, b, eps):
        x = x.contiguous()
        D = x.shape[-1]
        rows = x.numel() // D
        y = torch.empty_like(x)
        mean = x.new_empty(rows)
        rstd = x.new_empty(rows)
        native.get().layernorm_fwd(x, g.contiguous() if g is not None else None,
                                   b.contiguous() if b is not None else None, y, mean, rstd, float(eps))
        ctx.save_for_backward(x, g, mean, rstd)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, g, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous().float()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dg = torch.zeros_like(g) if g is not None and ctx.needs_input_grad[1] else None
        db = torch.zeros(x.shape[-1], device=x.device) if ctx.has_b and ctx.needs_input_grad[2] else None
        native.get().layernorm_bwd(dy, x, g, mean, rstd, dx, dg, db)
        return dx, dg, db, None


def layer_norm(x, weight, bias, eps):
    D = x.shape[-1]
    if x.is_cuda and x.dtype == torch.float32 and D <= 4096:
        return _LayerNorm.apply(x, weight, bias, eps)
    return F.layer_norm(x, (D,), weight, bias, eps)
