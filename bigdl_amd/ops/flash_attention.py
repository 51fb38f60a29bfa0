"""Fused attention on csrc/attention.hip (forward: online softmax, scores never in HBM; backward: recompute from
the saved log-sum-exp, dQ via fp32 atomics). q / k / v: [B, H, L, D] fp32 (converted to bf16 MFMA operands),
D = 64 or 128; bias broadcastable to [B, H, Lq, Lk] or a causal mask.

The bias is treated as a constant (attention masks): its gradient is not produced by the fused path."""
import torch

from . import native


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, bias, causal):
        B, H, Lq, D = q.shape
        Lk = k.shape[2]
        bf = torch.bfloat16
        q16 = q.detach().reshape(B * H, Lq, D).to(bf).contiguous()
        k16 = k.detach().reshape(B * H, Lk, D).to(bf).contiguous()
        v16 = v.detach().reshape(B * H, Lk, D).to(bf).contiguous()
        b = None
        if bias is not None:
            b = bias.detach().float()
            while b.dim() < 4:
                b = b.unsqueeze(0)
        o = q.new_empty(B * H, Lq, D, dtype=torch.float32)
        lse = q.new_empty(B * H, Lq, dtype=torch.float32)
        native.get().attn_fwd(q16, k16, v16, b, H, bool(causal), o, lse)
        ctx.save_for_backward(q16, k16, v16, o, lse)
        ctx.bias, ctx.H, ctx.causal, ctx.shape = b, H, bool(causal), (B, H, Lq, Lk, D)
        return o.view(B, H, Lq, D)

    @staticmethod
    def backward(ctx, do):
        q16, k16, v16, o, lse = ctx.saved_tensors
        B, H, Lq, Lk, D = ctx.shape
        do = do.reshape(B * H, Lq, D).float().contiguous()
        dq = torch.zeros(B * H, Lq, D, device=do.device)
        dk = torch.empty(B * H, Lk, D, device=do.device)
        dv = torch.empty(B * H, Lk, D, device=do.device)
        delta = torch.empty(B * H, Lq, device=do.device)
        native.get().attn_bwd(q16, k16, v16, ctx.bias, ctx.H, ctx.causal, o, lse, do, dq, dk, dv, delta)
        return dq.view(B, H, Lq, D), dk.view(B, H, Lk, D), dv.view(B, H, Lk, D), None, None


def flash_attention(q, k, v, bias=None, causal=False):
    return _FlashAttention.apply(q, k, v, bias, causal)
