"""Fused attention on csrc/attention.hip (forward: online softmax, scores never in HBM; backward: recompute from
the saved log-sum-exp, dQ via fp32 atomics). q / k / v: [B, H, L, D] fp32 (converted to bf16 MFMA operands),
D = 32, 64, 96 or 128; bias broadcastable to [B, H, Lq, Lk] or a causal mask; attention dropout (reference
S/nn/Attention.scala:59 ``attentionDropout``) in-kernel: the keep mask is a counter-based hash of (seed, row, key)
that the backward regenerates, so nothing of size Lq x Lk is ever stored (``dropout_mask`` reproduces it on the
host for tests).

The bias is treated as a constant (attention masks): its gradient is not produced by the fused path."""
import torch

from . import native


def _mix32(x):
    x = x & 0xFFFFFFFF
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    return x ^ (x >> 16)


def dropout_mask(seed, BH, Lq, Lk, p):
    """The kernel's keep-scale mask [BH, Lq, Lk] (0 or 1 / (1 - p)) on the host: keep iff
    mix32(mix32((bh * Lq + q) ^ seed_lo) + k * 0x9E3779B9 + seed_hi) >= p * 2^32 (csrc/attention.hip)."""
    lo, hi = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    rows = torch.arange(BH * Lq, dtype=torch.int64).view(BH, Lq, 1)
    keys = torch.arange(Lk, dtype=torch.int64).view(1, 1, Lk)
    r = _mix32(rows ^ lo)
    h = _mix32(r + ((keys * 0x9E3779B9) & 0xFFFFFFFF) + hi)
    thr = min(int(p * 4294967296.0), 4294967295) if p > 0 else 0
    keep = (h >= max(thr, 1 if p > 0 else 0)).float()
    return keep / (1.0 - p) if p > 0 else keep


class _FlashAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, bias, causal, dropout_p=0.0, seed=0):
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
        native.get().attn_fwd(q16, k16, v16, b, H, bool(causal), o, lse, float(dropout_p), int(seed))
        ctx.save_for_backward(q16, k16, v16, o, lse)
        ctx.bias, ctx.H, ctx.causal, ctx.shape = b, H, bool(causal), (B, H, Lq, Lk, D)
        ctx.drop = (float(dropout_p), int(seed))
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
        native.get().attn_bwd(q16, k16, v16, ctx.bias, ctx.H, ctx.causal, o, lse, do, dq, dk, dv, delta,
                              ctx.drop[0], ctx.drop[1])
        return dq.view(B, H, Lq, D), dk.view(B, H, Lk, D), dv.view(B, H, Lk, D), None, None, None, None


def flash_attention(q, k, v, bias=None, causal=False, dropout_p=0.0, seed=0):
    return _FlashAttention.apply(q, k, v, bias, causal, float(dropout_p), int(seed) & 0x7FFFFFFFFFFFFFFF)
