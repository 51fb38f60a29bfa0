"""Scaled-dot-product attention core: softmax(q k^T + bias) v over [B, heads, L, depth] tensors.

Reference: the MM(transB) -> CAddTable(bias) -> SoftMax -> Dropout -> MM chain of S/nn/Attention.scala:90-103.
GPU engine: the fused flash kernel (ops/flash_attention.py -> csrc/attention.hip) for head dims 32 / 64 / 96 / 128,
attention dropout included (in-kernel counter-hash mask, regenerated in the backward).
Math path (CPU engine, other head dims): explicit GEMMs + softmax under autograd
(q is pre-scaled by depth^-0.5 as in SplitHeads(mul=true), Attention.scala:256-275).
"""
import torch

from . import native


def _flash_ok(q, k, v, bias, dropout_p):
    """The fused kernel (csrc/attention.hip) covers head dims 32 / 64 / 96 / 128 (with or without attention
    dropout); a bias that needs a gradient (anything but a constant mask) keeps the math path."""
    if not q.is_cuda or not (0.0 <= dropout_p < 1.0):
        return False
    if bias is not None and bias.requires_grad and not getattr(bias, "_bigdl_mask", True):
        return False
    d = q.shape[-1]
    return d in (32, 64, 96, 128) and q.shape[-2] >= 1 and k.shape[-2] >= 1 and (bias is None or bias.dim() <= 4)


def attention_math(q, k, v, bias=None, dropout_p=0.0, training=False):
    s = torch.matmul(q, k.transpose(-1, -2))
    if bias is not None:
        s = s + bias
    p = torch.softmax(s, dim=-1)
    if training and dropout_p > 0.0:
        p = torch.nn.functional.dropout(p, dropout_p, True)
    return torch.matmul(p, v)


def attention(q, k, v, bias=None, dropout_p=0.0, training=False, causal=False):
    """q: [B, H, Lq, D] (already scaled), k/v: [B, H, Lk, D], bias broadcastable to [B, H, Lq, Lk].

    ``causal`` is a hint that ``bias`` is the lower-triangular -1e9 mask (Transformer SelfAttentionMask), which
    lets the fused kernel skip fully-masked key blocks.
    """
    p = dropout_p if training else 0.0
    if _flash_ok(q, k, v, bias, p):
        from .flash_attention import flash_attention

        seed = 0
        if p > 0.0:
            from .nnk import next_seed

            seed = next_seed()
        return flash_attention(q, k, v, None if causal else bias, causal, p, seed)
    return attention_math(q, k, v, bias, dropout_p, training)
