"""Batched matrix products on the native bf16 MFMA GEMM (csrc/bmm.hip): ``matmul`` for MM / MV / LocallyConnected /
tree-LSTM on the GPU engine, with its backward on the same kernel.

One kernel computes C[b] = A[b] B[b]^T over K-contiguous bf16 operands (K zero-padded to a multiple of 32); the
forward and both gradients are that product of suitably transposed operands:
    C  = A  @ B        -> nt(A,     B^T)
    dA = dC @ B^T      -> nt(dC,    B)
    dB = A^T @ dC      -> nt(A^T,   dC^T)
Operands are fp32 (or bf16) tensors of shape [..., M, K] x [..., K, N] with broadcastable leading dimensions;
the result is fp32. CPU tensors fall back to torch.
"""
import torch

from . import native

BF16 = torch.bfloat16


def _kpad(t, K):
    """[B, R, K] -> contiguous bf16 [B, R, Kp] with Kp = K rounded up to 32 (zero padded)."""
    Kp = -(-K // 32) * 32
    if Kp == K:
        return t.to(BF16).contiguous()
    out = torch.zeros(t.shape[0], t.shape[1], Kp, dtype=BF16, device=t.device)
    out[:, :, :K].copy_(t)
    return out


def nt(a, b):
    """[B, M, K] x [B, N, K] -> [B, M, N] fp32 = a @ b^T on the MFMA kernel."""
    Bt, M, K = a.shape
    N = b.shape[1]
    c = torch.empty(Bt, M, N, dtype=torch.float32, device=a.device)
    native.get().bmm_nt(_kpad(a, K), _kpad(b, K), c)
    return c


class _MatMul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return nt(a, b.transpose(1, 2))

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga = gb = None
        if ctx.needs_input_grad[0]:
            ga = nt(g, b)
        if ctx.needs_input_grad[1]:
            gb = nt(a.transpose(1, 2), g.transpose(1, 2))
        return ga, gb


def matmul(a, b):
    """a [..., M, K] @ b [..., K, N] (broadcast leading dims; 1-D b is a vector) on the GPU MFMA kernel."""
    if not (a.is_cuda and b.is_cuda):
        return torch.matmul(a, b)
    vec = b.dim() == 1
    if vec:
        b = b.unsqueeze(-1)
    a2 = a.unsqueeze(0) if a.dim() == 2 else a
    b2 = b.unsqueeze(0) if b.dim() == 2 else b
    lead = torch.broadcast_shapes(a2.shape[:-2], b2.shape[:-2])
    M, K = a2.shape[-2:]
    N = b2.shape[-1]
    af = a2.float().expand(*lead, M, K).reshape(-1, M, K)
    bf = b2.float().expand(*lead, K, N).reshape(-1, K, N)
    out = _MatMul.apply(af, bf).reshape(*lead, M, N)
    if a.dim() == 2 and b.dim() == 2:
        out = out.squeeze(0)
    if vec:
        out = out.squeeze(-1)
    return out
