"""Transformer LM on the GPU engine (MFMA Linear FFN, attention core) vs the fp32 CPU engine."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_transformer_lm_gpu_matches_cpu():
    from bigdl_amd import nn
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(0)
    cpu = nn.Transformer(100, 128, 2, 256, 2, 1.0, 1.0, 1.0)
    gpu = copy.deepcopy(cpu).to("cuda")
    ids = torch.randint(1, 101, (4, 64)).float()
    yc = cpu.forward(ids)
    yg = gpu.forward(ids.cuda())
    assert _rel(yg, yc) < 3e-2
    gy = torch.randn_like(yc)
    cpu.backward(ids, gy)
    gpu.backward(ids.cuda(), gy.cuda())
    wc = torch.cat([g.reshape(-1) for g in cpu.parameters()[1]])
    wg = torch.cat([g.float().cpu().reshape(-1) for g in gpu.parameters()[1]])
    assert _rel(wg, wc) < 5e-2


@pytest.mark.parametrize("B,H,Lq,Lk,D,mode", [(2, 4, 128, 128, 64, "none"), (1, 2, 100, 77, 128, "pad"),
                                              (2, 2, 130, 130, 64, "causal"), (3, 1, 64, 200, 128, "full"),
                                              (1, 8, 1, 50, 64, "pad")])
def test_fused_attention_matches_fp32(B, H, Lq, Lk, D, mode):
    """csrc/attention.hip forward and backward vs the fp32 softmax(q k^T + bias) v reference."""
    from bigdl_amd.ops.flash_attention import flash_attention

    torch.manual_seed(0)
    q = (torch.randn(B, H, Lq, D) * D ** -0.5).to(torch.bfloat16).float()
    k = torch.randn(B, H, Lk, D).to(torch.bfloat16).float()
    v = torch.randn(B, H, Lk, D).to(torch.bfloat16).float()
    bias, causal = None, False
    if mode == "pad":
        bias = torch.zeros(B, 1, 1, Lk)
        bias[..., Lk - Lk // 4:] = -1e9
    elif mode == "full":
        bias = torch.randn(B, H, Lq, Lk)
    elif mode == "causal":
        causal = True
    leaves = [t.clone().double().requires_grad_(True) for t in (q, k, v)]
    s = leaves[0] @ leaves[1].transpose(-1, -2)
    if bias is not None:
        s = s + bias.double()
    if causal:
        s = s + torch.triu(torch.full((Lq, Lk), -1e9, dtype=torch.float64), 1)
    ref = torch.softmax(s, -1) @ leaves[2]
    go = torch.randn_like(ref)
    ref.backward(go)
    dev = [t.cuda().requires_grad_(True) for t in (q, k, v)]
    o = flash_attention(dev[0], dev[1], dev[2], bias.cuda() if bias is not None else None, causal)
    o.backward(go.float().cuda())
    assert _rel(o, ref) < 1e-2, _rel(o, ref)
    for d, r in zip(dev, leaves):
        assert _rel(d.grad, r.grad) < 2e-2, (d.shape, _rel(d.grad, r.grad))


@pytest.mark.parametrize("D", [32, 64, 96, 128])
@pytest.mark.parametrize("p", [0.0, 0.25])
def test_fused_attention_dropout_and_head_dims(D, p, monkeypatch):
    """Fused attention with in-kernel attention dropout (reference S/nn/Attention.scala:59) and head dims 32 / 96
    beside 64 / 128, forward and backward vs an fp32 autograd reference that applies the same keep mask
    (ops.flash_attention.dropout_mask reproduces the kernel's counter hash). torch.matmul / softmax are patched to
    raise while the fused path runs."""
    from bigdl_amd.ops.flash_attention import dropout_mask, flash_attention

    torch.manual_seed(3)
    B, H, Lq, Lk = 2, 3, 80, 72
    dev = torch.device("cuda:0")
    q = torch.randn(B, H, Lq, D, device=dev) * D ** -0.5
    k = torch.randn(B, H, Lk, D, device=dev)
    v = torch.randn(B, H, Lk, D, device=dev)
    bias = torch.randn(1, 1, Lq, Lk, device=dev) * 0.5
    go = torch.randn(B, H, Lq, D, device=dev)
    seed = 0x1234_5678_9ABC
    qg, kg, vg = (t.clone().requires_grad_(True) for t in (q, k, v))

    def boom(*a, **kw):
        raise AssertionError("aten attention math on the fused path")

    with monkeypatch.context() as mp:
        mp.setattr(torch, "matmul", boom)
        mp.setattr(torch, "softmax", boom)
        o = flash_attention(qg, kg, vg, bias, False, p, seed)
        o.backward(go)
    # reference on the bf16-rounded operands, in fp32
    qr, kr, vr = (t.to(torch.bfloat16).float().requires_grad_(True) for t in (q, k, v))
    s = qr @ kr.transpose(-1, -2) + bias
    P = torch.softmax(s, dim=-1)
    mask = dropout_mask(seed, B * H, Lq, Lk, p).view(B, H, Lq, Lk).to(dev)
    oref = (P * mask) @ vr
    oref.backward(go)

    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()

    assert rel(o, oref) < 2e-2, rel(o, oref)
    assert rel(qg.grad, qr.grad) < 3e-2, rel(qg.grad, qr.grad)
    assert rel(kg.grad, kr.grad) < 3e-2, rel(kg.grad, kr.grad)
    assert rel(vg.grad, vr.grad) < 3e-2, rel(vg.grad, vr.grad)
    if p > 0:
        kept = (mask > 0).float().mean().item()
        assert abs(kept - (1 - p)) < 0.02, kept
