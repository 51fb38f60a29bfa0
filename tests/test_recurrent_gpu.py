"""Recurrent layers on the GPU engine: MFMA Linear input projection (bf16) + fused HIP LSTM cell kernels vs
the fp32 CPU engine."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("cellname", ["LSTM", "GRU"])
def test_recurrent_gpu_matches_cpu(cellname):
    from bigdl_amd import nn
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(0)
    cell = getattr(nn, cellname)(64, 128)
    cpu = nn.Sequential().add(nn.Recurrent().add(cell)).add(nn.TimeDistributed(nn.Linear(128, 16)))
    gpu = copy.deepcopy(cpu).to("cuda")
    x = torch.randn(8, 20, 64).to(torch.bfloat16).float()
    yc = cpu.forward(x)
    yg = gpu.forward(x.cuda())
    assert _rel(yg, yc) < 2e-2
    gy = torch.randn_like(yc)
    gc = cpu.backward(x, gy)
    gg = gpu.backward(x.cuda(), gy.cuda())
    assert _rel(gg, gc) < 3e-2
    wc = torch.cat([g.reshape(-1) for g in cpu.parameters()[1]])
    wg = torch.cat([g.float().cpu().reshape(-1) for g in gpu.parameters()[1]])
    assert _rel(wg, wc) < 3e-2


def test_lstm_cell_kernel_is_used():
    """The fused sequence path must call the native kernel on the GPU (fails loudly without the extension)."""
    from bigdl_amd.nn.recurrent import _LSTMSeq

    B, T, H = 4, 6, 32
    xg = torch.randn(B, T, 4 * H, device="cuda")
    h0 = torch.zeros(B, H, device="cuda")
    c0 = torch.zeros(B, H, device="cuda")
    U = torch.randn(4 * H, H, device="cuda") * 0.1
    out, h, c = _LSTMSeq.apply(xg, h0, c0, U)
    ref, hr, cr = _LSTMSeq.apply(xg.cpu(), h0.cpu(), c0.cpu(), U.cpu())
    assert torch.allclose(out.cpu(), ref, atol=1e-5) and torch.allclose(c.cpu(), cr, atol=1e-5)
