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
