"""Deferred BatchNorm + ReLU (csrc/kernels.h ConvArgs::pre): the consumer applies relu(x * scale + shift) on load.

Each kernel path is checked bit-for-bit against the same kernel on the materialised BN output (bn_apply), and against
a plain fp32 PyTorch reference of the same op; the module path against BIGDL_BN_DEFER off."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last
BF = torch.bfloat16


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _aff(C, dev):
    # shifts of both signs and well away from 0: relu(shift) > 0 on half the channels, so a zero-padding pixel that
    # went through the transform (it must not) changes the border outputs
    sc = torch.linspace(0.5, 1.5, C, device=dev)
    sh = torch.linspace(-0.8, 0.8, C, device=dev)
    return torch.cat([sc, sh]).contiguous()


def _ref_input(x, aff):
    C = x.shape[1]
    return torch.relu(x.float() * aff[:C].view(1, C, 1, 1) + aff[C:].view(1, C, 1, 1)).to(BF).float()


# N, C, H, K: 3x3 / stride 1 / pad 1 shapes the halo kernel takes (ResNet-50 layers 2, 10, 16, 22 and odd ones)
HALO_CASES = [(2, 64, 56, 64), (3, 128, 28, 128), (2, 256, 14, 256), (4, 512, 7, 512), (7, 64, 7, 128),
              (3, 96, 14, 128)]


@pytest.mark.parametrize("case", HALO_CASES)
def test_halo_pre(case):
    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import conv as cv

    N, C, H, K = case
    dev = torch.device("cuda:0")
    torch.manual_seed(3)
    x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
    w = (torch.randn(K, C, 3, 3, device=dev) * (1.0 / (9 * C) ** 0.5)).to(BF, memory_format=CL)
    aff = _aff(C, dev)
    ymat = bnops.materialize(bnops.deferred(x, aff))
    assert _rel(ymat, _ref_input(x, aff)) < 1e-2
    st0, st1 = bnops.new_stats(K, dev), bnops.new_stats(K, dev)
    y0 = cv.conv2d_fwd(ymat, w, None, (1, 1), (1, 1), stats=st0)
    y1, mat = cv.conv2d_fwd(x, w, None, (1, 1), (1, 1), stats=st1, pre=aff)
    torch.cuda.synchronize()
    assert mat is None, "the halo kernel should apply the BN on load"
    assert torch.equal(y1, y0)
    assert _rel(st1.view(bnops.stat_slots(), 2, K).sum(0), st0.view(bnops.stat_slots(), 2, K).sum(0)) < 1e-5
    yr = F.conv2d(_ref_input(x, aff), w.float(), padding=1)
    assert _rel(y1, yr) < 1e-2
    s = st1.view(bnops.stat_slots(), 2, K).sum(0)
    assert _rel(s[0], y1.float().sum(dim=(0, 2, 3))) < 1e-4


# N, C, H, K: 1x1 / stride 1 with 64 or 128 input channels (the streaming kernel): ResNet-50 stage 1-2 conv3 shapes
S1_CASES = [(2, 64, 56, 256), (2, 128, 28, 512), (3, 64, 7, 64), (2, 128, 14, 128), (2, 256, 14, 1024),
            (3, 256, 9, 64)]


@pytest.mark.parametrize("bias", [False, True])
@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("case", S1_CASES)
def test_s1_pre(case, relu, bias):
    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import conv as cv

    N, C, H, K = case
    dev = torch.device("cuda:0")
    torch.manual_seed(5)
    x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
    w = (torch.randn(K, C, 1, 1, device=dev) * (1.0 / C ** 0.5)).to(BF, memory_format=CL)
    aff = _aff(C, dev)
    b = torch.randn(K, device=dev) if bias else None
    ymat = bnops.materialize(bnops.deferred(x, aff))
    st0, st1 = bnops.new_stats(K, dev), bnops.new_stats(K, dev)
    y0 = cv.conv2d_fwd(ymat, w, b, (1, 1), (0, 0), relu=relu, stats=st0)
    y1, mat = cv.conv2d_fwd(x, w, b, (1, 1), (0, 0), relu=relu, stats=st1, pre=aff)
    torch.cuda.synchronize()
    assert mat is None, "the streaming 1x1 kernel should apply the BN on load"
    assert torch.equal(y1, y0)
    # (the two launches may use different grids, so compare the slot sums, not the slots)
    assert _rel(st1.view(bnops.stat_slots(), 2, K).sum(0), st0.view(bnops.stat_slots(), 2, K).sum(0)) < 1e-5
    yr = F.conv2d(_ref_input(x, aff), w.float(), b)
    if relu:
        yr = torch.relu(yr)
    assert _rel(y1, yr) < 1e-2


def test_pre_fallback_materialises():
    """A GEMM no kernel applies it to (3x3 stride 2, bias) gets the materialised input from the binding, which it
    returns for the weight gradient."""
    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import conv as cv

    dev = torch.device("cuda:0")
    torch.manual_seed(7)
    x = torch.randn(2, 64, 28, 28, device=dev).to(BF, memory_format=CL)
    w = (torch.randn(64, 64, 3, 3, device=dev) * 0.05).to(BF, memory_format=CL)
    b = torch.randn(64, device=dev)
    aff = _aff(64, dev)
    ymat = bnops.materialize(bnops.deferred(x, aff))
    y0 = cv.conv2d_fwd(ymat, w, b, (2, 2), (1, 1))
    y1, mat = cv.conv2d_fwd(x, w, b, (2, 2), (1, 1), pre=aff)
    torch.cuda.synchronize()
    assert mat is not None and torch.equal(mat, ymat)
    assert torch.equal(y1, y0)


def test_maxpool_pre():
    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import pool as P

    dev = torch.device("cuda:0")
    torch.manual_seed(9)
    x = torch.randn(3, 64, 30, 30, device=dev).to(BF, memory_format=CL)
    aff = _aff(64, dev)
    ymat = bnops.materialize(bnops.deferred(x, aff))
    y0, i0 = P.maxpool_fwd_gpu(ymat, 3, 3, 2, 2, 1, 1)
    y1, i1 = P.maxpool_fwd_gpu(x, 3, 3, 2, 2, 1, 1, pre=aff)
    torch.cuda.synchronize()
    assert torch.equal(y1, y0) and torch.equal(i1, i0)
    yr = F.max_pool2d(_ref_input(x, aff), 3, 2, 1)
    assert _rel(y1, yr) < 1e-3      # (torch rounds x * s before + b; the kernels fuse the multiply-add)


def _grads(m):
    from bigdl_amd import nn

    out = []
    for l in m.flattened_layers():
        if isinstance(l, nn.SpatialConvolution):
            out.append(l.gradWeight.float().reshape(-1).clone())
    return torch.cat(out)


@pytest.mark.parametrize("n,H", [(64, 56), (128, 28)])
def test_bottleneck_deferred_matches_materialised(n, H):
    """A ResNet bottleneck with BN1 / BN2 deferred into the 3x3 halo and 1x1 streaming forwards (and re-applied for
    the weight gradients on the side stream) against BIGDL_BN_DEFER off: same output, input and weight gradients."""
    from bigdl_amd.models.resnet import _Builder
    from bigdl_amd.nn import fusion, normalization
    from bigdl_amd.nn.fusion import fuse_for_training

    b = _Builder("B", True)
    b.iChannels = 4 * n
    blk = b.bottleneck(n, 1)
    torch.manual_seed(11)
    for l in blk.flattened_layers():
        if type(l).__name__ == "SpatialBatchNormalization":
            l.weight.data.uniform_(0.5, 1.5)
            l.bias.data.uniform_(-0.3, 0.3)
    x = torch.randn(2, 4 * n, H, H).cuda().to(BF).contiguous(memory_format=CL)
    gy = torch.randn(2, 4 * n, H, H).cuda().to(BF).contiguous(memory_format=CL)
    res = {}
    saved, saved_lvl = normalization._DEFER[0], fusion.DEFER_LEVEL[0]
    fusion.DEFER_LEVEL[0] = 2          # 3x3 consumers too
    try:
        for on in (True, False):
            normalization._DEFER[0] = on
            m = copy.deepcopy(blk).to("cuda")
            fuse_for_training(m)
            y = m.forward(x).float().clone()
            branch = m.modules[0].modules[0]
            convs = [l for l in branch.modules if type(l).__name__.endswith("Convolution")]
            if on:
                assert getattr(branch.modules[2].output, "_bn_pre", None) is not None
                assert convs[1]._x16_pre is not None, "applied on load"
            g = m.backward(x, gy).float().clone()
            torch.cuda.synchronize()
            res[on] = (y, g, _grads(m))
    finally:
        normalization._DEFER[0], fusion.DEFER_LEVEL[0] = saved, saved_lvl
    assert _rel(res[True][0], res[False][0]) < 1e-3
    assert _rel(res[True][1], res[False][1]) < 1e-2
    assert _rel(res[True][2], res[False][2]) < 1e-2


@pytest.mark.parametrize("case", HALO_CASES)
def test_wgrad_halo_pre(case):
    """The halo 3x3 weight gradient applying a deferred BN + ReLU to its x tiles: bit-equal to the same kernel on the
    materialised input (fixed-order split reduce), and vs fp32 torch (conv2d_weight) and the bias column sums."""
    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import conv as cv

    N, C, H, K = case
    dev = torch.device("cuda:0")
    torch.manual_seed(17)
    x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
    gy = torch.randn(N, K, H, H, device=dev).to(BF, memory_format=CL)
    aff = _aff(C, dev)
    ymat = bnops.materialize(bnops.deferred(x, aff))
    dws = []
    for src, pre in ((ymat, None), (x, aff)):
        dw = torch.zeros(K, C, 3, 3, device=dev).contiguous(memory_format=CL)
        db = torch.zeros(K, device=dev)
        cv.conv2d_wgrad(gy, src, dw, db, (1, 1), (1, 1), pre=pre)
        dws.append((dw, db))
    torch.cuda.synchronize()
    assert torch.equal(dws[1][0], dws[0][0]) and torch.equal(dws[1][1], dws[0][1])
    ref = torch.nn.grad.conv2d_weight(_ref_input(x, aff), (K, C, 3, 3), gy.float(), padding=1)
    assert _rel(dws[1][0], ref) < 1e-2
    assert _rel(dws[1][1], gy.float().sum(dim=(0, 2, 3))) < 1e-3
