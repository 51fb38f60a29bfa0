"""Static int8 inference plan (quantized/int8_graph.py) and its kernels (csrc/quant.hip): requantizing conv
epilogue into concat slices, int8 max / average pooling, graph-input quantizer, and whole-graph numerics of the
planned int8 Graph against the float model."""
import pytest
import torch
import torch.nn.functional as F

from bigdl_amd import nn
from bigdl_amd.ops import native

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def test_conv_i8_requantized_output_into_slice():
    """int8 output written at a channel offset of a wider buffer equals round(clamp(y / s_out)) of the fp32 result."""
    from bigdl_amd.ops.conv import _fwd_taps, out_size

    N, C, H, W, K, R = 2, 48, 10, 9, 40, 3
    g = torch.Generator().manual_seed(3)
    x = torch.randint(-127, 128, (N, H, W, C), generator=g, dtype=torch.int8)
    w = torch.randint(-127, 128, (K, R, R, C), generator=g, dtype=torch.int8)
    xs, ws = 0.02, torch.rand(K, generator=g) * 0.01 + 0.001
    bias = torch.randn(K, generator=g)
    OH, OW = out_size(H, R, 1, 1), out_size(W, R, 1, 1)
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(0, 3, 1, 2).double(), None, 1, 1)
    ref = ref * xs * ws.double().view(1, K, 1, 1) + bias.double().view(1, K, 1, 1)
    ref = torch.relu(ref).permute(0, 2, 3, 1)
    s_out = float(ref.abs().max()) / 127
    buf = torch.full((N, OH, OW, 64), 99, dtype=torch.int8, device="cuda")
    sl = buf[..., 16:16 + K]
    geo = [N, H, W, C, OH, OW, 1, 1, R * R * C, K, 64, OH, OW, 1, 1, 0, 0]
    native.get().conv_i8(x.cuda(), w.cuda(), sl, bias.cuda(), None, ws.cuda(), geo, _fwd_taps(R, R, 1, 1, 1, 1), True,
                         xs, s_out)
    got = buf.cpu()
    exp = torch.clamp(torch.round(ref / s_out), -127, 127).to(torch.int8)
    assert (got[..., 16:16 + K].int() - exp.int()).abs().max() <= 1
    assert torch.all(got[..., :16] == 99) and torch.all(got[..., 16 + K:] == 99)


@pytest.mark.parametrize("avg,k,s,p,count_pad", [(False, 3, 2, 0, False), (False, 3, 1, 1, False),
                                                (True, 3, 1, 1, True), (True, 3, 1, 1, False), (True, 8, 8, 0, True)])
def test_pool_i8_matches_reference(avg, k, s, p, count_pad, shape=(2, 17, 17, 32)):
    from bigdl_amd.ops.conv import out_size

    N, H, W, C = shape
    g = torch.Generator().manual_seed(4)
    x = torch.randint(-127, 128, (N, H, W, C), generator=g, dtype=torch.int8)
    OH, OW = out_size(H, k, s, p), out_size(W, k, s, p)
    y = torch.zeros((N, OH, OW, C), dtype=torch.int8, device="cuda")
    native.get().pool_i8(x.cuda(), y, [N, H, W, C, OH, OW, k, k, s, s, p, p, C], avg, count_pad)
    xf = x.permute(0, 3, 1, 2).double()
    if avg:
        ref = torch.round(F.avg_pool2d(xf, k, s, p, count_include_pad=count_pad))
    else:
        ref = F.max_pool2d(xf, k, s, p)
    ref = ref.permute(0, 2, 3, 1)
    assert (y.cpu().double() - ref).abs().max() <= 1


@pytest.mark.parametrize("avg,count_pad,shape", [(True, True, (1, 35, 35, 48)), (True, False, (2, 8, 9, 16)),
                                                  (False, False, (1, 35, 35, 48)), (True, True, (3, 5, 3, 16)),
                                                  (True, True, (2, 17, 17, 768)), (True, True, (2, 8, 8, 2048)),
                                                  (False, False, (1, 17, 17, 528))])
def test_pool3s1_i8_runs(avg, count_pad, shape):
    """3x3 / stride-1 int8 pooling (Inception pool branches): partial runs, widths below 8, and Inception's wide
    channel counts (768 / 2048 / 528)."""
    test_pool_i8_matches_reference(avg, 3, 1, 1, count_pad, shape)


def test_quantize_nchw_input():
    x = torch.randn(2, 3, 7, 5, device="cuda")
    q = torch.zeros((2, 7, 5, 16), dtype=torch.int8, device="cuda")
    s = float(x.abs().max()) / 127
    native.get().quantize_nchw_f32(x, q, 16, s)
    ref = torch.clamp(torch.round(x.permute(0, 2, 3, 1) / s), -127, 127).to(torch.int8)
    assert (q[..., :3].int() - ref.int()).abs().max() <= 1 and torch.all(q[..., 3:] == 0)


def _small_inception():
    torch.manual_seed(0)
    inp = nn.Input()
    x = nn.ReLU()(nn.SpatialConvolution(3, 32, 3, 3, 2, 2)(inp))
    x = nn.ReLU()(nn.SpatialConvolution(32, 48, 3, 3, 1, 1, 1, 1)(x))
    x = nn.SpatialMaxPooling(3, 3, 2, 2)(x)
    a = nn.ReLU()(nn.SpatialConvolution(48, 32, 1, 1)(x))
    b = nn.ReLU()(nn.SpatialConvolution(48, 16, 1, 1)(x))
    b = nn.ReLU()(nn.SpatialConvolution(16, 32, 3, 3, 1, 1, 1, 1)(b))
    c = nn.SpatialAveragePooling(3, 3, 1, 1, 1, 1)(x)
    c = nn.ReLU()(nn.SpatialConvolution(48, 16, 1, 1)(c))
    d = nn.SpatialMaxPooling(3, 3, 1, 1, 1, 1)(x)
    j = nn.JoinTable(2, 0)(a, b, c, d)                                       # 32 + 32 + 16 + 48 = 128
    y = nn.ReLU()(nn.SpatialConvolution(128, 64, 1, 1)(j))
    y = nn.SpatialAveragePooling(7, 7, 1, 1)(y)
    y = nn.View(64).setNumInputDims(3)(y)
    y = nn.Linear(64, 10)(y)
    g = nn.Graph([inp], [y])
    g.evaluate()
    return g


def test_int8_plan_graph_matches_float():
    from bigdl_amd.quantized.int8_graph import I8Act
    from bigdl_amd.quantized.quantizer import quantize

    g = _small_inception()
    x = torch.randn(8, 3, 33, 33)
    ref = g.forward(x).clone()
    dev = torch.device("cuda:0")
    gd = g.cloneModule().to(dev)
    q = quantize(gd, calibration=x.to(dev))
    plan = q._int8_plan
    assert plan is not None and sum(plan.int8.values()) >= 8, plan.int8
    y = q.forward(x.to(dev))
    assert y.dtype == torch.float32 and y.shape == ref.shape
    assert _rel(y, ref) < 0.08
    # every conv produced int8 (requantizing epilogue) and the concat stayed int8
    n8 = sum(isinstance(v, I8Act) for v in q._outs.values())
    assert n8 >= 8
    y2 = q.forward(x.to(dev))
    assert _rel(y2, y) < 1e-6


def test_int8_plan_residual_conv_sum_fused():
    """conv -> BN -> Scale -> CAddTable(shortcut) -> ReLU: BN / Scale fold into the conv, the int8 epilogue adds the
    int8 shortcut and applies the ReLU; numerics vs the float graph."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(__file__))
    from test_graph_fusion_gpu import _inception_residual_graph

    from bigdl_amd.quantized.quantizer import quantize

    g = _inception_residual_graph()
    x = torch.randn(8, 3, 16, 16)
    ref = g.forward(x).clone()
    dev = torch.device("cuda:0")
    q = quantize(g.cloneModule().to(dev), calibration=x.to(dev))
    y = q.forward(x.to(dev))
    assert _rel(y, ref) < 0.08
    plan = q._int8_plan
    assert plan.res and all(plan.fused.get(a) for a in plan.res), "residual add was not fused into the int8 conv"


def test_quantize_wim2col_input():
    """Width im2col of the int8 stem input: y[n][h][ow][e*4 + c] = q(x[n][c][h][ow*sw + e - pw])."""
    N, C, H, W, S, sw, pw = 2, 3, 6, 13, 7, 2, 3
    OW = (W + 2 * pw - S) // sw + 1
    x = torch.randn(N, C, H, W, device="cuda")
    s = float(x.abs().max()) / 127
    y = torch.full((N, H, OW, 32), 99, dtype=torch.int8, device="cuda")
    native.get().quantize_wim2col_f32(x, y, OW, S, sw, pw, s)
    q = torch.clamp(torch.round(x.cpu() / s), -127, 127)
    ref = torch.zeros(N, H, OW, 8, 4)
    for ow in range(OW):
        for e in range(S):
            w = ow * sw + e - pw
            if 0 <= w < W:
                ref[:, :, ow, e, :C] = q[:, :, :, w].permute(0, 2, 1)
    assert (y.cpu().view(N, H, OW, 8, 4).double() - ref.double()).abs().max() <= 1


def test_int8_stem_width_im2col_equals_direct(monkeypatch):
    """7x7 / 2 stem (3 channels, pad 3) on the width-im2col path (R x 1 conv over 32-byte rows, reduction 224)
    gives exactly the int8 values of the direct 7x7 conv over 16-channel pixels (reduction 784)."""
    from bigdl_amd.quantized.int8_graph import I8Act, I8Stem
    from bigdl_amd.quantized.quantizer import quantize

    torch.manual_seed(3)
    inp = nn.Input()
    y = nn.ReLU()(nn.SpatialConvolution(3, 64, 7, 7, 2, 2, 3, 3)(inp))
    y = nn.SpatialMaxPooling(3, 3, 2, 2, 1, 1)(y)
    y = nn.ReLU()(nn.SpatialConvolution(64, 32, 1, 1)(y))
    g = nn.Graph([inp], [y])
    g.evaluate()
    x = torch.randn(4, 3, 37, 41)
    ref = g.forward(x).clone()
    dev = torch.device("cuda:0")
    outs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("BIGDL_I8_STEM", mode)
        q = quantize(g.cloneModule().to(dev), calibration=x.to(dev))
        outs[mode] = q.forward(x.to(dev)).float().clone()
        if mode == "1":
            assert any(isinstance(v, I8Stem) for v in q._outs.values()), "input was not quantized into the im2col"
            assert any(isinstance(v, I8Act) for v in q._outs.values()), "stem conv did not produce int8"
    assert torch.equal(outs["1"], outs["0"])
    assert _rel(outs["1"], ref) < 0.08
