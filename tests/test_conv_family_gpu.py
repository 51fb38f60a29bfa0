"""Conv-family layers on the native implicit-GEMM kernels (ops/conv_fn.py) vs the fp32 CPU engine: transposed,
temporal, connection-table, separable (pointwise half) and volumetric convolution, forward and all gradients."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _case(name):
    from bigdl_amd import nn

    if name == "full":
        return nn.SpatialFullConvolution(12, 20, 3, 3, 2, 2, 1, 1, 1, 1), (2, 12, 9, 9)
    if name == "full_nopad":
        return nn.SpatialFullConvolution(8, 16, 4, 4, 2, 2, 0, 0), (3, 8, 7, 6)
    if name == "temporal":
        return nn.TemporalConvolution(24, 40, 3, 2), (4, 17, 24)
    if name == "map":
        return nn.SpatialConvolutionMap(nn.SpatialConvolutionMap.full(6, 10), 3, 3, 1, 1, 1, 1), (2, 6, 11, 11)
    if name == "separable":
        return nn.SpatialSeparableConvolution(8, 24, 2, 3, 3, 1, 1, 1, 1), (2, 8, 10, 10)
    if name == "grouped":
        return nn.SpatialConvolution(16, 32, 3, 3, 1, 1, 1, 1, nGroup=4), (2, 16, 12, 12)
    if name == "depthwise":
        return nn.SpatialConvolution(24, 48, 3, 3, 2, 2, 1, 1, nGroup=24), (2, 24, 13, 13)
    if name == "grouped_wide":
        return nn.SpatialConvolution(64, 64, 3, 3, 1, 1, 1, 1, nGroup=2), (2, 64, 8, 8)
    if name == "volumetric":
        return nn.VolumetricConvolution(6, 16, 3, 3, 3, 1, 2, 2, 1, 1, 1), (2, 6, 7, 9, 9)
    if name == "full3d":
        return nn.VolumetricFullConvolution(6, 10, 3, 3, 3, 2, 2, 2, 1, 1, 1, 1, 1, 1), (2, 6, 4, 5, 5)
    if name == "convlstm":
        return nn.Recurrent().add(nn.ConvLSTMPeephole(4, 8, 3, 3)), (2, 3, 4, 6, 6)
    if name == "maxout":
        # pieces separated by their biases: a bf16 GEMM must not flip the argmax that routes the gradient
        m = nn.Maxout(16, 8, 3)
        m.bias.copy_((torch.arange(24) % 3).float() * 3.0)
        return m, (5, 16)
    if name == "highway":
        return nn.Highway(16), (5, 16)
    if name == "cosine":
        return nn.Cosine(16, 7), (5, 16)
    if name == "subnorm":
        return nn.SpatialSubtractiveNormalization(3, torch.ones(5, 5)), (2, 3, 9, 9)
    if name == "wclrn":
        return nn.SpatialWithinChannelLRN(5, 1.0, 0.75), (2, 3, 8, 8)
    if name == "gemm":
        g = torch.Generator().manual_seed(3)
        return nn.Gemm(0.5, 2.0, False, True, matrixB=torch.randn(10, 24, generator=g),
                       matrixC=torch.randn(6, 10, generator=g)), (6, 24)
    raise KeyError(name)


ALL = ["full", "full_nopad", "temporal", "map", "separable", "volumetric", "grouped", "depthwise", "grouped_wide",
       "full3d", "convlstm", "maxout", "highway", "cosine", "subnorm", "wclrn", "gemm"]


@pytest.mark.parametrize("name", ALL)
def test_conv_family_native_matches_cpu(name):
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(5)
    cpu, shape = _case(name)
    gpu = copy.deepcopy(cpu).to("cuda")
    x = torch.randn(*shape).to(torch.bfloat16).float()
    yc = cpu.forward(x)
    yg = gpu.forward(x.cuda())
    assert yg.shape == yc.shape
    assert _rel(yg, yc) < 1e-2, _rel(yg, yc)
    gy = torch.randn_like(yc)
    gc = cpu.backward(x, gy)
    gg = gpu.backward(x.cuda(), gy.cuda())
    assert _rel(gg, gc) < 2e-2, _rel(gg, gc)
    for a, b in zip((gpu.parameters() or ([], []))[1], (cpu.parameters() or ([], []))[1]):
        assert _rel(a, b) < 2e-2, (a.shape, _rel(a, b))


def test_conv_family_uses_no_vendor_conv(monkeypatch):
    """The GPU path must not reach torch's (MIOpen) convolutions for these layers."""
    import torch.nn.functional as F

    def boom(*a, **k):
        raise AssertionError("vendor convolution called on the GPU path")

    for fn in ("conv2d", "conv1d", "conv3d", "conv_transpose2d", "conv_transpose3d", "linear", "avg_pool2d"):
        monkeypatch.setattr(F, fn, boom)
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(1)
    for name in ("full", "temporal", "map", "volumetric", "separable", "grouped", "depthwise", "full3d", "convlstm",
                 "maxout", "highway", "cosine", "subnorm", "wclrn", "gemm"):
        m, shape = _case(name)
        m = m.to("cuda")
        y = m.forward(torch.randn(*shape, device="cuda"))
        m.backward(torch.randn(*shape, device="cuda"), torch.ones_like(y))


@pytest.mark.parametrize("shape", [(4, 7, 512), (33, 1000), (2, 3, 4096), (5, 96)])
def test_layernorm_native_matches_fp32(shape):
    from bigdl_amd.ops.norm import layer_norm

    torch.manual_seed(0)
    D = shape[-1]
    x = torch.randn(*shape) * 3 + 1
    g, b = torch.randn(D), torch.randn(D)
    dy = torch.randn(*shape)
    leaves = [t.clone().requires_grad_(True) for t in (x, g, b)]
    ref = torch.nn.functional.layer_norm(leaves[0], (D,), leaves[1], leaves[2], 1e-6)
    ref.backward(dy)
    dev = [t.cuda().requires_grad_(True) for t in (x, g, b)]
    y = layer_norm(dev[0], dev[1], dev[2], 1e-6)
    y.backward(dy.cuda())
    assert _rel(y, ref) < 1e-5
    for a, r in zip(dev, leaves):
        assert _rel(a.grad, r.grad) < 1e-4


PAIR_CASES = [
    # nIn, nOut, k, stride (h, w), pad, N, H, W: <= 4 input channels with width stride 2 -> pixel-pair packing
    (3, 64, 7, (2, 2), 3, 2, 38, 38),      # ResNet stem geometry
    (3, 16, 3, (2, 2), 1, 2, 29, 31),      # odd sizes, 3x3
    (4, 32, 5, (1, 2), 2, 2, 20, 26),      # height stride 1
    (1, 8, 7, (2, 2), 0, 3, 23, 23),       # 1 channel, no padding
    (3, 64, 7, (2, 2), 3, 2, 224, 224),    # ImageNet stem: the dedicated halo kernel (csrc/stem_fwd.hip)
]


@pytest.mark.parametrize("case", PAIR_CASES)
def test_stem_pixel_pair_conv_matches_cpu(case):
    """SpatialConvolution with <= 4 input channels and width stride 2 runs the pixel-pair packed implicit GEMM
    (csrc/stem.hip + conv_igemm.hip): forward, BN statistics epilogue, gradient input and weight / bias gradients vs
    the fp32 CPU engine."""
    from bigdl_amd import nn
    from bigdl_amd.utils.random_generator import RNG

    nin, nout, k, (sh, sw), p, N, H, W = case
    RNG.setSeed(9)
    cpu = nn.SpatialConvolution(nin, nout, k, k, sw, sh, p, p)
    gpu = copy.deepcopy(cpu).to("cuda")
    x = torch.randn(N, nin, H, W).to(torch.bfloat16).float()
    yc = cpu.forward(x)
    yg = gpu.forward(x.cuda())
    assert getattr(gpu, "_xpair", None) is not None           # the pair path ran
    assert yg.shape == yc.shape
    assert _rel(yg, yc) < 1e-2, _rel(yg, yc)
    gy = torch.randn_like(yc).to(torch.bfloat16).float()
    gc = cpu.backward(x, gy)
    gg = gpu.backward(x.cuda(), gy.cuda())
    assert _rel(gg, gc) < 2e-2, _rel(gg, gc)
    for a, b in zip(gpu.parameters()[1], cpu.parameters()[1]):
        assert _rel(a, b) < 1e-2, (a.shape, _rel(a, b))


def test_stem_fwd_kernel_matches_gemm_path():
    """The dedicated 7x7/2 stem kernel (csrc/stem_fwd.hip: input-row halo in LDS, 7 row-tap K-steps, lean epilogue)
    against fp32 torch and against the implicit-GEMM path it replaces (BIGDL_STEM_FWD off): output, bias + ReLU,
    BN statistics of the rounded output."""
    import torch.nn.functional as F

    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import conv as cv
    from bigdl_amd.ops import native

    C_ = native.get()
    torch.manual_seed(5)
    N = 3
    x = torch.randn(N, 3, 224, 224, device="cuda")
    w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).to(torch.bfloat16)
    b = torch.randn(64, device="cuda")
    OH, OW, S2, _, _ = cv.pair_geometry(224, 224, 7, 7, 2, 3, 3)
    xp = cv.to_pairs_bf16(x, 7, 7, 2, 3, 3)
    wp = cv.pair_weight(w.contiguous(memory_format=torch.channels_last))
    ref = F.conv2d(x.to(torch.bfloat16).float(), w.float(), stride=2, padding=3)
    res = {}
    for on in (1, 0):
        C_.set_stem_fwd(on)
        try:
            st = bnops.new_stats(64, "cuda")
            y = cv.conv2d_pairs_fwd(xp, wp, None, 64, OH, OW, 7, S2, 2, stats=st)
            y2 = cv.conv2d_pairs_fwd(xp, wp, b, 64, OH, OW, 7, S2, 2, relu=True)
            torch.cuda.synchronize()
            res[on] = (y, st, y2)
        finally:
            C_.set_stem_fwd(1)
    y, st, y2 = res[1]
    assert _rel(y, ref) < 1e-2 and _rel(y, res[0][0]) < 1e-2
    assert _rel(y2, torch.relu(ref + b.view(1, -1, 1, 1))) < 1e-2
    s2 = st.view(bnops.stat_slots(), 2, 64).sum(0)
    assert _rel(s2[0], y.float().sum(dim=(0, 2, 3))) < 1e-4
    assert _rel(s2[1], (y.float() ** 2).sum(dim=(0, 2, 3))) < 1e-4


def test_stem_wgrad_kernel_matches_gemm_path():
    """The pair-view stem weight-gradient kernel (csrc/stem_fwd.hip: 7 row-tap waves, transposed LDS reads of dy rows
    and overlapping input windows, fixed-order partial reduce) against the split-K implicit-GEMM path (off) and fp32
    torch; the bias gradient too."""
    from bigdl_amd.ops import conv as cv
    from bigdl_amd.ops import native

    C_ = native.get()
    torch.manual_seed(6)
    N = 3
    x = torch.randn(N, 3, 224, 224, device="cuda")
    dy = torch.randn(N, 64, 112, 112, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xp = cv.to_pairs_bf16(x, 7, 7, 2, 3, 3)
    S2 = 4
    res = {}
    for on in (1, 0):
        C_.set_stem_wgrad(on)
        try:
            dwp = torch.zeros(64, 7 * S2 * 8, device="cuda")
            db = torch.zeros(64, device="cuda")
            cv.conv2d_pairs_wgrad(dy, xp, 7, S2, 2, dwp, db)
            torch.cuda.synchronize()
            res[on] = (dwp, db)
        finally:
            C_.set_stem_wgrad(1)
    assert _rel(res[1][0], res[0][0]) < 1e-3, _rel(res[1][0], res[0][0])
    assert _rel(res[1][1], res[0][1]) < 1e-4
    ref = torch.nn.grad.conv2d_weight(x.to(torch.bfloat16).float(), (64, 3, 7, 7), dy.float(), stride=2, padding=3)
    # pair layout back to (K, C, R, S): w'[k][r][j][e * 4 + c] = w[k][c][r][2 j + e]
    wpv = res[1][0].view(64, 7, S2, 2, 4)
    got = torch.zeros(64, 3, 7, 7, device="cuda")
    for j in range(S2):
        for e in range(2):
            s_ = 2 * j + e
            if s_ < 7:
                got[:, :, :, s_] = wpv[:, :, j, e, :3].permute(0, 2, 1)
    assert _rel(got, ref) < 1e-2, _rel(got, ref)
    assert _rel(res[1][1], dy.float().sum(dim=(0, 2, 3))) < 1e-3


def _bmm_case(name):
    from bigdl_amd import nn
    from bigdl_amd.utils.table import Table

    g = torch.Generator().manual_seed(4)
    if name == "mm":
        return nn.MM(), Table(torch.randn(3, 20, 37, generator=g), torch.randn(3, 37, 50, generator=g))
    if name == "mm_trans":
        return nn.MM(True, True), Table(torch.randn(2, 33, 17, generator=g), torch.randn(2, 70, 33, generator=g))
    if name == "mm_2d":
        return nn.MM(), Table(torch.randn(65, 40, generator=g), torch.randn(40, 3, generator=g))
    if name == "mv":
        return nn.MV(), Table(torch.randn(4, 19, 45, generator=g), torch.randn(4, 45, generator=g))
    if name == "lc2d":
        return nn.LocallyConnected2D(5, 9, 8, 12, 3, 3, 2, 1, 1, 1), torch.randn(3, 5, 8, 9, generator=g)
    if name == "lc1d":
        return nn.LocallyConnected1D(11, 6, 10, 3, 2), torch.randn(4, 11, 6, generator=g)
    if name == "treelstm":
        t1 = torch.tensor([[2, 5, -1], [0, 0, 1], [0, 0, 2], [0, 0, 3], [3, 4, 0], [-1, -1, -1]], dtype=torch.float32)
        t2 = torch.tensor([[2, 3, -1], [4, 5, 0], [0, 0, 3], [0, 0, 1], [0, 0, 2], [-1, -1, -1]], dtype=torch.float32)
        return nn.BinaryTreeLSTM(16, 24), Table(torch.randn(2, 3, 16, generator=g), torch.stack([t1, t2]))
    raise KeyError(name)


@pytest.mark.parametrize("name", ["mm", "mm_trans", "mm_2d", "mv", "lc2d", "lc1d", "treelstm"])
def test_matrix_product_layers_native_match_cpu(name, monkeypatch):
    """MM / MV (S/nn/MM.scala:34, S/nn/MV.scala:33), LocallyConnected1D/2D (S/nn/LocallyConnected2D.scala:233) and
    BinaryTreeLSTM on the GPU engine run the native batched MFMA GEMM (csrc/bmm.hip) / linear kernels: forward and
    all gradients vs the fp32 CPU engine, with torch's matmul / bmm / einsum / addmm patched to raise."""
    from bigdl_amd.utils.random_generator import RNG
    from bigdl_amd.utils.table import Table

    RNG.setSeed(6)
    cpu, x = _bmm_case(name)
    gpu = copy.deepcopy(cpu).to("cuda")

    def to_dev(a):
        if isinstance(a, Table):
            out = Table()
            for k, v in a.items():
                out[k] = to_dev(v)
            return out
        return a.to(torch.bfloat16).float().cuda() if a.is_floating_point() and a.dim() > 1 and name != "treelstm" \
            else a.cuda()

    def to_cpu_ref(a):
        if isinstance(a, Table):
            out = Table()
            for k, v in a.items():
                out[k] = to_cpu_ref(v)
            return out
        return a.to(torch.bfloat16).float() if a.is_floating_point() and a.dim() > 1 and name != "treelstm" else a

    xc, xg = to_cpu_ref(x), to_dev(x)
    yc = cpu.forward(xc)

    def boom(*a, **k):
        raise AssertionError("aten matrix product on the GPU path")

    with monkeypatch.context() as mp:
        for fn in ("matmul", "bmm", "einsum", "addmm", "mm"):
            mp.setattr(torch, fn, boom)
        yg = gpu.forward(xg)
        gy = torch.randn_like(yc)
        gg = gpu.backward(xg, gy.cuda())
    gc = cpu.backward(xc, gy)
    assert _rel(yg, yc) < 1e-2, _rel(yg, yc)
    if isinstance(gc, Table):
        for k in (1, 2):
            if gc[k] is not None and torch.is_tensor(gc[k]) and gc[k].is_floating_point() and gc[k].abs().sum() > 0:
                assert _rel(gg[k], gc[k]) < 2e-2, (k, _rel(gg[k], gc[k]))
    else:
        assert _rel(gg, gc) < 2e-2, _rel(gg, gc)
    for a, b in zip((gpu.parameters() or ([], []))[1], (cpu.parameters() or ([], []))[1]):
        assert _rel(a, b) < 2e-2, (a.shape, _rel(a, b))
