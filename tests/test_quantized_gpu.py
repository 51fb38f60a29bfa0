"""Int8 HIP kernels (csrc/quant.hip) vs exact integer / CPU-emulated references (GPU only)."""
import pytest
import torch
import torch.nn.functional as F

from bigdl_amd import nn
from bigdl_amd.ops import native
from bigdl_amd.quantized import QuantizedLinear, QuantizedSpatialConvolution, quantize_per_sample_ref
from bigdl_amd.quantized.modules import quantize_act_gpu
from bigdl_amd.utils.random_generator import RNG

pytestmark = pytest.mark.gpu
CL = torch.channels_last


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_quantize_act_matches_reference(dtype):
    torch.manual_seed(0)
    x = torch.randn(3, 5, 7, 24).to(dtype)
    q, s = quantize_act_gpu(x.cuda(), 24, 32)
    qr, sr = quantize_per_sample_ref(x)
    assert torch.equal(q.cpu()[..., :24].reshape(3, 5, 7, 24), qr)
    assert torch.all(q.cpu()[..., 24:] == 0)
    assert torch.allclose(s.cpu(), sr)


# N, C, H, W, K, R, S, stride, pad, dil
I8_CASES = [
    (2, 16, 9, 9, 24, 3, 3, 1, 1, 1),
    (3, 64, 14, 14, 200, 1, 1, 1, 0, 1),
    (2, 48, 11, 13, 64, 3, 3, 2, 1, 1),
    (1, 32, 12, 12, 16, 3, 3, 1, 2, 2),
    (4, 128, 7, 7, 130, 3, 3, 1, 1, 1),
    (2, 16, 20, 20, 8, 7, 7, 2, 3, 1),
    (2, 256, 9, 9, 256, 3, 3, 1, 1, 1),     # 36 K-steps through the 3-stage pipeline
    (5, 192, 6, 6, 320, 1, 1, 1, 0, 1),     # Cs % 128 != 0 but % 64 == 0, Ncol tail, M tail
    (2, 64, 12, 12, 64, 3, 3, 1, 1, 1),     # narrow 256 x 64 tile
    (3, 128, 9, 9, 24, 1, 1, 1, 0, 1),      # narrow 256 x 32 tile (Ncol tail)
    (2, 64, 15, 15, 40, 3, 3, 2, 1, 1),     # 256 x 64, stride 2, Ncol tail
]


@pytest.mark.parametrize("cpl", [8, 16])
@pytest.mark.parametrize("g3", [1, 0, 3])
@pytest.mark.parametrize("case", I8_CASES)
def test_conv_i8_exact_integer(case, g3, cpl):
    """Scales are forced to exactly 1 (row maxima 127), so the fp32 output must equal the integer conv — for the
    3-stage counted-vmcnt kernel (BIGDL_I8_G3, 128 x 128 tiles, Cs % 64 == 0; 3 = its 256 x 128 tile) and the 2-stage one."""
    from bigdl_amd.ops.conv import _fwd_taps, out_size

    C_ = native.get()
    old, old_cpl = C_.get_i8_g3(), C_.get_i8_cpl()
    C_.set_i8_g3(g3)
    C_.set_i8_cpl(cpl)     # channels per lane in the 3-stage kernel's LDS-staged epilogue (16: 16-byte stores)
    C_.set_i8_epi(1 if cpl == 16 else 0)   # cpl 16: the register-direct epilogue (BIGDL_I8_EPI=1) where it applies
    try:
        _conv_i8_exact(case)
    finally:
        C_.set_i8_g3(old)
        C_.set_i8_cpl(old_cpl)
        C_.set_i8_epi(0)


I8_SHORTK_CASES = [
    (3, 64, 14, 14, 200, 1, 1, 1, 0, 1),    # one K-step, Ncol tail
    (3, 128, 13, 13, 256, 1, 1, 1, 0, 1),   # two K-steps, M tail
    (2, 64, 15, 15, 136, 1, 1, 2, 0, 1),    # stride 2, Ncol tail
]


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("case", I8_SHORTK_CASES)
def test_conv_i8_shortk_exact_integer(case, mode):
    """Two-stage 128 x 128 short-K int8 kernel (Kdim <= 128; BIGDL_I8_SHORTK 1: 16 channels per lane in the epilogue,
    2: 8; off by default): fp32 output equal to the integer conv."""
    C_ = native.get()
    C_.set_i8_shortk(mode)
    try:
        _conv_i8_exact(case)
    finally:
        C_.set_i8_shortk(0)


I8_P8_CASES = [
    (2, 256, 9, 9, 256, 3, 3, 1, 1, 1),     # one 256 x 256 tile, 18 K-tiles, padding taps
    (3, 1024, 7, 7, 512, 1, 1, 1, 0, 1),    # 1x1, two N tiles, M tail
    (2, 128, 14, 14, 272, 3, 3, 2, 1, 1),   # stride 2, Ncol tail (272)
    (5, 512, 7, 7, 2048, 1, 1, 1, 0, 1),    # 8 N tiles
]


@pytest.mark.parametrize("case", I8_P8_CASES)
def test_conv_i8_p8_exact_integer(case):
    """256 x 256 phase-interleaved int8 kernel (BIGDL_I8_P8=2 forces it wherever Cs % 128 == 0, Kdim >= 1024,
    Ncol >= 256): fp32 output equal to the integer conv."""
    C_ = native.get()
    C_.set_i8_p8(2)
    try:
        _conv_i8_exact(case)
    finally:
        C_.set_i8_p8(1)


@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("g3", [1, 0, 3])
@pytest.mark.parametrize("case", [I8_CASES[1], I8_CASES[4], I8_CASES[7], I8_CASES[9], I8_P8_CASES[1]])
def test_conv_i8_int8_output_exact(case, g3, relu):
    """int8 output (requantized, out_scale 1) with an int8 residual addend: with unit scales the result is the integer
    conv + bias + addend, clamped to [-127, 127] (or [0, 127] with the ReLU) — exact, for every int8 kernel."""
    from bigdl_amd.ops.conv import _fwd_taps, out_size

    C_ = native.get()
    old = C_.get_i8_g3()
    C_.set_i8_g3(g3)
    C_.set_i8_p8(2 if g3 == 3 else 1)   # g3 == 3: the 256 x 256 kernel wherever the shape allows
    try:
        N, C, H, W, K, R, S, st, pd, dl = case
        g = torch.Generator().manual_seed(3)
        x = torch.randint(-3, 4, (N, H, W, C), generator=g, dtype=torch.int8)   # small: most outputs inside the range
        w = torch.randint(-3, 4, (K, R, S, C), generator=g, dtype=torch.int8)
        OH, OW = out_size(H, R, st, pd, dl), out_size(W, S, st, pd, dl)
        ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(0, 3, 1, 2).double(), None, st, pd, dl)
        ref = ref.permute(0, 2, 3, 1).reshape(N * OH * OW, K)
        bias = torch.randint(-20, 21, (K,), generator=g).float()
        add = torch.randint(-127, 128, (N * OH * OW, K), generator=g, dtype=torch.int8)
        exp = (ref + bias.double() + add.double()).clamp(0 if relu else -127, 127).to(torch.int8)
        out = torch.zeros(N * OH * OW, K, dtype=torch.int8, device="cuda")
        ones_x, ones_w = torch.ones(N, device="cuda"), torch.ones(K, device="cuda")
        geo = [N, H, W, C, OH, OW, st, st, R * S * C, K, K, OH, OW, 1, 1, 0, 0]
        C_.conv_i8(x.cuda(), w.cuda(), out, bias.cuda(), ones_x, ones_w, geo, _fwd_taps(R, S, pd, pd, dl, dl), relu,
                   1.0, 1.0, add.view(N, OH, OW, K).cuda(), 1.0)
        torch.cuda.synchronize()
        assert torch.equal(out.cpu(), exp)
    finally:
        C_.set_i8_g3(old)
        C_.set_i8_p8(1)


def _conv_i8_exact(case):
    from bigdl_amd.ops.conv import _fwd_taps, out_size

    N, C, H, W, K, R, S, st, pd, dl = case
    g = torch.Generator().manual_seed(1)
    x = torch.randint(-127, 128, (N, H, W, C), generator=g, dtype=torch.int8)
    w = torch.randint(-127, 128, (K, R, S, C), generator=g, dtype=torch.int8)
    OH, OW = out_size(H, R, st, pd, dl), out_size(W, S, st, pd, dl)
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(0, 3, 1, 2).double(), None, st, pd, dl)
    ref = ref.permute(0, 2, 3, 1).reshape(N * OH * OW, K)
    bias = torch.arange(K, dtype=torch.float32)
    out = torch.full((N * OH * OW, K), float("nan"), device="cuda")
    ones_x, ones_w = torch.ones(N, device="cuda"), torch.ones(K, device="cuda")
    geo = [N, H, W, C, OH, OW, st, st, R * S * C, K, K, OH, OW, 1, 1, 0, 0]
    native.get().conv_i8(x.cuda(), w.cuda(), out, bias.cuda(), ones_x, ones_w, geo,
                         _fwd_taps(R, S, pd, pd, dl, dl), False)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu().double(), ref + bias.double())


def test_quantized_linear_gpu_matches_cpu():
    RNG.setSeed(2)
    f = nn.Linear(300, 77)
    q = QuantizedLinear(300, 77, initWeight=f.weight, initBias=f.bias)
    x = torch.randn(33, 300)
    y_cpu = q.forward(x).clone()
    q.cuda()
    y = q.forward(x.cuda())
    assert y.dtype == torch.float32
    assert torch.allclose(y.cpu(), y_cpu, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("groups", [1, 2])
def test_quantized_conv_gpu_matches_cpu(groups):
    RNG.setSeed(4)
    f = nn.SpatialConvolution(32, 64, 3, 3, 1, 1, 1, 1, nGroup=groups)
    q = QuantizedSpatialConvolution(32, 64, 3, 3, 1, 1, 1, 1, nGroup=groups, initWeight=f.weight, initBias=f.bias)
    q.fuse_relu = True
    x = torch.randn(4, 32, 15, 15)
    y_cpu = q.forward(x).clone()
    q.cuda()
    y = q.forward(x.cuda().contiguous(memory_format=CL))
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=CL)
    assert _rel(y.cpu(), y_cpu) < 1e-2


def test_quantized_resnet_block_model_gpu():
    RNG.setSeed(6)
    seq = nn.Sequential()
    seq.add(nn.SpatialConvolution(3, 32, 3, 3, 1, 1, 1, 1)).add(nn.SpatialBatchNormalization(32)).add(nn.ReLU())
    seq.add(nn.SpatialConvolution(32, 64, 3, 3, 2, 2, 1, 1)).add(nn.SpatialBatchNormalization(64)).add(nn.ReLU())
    seq.add(nn.SpatialAveragePooling(8, 8, 1, 1)).add(nn.Reshape([64])).add(nn.Linear(64, 10))
    seq.evaluate()
    x = torch.randn(8, 3, 16, 16)
    ref = seq.forward(x).clone()
    q = seq.quantize()
    y_cpu = q.forward(x).clone()
    assert _rel(y_cpu, ref) < 0.05
    q.cuda()
    y = q.forward(x.cuda())
    assert _rel(y.float().cpu(), y_cpu) < 2e-2


I8_S1_CASES = [
    # 1x1 stride-1 layers the streaming int8 kernel takes (Cs in {64, 128, 256}, Ncol % 64 == 0)
    (3, 64, 14, 14, 256, 1, 1, 1, 0, 1),    # four channel groups, M tail
    (2, 128, 13, 13, 512, 1, 1, 1, 0, 1),   # two channel blocks
    (4, 256, 9, 9, 64, 1, 1, 1, 0, 1),      # K 256 (4 i8 MFMA K-steps), one channel group
    (5, 64, 11, 11, 128, 1, 1, 1, 0, 1),    # two channel groups
    (2, 256, 7, 7, 192, 1, 1, 1, 0, 1),     # three one-group channel blocks
]


@pytest.mark.parametrize("case", I8_S1_CASES)
def test_conv_i8_s1_exact(case):
    """Streaming 1x1 int8 kernel (conv_i8_s1_kernel): fp32 output equal to the integer conv (unit scales), int8
    output with an int8 residual and ReLU exactly clamped, and the same int8 bytes as the per-tile kernels."""
    from bigdl_amd.ops.conv import _fwd_taps, out_size

    C_ = native.get()
    _conv_i8_exact(case)
    N, C, H, W, K, R, S, st, pd, dl = case
    g = torch.Generator().manual_seed(3)
    x = torch.randint(-3, 4, (N, H, W, C), generator=g, dtype=torch.int8)
    w = torch.randint(-3, 4, (K, R, S, C), generator=g, dtype=torch.int8)
    OH, OW = out_size(H, R, st, pd, dl), out_size(W, S, st, pd, dl)
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(0, 3, 1, 2).double(), None, st, pd, dl)
    ref = ref.permute(0, 2, 3, 1).reshape(N * OH * OW, K)
    bias = torch.randint(-20, 21, (K,), generator=g).float()
    add = torch.randint(-127, 128, (N * OH * OW, K), generator=g, dtype=torch.int8)
    geo = [N, H, W, C, OH, OW, st, st, R * S * C, K, K, OH, OW, 1, 1, 0, 0]
    outs = {}
    for s1 in (1, 0):
        C_.set_i8_s1(s1)
        try:
            for relu in (False, True):
                out = torch.zeros(N * OH * OW, K, dtype=torch.int8, device="cuda")
                C_.conv_i8(x.cuda(), w.cuda(), out, bias.cuda(), torch.ones(N, device="cuda"),
                           torch.ones(K, device="cuda"), geo, _fwd_taps(R, S, pd, pd, dl, dl), relu, 1.0, 1.0,
                           add.view(N, OH, OW, K).cuda(), 1.0)
                bf = torch.zeros(N * OH * OW, K, dtype=torch.bfloat16, device="cuda")
                xs = torch.rand(N, device="cuda") + 0.5
                C_.conv_i8(x.cuda(), w.cuda(), bf, bias.cuda(), xs, torch.ones(K, device="cuda"), geo,
                           _fwd_taps(R, S, pd, pd, dl, dl), relu)
                torch.cuda.synchronize()
                outs[(s1, relu)] = (out.cpu(), bf.float().cpu(), xs.cpu())
        finally:
            C_.set_i8_s1(1)
    for relu in (False, True):
        exp = (ref + bias.double() + add.double()).clamp(0 if relu else -127, 127).to(torch.int8)
        assert torch.equal(outs[(1, relu)][0], exp)
        assert torch.equal(outs[(1, relu)][0], outs[(0, relu)][0])
        xs = outs[(1, relu)][2].double().repeat_interleave(OH * OW).view(-1, 1)
        yb = ref * xs + bias.double()
        if relu:
            yb = yb.clamp(min=0)
        assert _rel(outs[(1, relu)][1], yb) < 1e-2


I8_HALO_CASES = [
    # 3x3 / stride-1 / pad-1 layers the int8 halo-tile kernel takes (csrc/conv_halo.hip EB = 1): H in {56, 28, 14, 7}
    (2, 64, 56, 56, 64, 3, 3, 1, 1, 1),
    (2, 128, 28, 28, 128, 3, 3, 1, 1, 1),
    (3, 256, 14, 14, 256, 3, 3, 1, 1, 1),
    (4, 512, 7, 7, 512, 3, 3, 1, 1, 1),
    (5, 64, 7, 7, 128, 3, 3, 1, 1, 1),
]


@pytest.mark.parametrize("case", I8_HALO_CASES)
def test_conv_i8_halo_exact(case):
    """int8 3x3 halo kernel: fp32 output equal to the integer conv + bias (unit scales), int8 output with ReLU equal to
    the exactly clamped integer result, and the same int8 bytes as the im2col int8 kernels (BIGDL_CONV_HALO off)."""
    from bigdl_amd.ops.conv import _fwd_taps, out_size

    C_ = native.get()
    _conv_i8_exact(case)
    N, C, H, W, K, R, S, st, pd, dl = case
    g = torch.Generator().manual_seed(7)
    x = torch.randint(-4, 5, (N, H, W, C), generator=g, dtype=torch.int8)
    w = torch.randint(-4, 5, (K, R, S, C), generator=g, dtype=torch.int8)
    OH, OW = out_size(H, R, st, pd, dl), out_size(W, S, st, pd, dl)
    ref = F.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(0, 3, 1, 2).double(), None, st, pd, dl)
    ref = ref.permute(0, 2, 3, 1).reshape(N * OH * OW, K)
    bias = torch.randint(-20, 21, (K,), generator=g).float()
    geo = [N, H, W, C, OH, OW, st, st, R * S * C, K, K, OH, OW, 1, 1, 0, 0]
    outs = {}
    for halo in (1, 0):
        C_.set_conv_halo(halo)
        try:
            out = torch.zeros(N * OH * OW, K, dtype=torch.int8, device="cuda")
            C_.conv_i8(x.cuda(), w.cuda(), out, bias.cuda(), torch.ones(N, device="cuda"),
                       torch.ones(K, device="cuda"), geo, _fwd_taps(R, S, pd, pd, dl, dl), True, 1.0, 1.0)
            torch.cuda.synchronize()
            outs[halo] = out.cpu()
        finally:
            C_.set_conv_halo(1)
    exp = (ref + bias.double()).clamp(0, 127).to(torch.int8)
    assert torch.equal(outs[1], exp)
    assert torch.equal(outs[1], outs[0])


@pytest.mark.parametrize("N,H,relu,mode", [(2, 224, True, "i8"), (1, 224, False, "f32"), (3, 224, True, "bf16")])
def test_stem_i8_kernel_exact(N, H, relu, mode):
    """int8 7x7/2 image stem over the width im2col (staged-row kernel, conv_halo.hip stem_i8_kernel): fp32 output equal
    to the exact integer convolution of the quantized image (+ bias, unit scales), and int8 / bf16 outputs equal to the
    generic int8 implicit GEMM's (BIGDL_STEM_I8 off)."""
    from bigdl_amd.ops.conv import _fwd_taps

    C_ = native.get()
    g = torch.Generator().manual_seed(11)
    K, W, OW, OH = 64, 224, 112, H // 2
    x = torch.randint(-40, 41, (N, 3, H, W), generator=g).float()          # integers: quantization at scale 1 is exact
    w = torch.randint(-6, 7, (K, 3, 7, 7), generator=g, dtype=torch.int8)
    q = torch.empty((N, H, OW, 32), dtype=torch.int8, device="cuda")
    C_.quantize_wim2col_f32(x.cuda(), q, OW, 7, 2, 3, 1.0)
    # weight bytes [k][r * 32 + e * 4 + c] (c < 3, e < 7), the im2col's byte order
    wp = torch.zeros(K, 7, 8, 4, dtype=torch.int8)
    wp[:, :, :7, :3] = w.permute(0, 2, 3, 1)
    wp = wp.reshape(K, 224).contiguous()
    bias = torch.randint(-50, 51, (K,), generator=g).float()
    geo = [N, H, OW, 32, OH, OW, 2, 1, 224, K, K, OH, OW, 1, 1, 0, 0]
    dt = {"i8": torch.int8, "f32": torch.float32, "bf16": torch.bfloat16}[mode]
    outs = {}
    for on in (1, 0):
        C_.set_stem_i8(on)
        try:
            out = torch.zeros(N * OH * OW, K, dtype=dt, device="cuda")
            C_.conv_i8(q, wp.cuda(), out, bias.cuda(), None, torch.ones(K, device="cuda"), geo,
                       _fwd_taps(7, 1, 3, 0, 1, 1), relu, 1.0, 1.0 if mode == "i8" else 0.0, None, 0.0)
            torch.cuda.synchronize()
            outs[on] = out.cpu()
        finally:
            C_.set_stem_i8(1)
    # the same from the fp32 image: the kernel quantizes its operands itself (stem_i8f_kernel)
    out = torch.zeros(N * OH * OW, K, dtype=dt, device="cuda")
    assert C_.conv_i8_stem_f32(x.cuda(), wp.cuda(), out, bias.cuda(), torch.ones(K, device="cuda"), geo,
                               _fwd_taps(7, 1, 3, 0, 1, 1), relu, 1.0, 1.0 if mode == "i8" else 0.0)
    torch.cuda.synchronize()
    outs["f"] = out.cpu()
    ref = F.conv2d(x.double(), w.double(), None, 2, 3).permute(0, 2, 3, 1).reshape(-1, K) + bias.double()
    if relu:
        ref = ref.clamp_min(0)
    if mode == "f32":
        assert torch.equal(outs[1].double(), ref)
    if mode == "i8":
        assert torch.equal(outs[1], ref.clamp(-127, 127).round().to(torch.int8))
    assert torch.equal(outs[1], outs[0])
    assert torch.equal(outs["f"], outs[1])


def test_stem_i8_f32_quantizes_like_the_im2col_pass():
    """Non-integer image values at a non-unit scale: the stem that quantizes its own operands gives the same int8
    output as quantize_wim2col_f32 followed by the im2col stem (the same rint(x / scale) per element)."""
    from bigdl_amd.ops.conv import _fwd_taps

    C_ = native.get()
    g = torch.Generator().manual_seed(5)
    N, H, K, OW = 2, 224, 64, 112
    x = torch.randn(N, 3, H, 224, generator=g) * 2.0
    scale = float(x.abs().max()) / 127.0
    w = torch.randint(-20, 21, (K, 224), generator=g, dtype=torch.int8)
    w.view(K, 7, 8, 4)[:, :, 7, :] = 0
    w.view(K, 7, 8, 4)[:, :, :, 3] = 0
    ws = torch.rand(K, generator=g) * 0.01 + 0.001
    bias = torch.randn(K, generator=g)
    geo = [N, H, OW, 32, OH := H // 2, OW, 2, 1, 224, K, K, OH, OW, 1, 1, 0, 0]
    taps = _fwd_taps(7, 1, 3, 0, 1, 1)
    q = torch.empty((N, H, OW, 32), dtype=torch.int8, device="cuda")
    C_.quantize_wim2col_f32(x.cuda(), q, OW, 7, 2, 3, scale)
    a = torch.zeros(N * OH * OW, K, dtype=torch.int8, device="cuda")
    C_.conv_i8(q, w.cuda(), a, bias.cuda(), None, ws.cuda(), geo, taps, True, scale, 0.05, None, 0.0)
    b = torch.zeros_like(a)
    assert C_.conv_i8_stem_f32(x.cuda(), w.cuda(), b, bias.cuda(), ws.cuda(), geo, taps, True, scale, 0.05)
    torch.cuda.synchronize()
    assert torch.equal(a.cpu(), b.cpu())
