"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference of the same op (GPU only)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CL = torch.channels_last
BF = torch.bfloat16


def _dev():
    return torch.device("cuda:0")


def _rel(a, b):
    a = a.float()
    b = b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


CONV_CASES = [
    # N, C, H, W, K, R, S, stride, pad
    (2, 64, 14, 14, 64, 3, 3, 1, 1),
    (2, 64, 14, 14, 128, 1, 1, 1, 0),
    (3, 32, 9, 11, 48, 3, 3, 2, 1),
    (2, 128, 8, 8, 256, 1, 1, 2, 0),
    (2, 8, 30, 30, 64, 7, 7, 2, 3),     # stem-like (C padded to 8)
    (4, 256, 7, 7, 512, 3, 3, 1, 1),
    (1, 16, 5, 5, 24, 5, 5, 1, 0),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(case):
    from bigdl_amd.ops import conv as cv

    N, C, H, W, K, R, S, st, pd = case
    torch.manual_seed(0)
    dev = _dev()
    x32 = torch.randn(N, C, H, W, device=dev)
    w32 = torch.randn(K, C, R, S, device=dev) * (1.0 / (C * R * S) ** 0.5)
    b32 = torch.randn(K, device=dev)
    x = x32.to(BF, memory_format=CL)
    w = w32.to(BF, memory_format=CL)
    xr, wr = x.float(), w.float()
    # forward (+bias, +stats)
    from bigdl_amd.ops import bn as bnops

    stats = bnops.new_stats(K, dev)
    y = cv.conv2d_fwd(x, w, b32, (st, st), (pd, pd), stats=stats)
    # fp32 references on the CPU (small shapes; keeps MIOpen's find-mode solver evaluation out of the GPU tier)
    xr, wr = xr.cpu(), wr.cpu()
    yr = F.conv2d(xr, wr, b32.cpu(), stride=st, padding=pd).to(dev)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-2
    st2 = stats.view(bnops.stat_slots(), 2, K).sum(0)
    assert _rel(st2[0], y.float().sum(dim=(0, 2, 3))) < 2e-2
    assert _rel(st2[1], (y.float() ** 2).sum(dim=(0, 2, 3))) < 2e-2
    # relu epilogue
    y2 = cv.conv2d_fwd(x, w, b32, (st, st), (pd, pd), relu=True)
    assert _rel(y2, torch.relu(yr)) < 1e-2
    # dgrad
    gy = torch.randn_like(yr).to(BF, memory_format=CL)
    wt = cv.transpose_w(w)
    dx = cv.conv2d_dgrad(gy, wt, x.shape, (st, st), (pd, pd))
    dxr = torch.nn.grad.conv2d_input(x.shape, wr, gy.float().cpu(), stride=st, padding=pd).to(dev)
    assert _rel(dx, dxr) < 1e-2
    # wgrad
    dw = torch.zeros(K, C, R, S, device=dev).contiguous(memory_format=CL)
    db = torch.zeros(K, device=dev)
    cv.conv2d_wgrad(gy, x, dw, db, (st, st), (pd, pd))
    dwr = torch.nn.grad.conv2d_weight(xr, wr.shape, gy.float().cpu(), stride=st, padding=pd).to(dev)
    assert _rel(dw, dwr) < 1e-2
    assert _rel(db, gy.float().sum(dim=(0, 2, 3))) < 1e-2


BIG_CASES = [
    # N, C, H, K, R, stride, pad: grids large enough for the 256-pixel deep-pipelined kernel
    (32, 64, 56, 128, 3, 1, 1),
    (32, 256, 56, 64, 1, 1, 0),
    (16, 128, 56, 256, 3, 2, 1),
    (8, 512, 28, 1000, 1, 1, 0),     # Ncol tail (1000 % 128 != 0)
    (16, 64, 56, 200, 1, 1, 0),      # persistent kernel: 784 tiles, Ncol tail
    (24, 64, 57, 128, 1, 1, 0),      # persistent kernel: M tail
]


@pytest.mark.parametrize("impl", [0, 1, 2, 3])
@pytest.mark.parametrize("case", BIG_CASES)
def test_conv_nt_variants_large(case, impl):
    """Register-staged (0), LDS-DMA (1), deep-pipelined 3-stage LDS-DMA (2) and persistent LDS-DMA (3) NT
    kernels, fwd (+stats) and dgrad, vs fp32 torch."""
    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import conv as cv
    from bigdl_amd.ops import native

    N, C, H, K, R, st, pd = case
    C_ = native.get()
    old = C_.get_conv_impl()
    C_.set_conv_impl(impl)
    try:
        torch.manual_seed(1)
        dev = _dev()
        x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
        w = (torch.randn(K, C, R, R, device=dev) * (1.0 / (C * R * R) ** 0.5)).to(BF, memory_format=CL)
        stats = bnops.new_stats(K, dev)
        y = cv.conv2d_fwd(x, w, None, (st, st), (pd, pd), stats=stats)
        yr = F.conv2d(x.float(), w.float(), None, stride=st, padding=pd)
        assert _rel(y, yr) < 1e-2
        st2 = stats.view(bnops.stat_slots(), 2, K).sum(0)
        assert _rel(st2[0], y.float().sum(dim=(0, 2, 3))) < 2e-2
        gy = torch.randn_like(yr).to(BF, memory_format=CL)
        dx = cv.conv2d_dgrad(gy, cv.transpose_w(w), x.shape, (st, st), (pd, pd))
        dxr = torch.nn.grad.conv2d_input(x.shape, w.float(), gy.float(), stride=st, padding=pd)
        assert _rel(dx, dxr) < 1e-2
    finally:
        C_.set_conv_impl(old)


WGRAD_CASES = [
    # N, C, H, K, R, stride, pad: split-K workspace and atomic paths, incl. 64-column layers and the stem
    (16, 64, 56, 64, 3, 1, 1),
    (16, 256, 56, 64, 1, 1, 0),
    (8, 8, 224, 64, 7, 2, 3),
    (16, 64, 56, 256, 1, 1, 0),
    (8, 40, 30, 48, 3, 1, 1),       # Ncol < 64 and Kdim tails
]


@pytest.mark.parametrize("case", WGRAD_CASES)
def test_conv_wgrad_large(case):
    """Weight gradient (+bias) at ResNet-like sizes (split-K LDS-DMA and atomic kernels) vs fp32 torch."""
    from bigdl_amd.ops import conv as cv

    N, C, H, K, R, st, pd = case
    torch.manual_seed(2)
    dev = _dev()
    x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
    w = (torch.randn(K, C, R, R, device=dev) * (1.0 / (C * R * R) ** 0.5)).to(BF, memory_format=CL)
    yr = F.conv2d(x.float(), w.float(), None, stride=st, padding=pd)
    gy = torch.randn_like(yr).to(BF, memory_format=CL)
    dw = torch.zeros(K, C, R, R, device=dev).contiguous(memory_format=CL)
    db = torch.zeros(K, device=dev)
    cv.conv2d_wgrad(gy, x, dw, db, (st, st), (pd, pd))
    dwr = torch.nn.grad.conv2d_weight(x.float(), w.shape, gy.float(), stride=st, padding=pd)
    assert _rel(dw, dwr) < 1e-2
    assert _rel(db, gy.float().sum(dim=(0, 2, 3))) < 1e-2


def test_linear_as_conv1x1():
    from bigdl_amd.ops import conv as cv

    dev = _dev()
    B, I, O = 37, 96, 200
    x = torch.randn(B, I, 1, 1, device=dev).to(BF, memory_format=CL)
    w = (torch.randn(O, I, 1, 1, device=dev) * 0.1).to(BF, memory_format=CL)
    y = cv.conv2d_fwd(x, w, None, (1, 1), (0, 0))
    assert _rel(y.view(B, O), x.view(B, I).float() @ w.view(O, I).float().t()) < 1e-2


@pytest.mark.parametrize("res,relu", [(False, False), (False, True), (True, True)])
def test_bn_fwd_bwd(res, relu):
    from bigdl_amd.ops import bn

    dev = _dev()
    N, C, H, W = 4, 64, 9, 7
    x = (torch.randn(N, C, H, W, device=dev) * 2 + 0.5).to(BF, memory_format=CL)
    r = torch.randn(N, C, H, W, device=dev).to(BF, memory_format=CL) if res else None
    g = torch.rand(C, device=dev) + 0.5
    b = torch.randn(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    y, sm, si, aff = bn.bn_forward_gpu(x, g, b, rm, rv, 1e-3, 0.1, True, res=r, relu=relu)
    xr = x.float().requires_grad_(True)
    ref = F.batch_norm(xr, None, None, g, b, True, 0.1, 1e-3)
    if res:
        ref = ref + r.float()
    if relu:
        ref = torch.relu(ref)
    assert _rel(y, ref) < 1e-2
    assert _rel(rm, 0.1 * x.float().mean(dim=(0, 2, 3))) < 1e-3
    gz = torch.randn_like(ref)
    ref.backward(gz)
    dg, dbt = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    gzb = gz.to(BF, memory_format=CL)
    dx, dres = bn.bn_backward_gpu(gzb, y if relu else None, x, sm, si, g, dg, dbt, need_dres=res)
    # reference computed on the bf16-rounded gradient
    xr2 = x.float().requires_grad_(True)
    out2 = F.batch_norm(xr2, None, None, g, b, True, 0.1, 1e-3)
    if res:
        out2 = out2 + r.float()
    if relu:
        out2 = torch.relu(out2)
    out2.backward(gzb.float())
    assert _rel(dx, xr2.grad) < 2e-2
    if relu and not res:       # mask recomputed from x*scale + shift instead of reading y back
        dg2, db2 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dx2, _ = bn.bn_backward_gpu(gzb, None, x, sm, si, g, dg2, db2, aff=aff)
        assert _rel(dx2, dx) < 1e-3 and _rel(dg2, dg) < 1e-3 and _rel(db2, dbt) < 1e-3
    if res:
        mask = (y.float() > 0).float() if relu else 1.0
        assert _rel(dres, gzb.float() * mask) < 1e-2
    if relu and res:
        # sign-mask path (bn_apply writes one bit per element; the backward reads it instead of y): same y, the same
        # residual gradient bit for bit, and the same gradients / reductions up to fp32 atomic order
        rm2, rv2 = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        zm = torch.full((N * C * H * W // 8,), 0x5A, dtype=torch.uint8, device=dev)
        y2, sm2, si2, _ = bn.bn_forward_gpu(x, g, b, rm2, rv2, 1e-3, 0.1, True, res=r, relu=relu, zm=zm)
        assert torch.equal(y2, y)
        bits = torch.stack([(zm >> e) & 1 for e in range(8)], dim=1).reshape(N, H, W, C).permute(0, 3, 1, 2)
        assert torch.equal(bits.bool(), y.float() > 0)
        dg3, db3 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        dx3, dres3 = bn.bn_backward_gpu(gzb, None, x, sm2, si2, g, dg3, db3, need_dres=True, zm=zm)
        assert torch.equal(dres3, dres)
        assert _rel(dx3, dx) < 1e-5 and _rel(dg3, dg) < 1e-5 and _rel(db3, dbt) < 1e-5


@pytest.mark.parametrize("C,zmask", [(64, True), (256, False), (512, True), (2048, True), (24, True)])
def test_bn_bwd_apply_second_bn_reduction(C, zmask):
    """The residual-branch gradient pass also reducing a second (ReLU-less) BN over dres (projection shortcut): the
    slotted sums equal bn_bwd_reduce over the dres it wrote, and dx / dres are unchanged bit for bit."""
    from bigdl_amd.ops import bn, native

    dev = _dev()
    torch.manual_seed(2)
    N, H, W = 3, 7, 9
    x = (torch.randn(N, C, H, W, device=dev) * 2 + 0.5).to(BF, memory_format=CL)
    r = torch.randn(N, C, H, W, device=dev).to(BF, memory_format=CL)
    x2 = (torch.randn(N, C, H, W, device=dev) - 0.2).to(BF, memory_format=CL)
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    zm = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev) if zmask else None
    y, sm, si, _ = bn.bn_forward_gpu(x, g, b, rm, rv, 1e-3, 0.1, True, res=r, relu=True, zm=zm)
    z = None if zmask else y
    mean2 = torch.randn(C, device=dev) * 0.1
    gz = torch.randn(N, C, H, W, device=dev).to(BF, memory_format=CL)
    dg0, db0 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dx0, dres0 = bn.bn_backward_gpu(gz, z, x, sm, si, g, dg0, db0, need_dres=True, zm=zm)
    red2 = bn.new_stats(C, dev)
    dg1, db1 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dx1, dres1 = bn.bn_backward_gpu(gz, z, x, sm, si, g, dg1, db1, need_dres=True, zm=zm, sec=(x2, mean2, red2))
    assert torch.equal(dres1, dres0) and _rel(dx1, dx0) < 1e-5
    ref = bn.new_stats(C, dev)
    native.get().bn_bwd_reduce(dres0, None, x2, mean2, ref, N * H * W, C, None, None)
    assert torch.allclose(red2.view(-1, 2 * C).sum(0), ref.view(-1, 2 * C).sum(0), rtol=1e-4, atol=1e-3)


def test_maxpool_avgpool():
    from bigdl_amd.ops import pool

    dev = _dev()
    x = torch.randn(2, 64, 15, 15, device=dev).to(BF, memory_format=CL)
    y, idx = pool.maxpool_fwd_gpu(x, 3, 3, 2, 2, 1, 1)
    xr = x.float().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(y.float(), yr)
    gy = torch.randn_like(yr).to(BF, memory_format=CL)
    dx = pool.maxpool_bwd_gpu(gy, idx, x.shape, 3, 3, 2, 2, 1, 1)
    yr.backward(gy.float())
    assert _rel(dx, xr.grad) < 1e-2
    a = pool.avgpool_fwd_gpu(x, 7, 7, 1, 1, 0, 0)
    xr = x.float().requires_grad_(True)
    ar = F.avg_pool2d(xr, 7, 1, 0)
    assert _rel(a, ar) < 1e-2
    ga = torch.randn_like(ar).to(BF, memory_format=CL)
    da = pool.avgpool_bwd_gpu(ga, x.shape, 7, 7, 1, 1, 0, 0)
    ar.backward(ga.float())
    assert _rel(da, xr.grad) < 1e-2


@pytest.mark.parametrize("shape,k,s,p,ceil", [((2, 64, 15, 15), 3, 2, 1, False), ((3, 24, 16, 13), 3, 2, 0, True),
                                                ((2, 8, 112, 112), 3, 2, 1, False), ((2, 16, 9, 9), 3, 1, 1, False),
                                                ((3, 16, 20, 14), 3, 2, 1, False),
                                                ((2, 32, 10, 11), 2, 2, 0, False)])
def test_maxpool_window_variants(shape, k, s, p, ceil):
    """The fixed 3x3/2 kernels and the generic ones against torch (values exact, gradients summed per winner)."""
    from bigdl_amd.ops import pool

    torch.manual_seed(0)
    x = torch.randn(*shape, device=_dev()).to(BF, memory_format=CL)
    y, idx = pool.maxpool_fwd_gpu(x, k, k, s, s, p, p, ceil)
    xr = x.float().requires_grad_(True)
    yr = F.max_pool2d(xr, k, s, p, ceil_mode=ceil)
    assert y.shape == yr.shape and torch.equal(y.float(), yr)
    gy = torch.randn_like(yr).to(BF, memory_format=CL)
    dx = pool.maxpool_bwd_gpu(gy, idx, x.shape, k, k, s, s, p, p)
    yr.backward(gy.float())
    assert _rel(dx, xr.grad) < 1e-2


@pytest.mark.parametrize("shape,mask", [((4, 64, 28, 22), "aff"), ((3, 64, 16, 20), "zm"), ((2, 128, 12, 14), "aff"),
                                        ((2, 16, 10, 8), "zm")])
def test_maxpool_bwd_bn_reduction(shape, mask):
    """k3 s2 maxpool backward fused with the producing BN's backward reduction (the ResNet stem): dx bit-exact vs the
    plain kernel, the slotted sums vs bn_bwd_reduce over that dx, and the BN backward from them vs the unfused one."""
    from bigdl_amd.ops import bn, native, pool

    dev = _dev()
    torch.manual_seed(1)
    N, C, H, W = shape
    x = (torch.randn(*shape, device=dev) * 2 + 0.3).to(BF, memory_format=CL)
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    zm = torch.empty(x.numel() // 8, dtype=torch.uint8, device=dev) if mask == "zm" else None
    y, sm, si, aff = bn.bn_forward_gpu(x, g, b, rm, rv, 1e-3, 0.1, True, relu=True, zm=zm)
    p, idx = pool.maxpool_fwd_gpu(y, 3, 3, 2, 2, 1, 1)
    gp = torch.randn(p.shape, device=dev).to(BF, memory_format=CL)
    dx0 = pool.maxpool_bwd_gpu(gp, idx, y.shape, 3, 3, 2, 2, 1, 1)
    src = (None, x, sm, aff if zm is None else None, zm if zm is not None else False)
    dx1, red = pool.maxpool_bwd_bnred_gpu(gp, idx, y.shape, 3, 3, 2, 2, 1, 1, src)
    assert red is not None and torch.equal(dx1, dx0)
    C_ = native.get()
    ref = bn.new_stats(C, dev)
    C_.bn_bwd_reduce(dx0, None, x, sm, ref, N * H * W, C, aff if zm is None else None, zm)
    s_fused = red.view(-1, 2 * C).sum(0)
    s_ref = ref.view(-1, 2 * C).sum(0)
    assert torch.allclose(s_fused, s_ref, rtol=1e-4, atol=1e-3)
    dg0, db0 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dg1, db1 = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    kw = dict(aff=aff) if zm is None else dict(zm=zm)
    bx0, _ = bn.bn_backward_gpu(dx0, None, x, sm, si, g, dg0, db0, **kw)
    bx1, _ = bn.bn_backward_gpu(dx1, None, x, sm, si, g, dg1, db1, red=red, **kw)
    assert _rel(bx1, bx0) < 1e-3 and _rel(dg1, dg0) < 1e-4 and _rel(db1, db0) < 1e-4


def test_softmax_xent():
    from bigdl_amd import ops

    dev = _dev()
    B, K = 33, 1000
    logits = torch.randn(B, K, device=dev).to(BF)
    labels = torch.randint(1, K + 1, (B,), device=dev).float()
    loss, dl = ops.softmax_xent_gpu(logits, labels, label_base=1.0)
    lr = logits.float().requires_grad_(True)
    ref = F.cross_entropy(lr, labels.long() - 1)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-3 * max(1.0, abs(ref.item()))
    assert _rel(dl, lr.grad) < 1e-2


def test_relu_add_cast():
    from bigdl_amd import ops

    dev = _dev()
    x = torch.randn(1001, device=dev).to(BF)
    y = ops.relu_gpu(x)
    assert torch.equal(y, torch.relu(x))
    dy = torch.randn(1001, device=dev).to(BF)
    dx = ops.relu_bwd_gpu(dy, y)
    assert torch.equal(dx, dy * (y > 0))
    z = ops.add_gpu(x, dy)
    assert _rel(z, x.float() + dy.float()) < 1e-2
    f = torch.randn(1003, device=dev)
    assert _rel(ops.to_f32(ops.to_bf16(f)), f) < 1e-2


def test_sgd_adam_kernels():
    from bigdl_amd.ops import native

    C = native.get()
    dev = _dev()
    n = 5000
    w = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    mom = torch.zeros(n, device=dev)
    w16 = torch.empty(n, dtype=BF, device=dev)
    wr, br = w.clone(), None
    for it in range(3):
        C.sgd_step(w, g, mom, w16, 0.1, 1e-4, 0.9, 0.0, False, it == 0)
        d = g + 1e-4 * wr
        br = d.clone() if br is None else 0.9 * br + d
        wr = wr - 0.1 * br
    assert _rel(w, wr) < 1e-5
    assert _rel(w16, wr) < 1e-2
    s = torch.zeros(1, device=dev)
    C.sumsq(g, s)
    assert abs(s.item() - (g * g).sum().item()) < 1e-2 * s.item()


def test_lstm_cell():
    from bigdl_amd.ops import native

    C = native.get()
    dev = _dev()
    B, H = 5, 33
    gates = torch.randn(B, 4 * H, device=dev, requires_grad=True)
    cp = torch.randn(B, H, device=dev, requires_grad=True)
    c = torch.empty(B, H, device=dev)
    h = torch.empty(B, H, device=dev)
    act = torch.empty(B, 4 * H, device=dev)
    C.lstm_cell_fwd(gates.detach(), cp.detach(), c, h, act)
    i, gg, f, o = gates.split(H, dim=1)
    cr = torch.sigmoid(f) * cp + torch.sigmoid(i) * torch.tanh(gg)
    hr = torch.sigmoid(o) * torch.tanh(cr)
    assert _rel(c, cr) < 1e-5 and _rel(h, hr) < 1e-5
    dh = torch.randn(B, H, device=dev)
    dcn = torch.randn(B, H, device=dev)
    (hr * dh + cr * dcn).sum().backward()
    dg = torch.empty(B, 4 * H, device=dev)
    dcp = torch.empty(B, H, device=dev)
    C.lstm_cell_bwd(act, cp.detach(), c, dh, dcn, dg, dcp)
    assert _rel(dg, gates.grad) < 1e-4
    assert _rel(dcp, cp.grad) < 1e-4


@pytest.mark.parametrize("nhwc", [False, True])
def test_image_augment_kernel(nhwc):
    from bigdl_amd.ops.image import augment_batch, augment_batch_ref, random_crop_params

    torch.manual_seed(0)
    src = torch.randint(0, 256, (6, 40, 48, 3), dtype=torch.uint8)
    p = random_crop_params(6, 40, 48, 32, 30)
    mean, std = (123.7, 116.3, 103.5), (58.4, 57.1, 57.4)
    ref = augment_batch_ref(src, p, 32, 30, mean, std, True, nhwc)
    out = augment_batch(src.cuda(), p, 32, 30, mean, std, True, nhwc).cpu()
    assert torch.allclose(out.float(), ref.float(), atol=2e-2 if nhwc else 1e-5)


# ---------------------------------------------------------------------------------------------- misc NN kernels
def test_lrn_kernel_matches_fp32_reference():
    from bigdl_amd.ops import nnk

    torch.manual_seed(0)
    for size in (5, 4):
        x = torch.randn(3, 13, 7, 5)
        ref_y = nnk.lrn_cpu(x.double(), size, 1e-2, 0.75, 2.0).float()
        xr = x.clone().double().requires_grad_(True)
        gy = torch.randn_like(x)
        nnk.lrn_cpu(xr, size, 1e-2, 0.75, 2.0).backward(gy.double())
        xg = x.cuda().requires_grad_(True)
        y = nnk.lrn(xg, size, 1e-2, 0.75, 2.0)
        y.backward(gy.cuda())
        assert torch.allclose(y.cpu(), ref_y, atol=1e-5, rtol=1e-4)
        assert torch.allclose(xg.grad.cpu(), xr.grad.float(), atol=1e-5, rtol=1e-4)
    if True:   # odd size agrees with torch's LRN too
        x = torch.randn(2, 9, 4, 4)
        assert torch.allclose(nnk.lrn_cpu(x, 5, 1e-3, 0.75, 1.0),
                              torch.nn.functional.local_response_norm(x, 5, 1e-3, 0.75, 1.0), atol=1e-6)


def test_dropout_kernel_mask_regenerated():
    from bigdl_amd import nn

    torch.manual_seed(0)
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(1001, 33, device="cuda").to(dt)
        d = nn.Dropout(0.3)
        y = d.forward(x)
        keep = (y != 0)
        frac = keep.float().mean().item()
        assert abs(frac - 0.7) < 0.01
        assert torch.allclose(y[keep].float(), (x[keep].float() / 0.7), rtol=1e-2)
        g = d.backward(x, torch.ones_like(x))
        assert torch.equal(g != 0, keep)
        y2 = d.forward(x)
        assert not torch.equal(y2 != 0, keep)          # a fresh mask each forward


def test_embedding_kernels_match_reference():
    from bigdl_amd import nn

    torch.manual_seed(0)
    lt = nn.LookupTable(50, 24)
    idx = torch.randint(1, 51, (7, 9)).float()
    ref = lt.weight[idx.long() - 1]
    gy = torch.randn(7, 9, 24)
    ref_g = torch.zeros(50, 24).index_add_(0, idx.long().reshape(-1) - 1, gy.reshape(-1, 24))
    lt = lt.to(torch.device("cuda"))
    out = lt.forward(idx.cuda())
    lt.zeroGradParameters()
    lt.backward(idx.cuda(), gy.cuda())
    assert torch.allclose(out.cpu(), ref)
    assert torch.allclose(lt.gradWeight.cpu(), ref_g, atol=1e-5)


@pytest.mark.parametrize("mask_zero,pad,ids_long,gbf16", [(False, 0, False, False), (True, 0, False, True),
                                                           (False, 3, True, False), (True, 5, True, True)])
def test_embedding_raw_id_kernels(mask_zero, pad, ids_long, gbf16):
    """LookupTable's GPU path reads the raw 1-based ids (f32 / int64) in the kernels: zero-id rows (maskZero -> zero
    row, else row 0), padding ids skipped in the gradient, bf16 output gradients; vs the reference index arithmetic."""
    from bigdl_amd import nn

    torch.manual_seed(1)
    lt = nn.LookupTable(40, 16, paddingValue=float(pad), maskZero=mask_zero)
    ids = torch.randint(0 if mask_zero else 1, 41, (6, 11)).float()
    ids[0, :3] = 0 if mask_zero else 1
    if pad:
        ids[1, :4] = pad
    idx = ids.long() - 1
    ref = lt.weight[idx.clamp_min(0)] * ((idx >= 0) | (not mask_zero)).unsqueeze(-1).float()
    gy = torch.randn(6, 11, 16)
    if gbf16:
        gy = gy.to(torch.bfloat16).float()
    keep = (idx >= 0) & ((idx != pad - 1) if pad else True)
    ref_g = torch.zeros(40, 16).index_add_(0, idx[keep], gy[keep])
    lt = lt.to(torch.device("cuda"))
    x = ids.long().cuda() if ids_long else ids.cuda()
    out = lt.forward(x)
    lt.zeroGradParameters()
    lt.backward(x, gy.cuda().to(torch.bfloat16) if gbf16 else gy.cuda())
    assert torch.allclose(out.cpu(), ref)
    assert torch.allclose(lt.gradWeight.cpu(), ref_g, atol=1e-5)


def test_resize_bilinear_and_log_softmax_kernels():
    from bigdl_amd.ops import nnk

    torch.manual_seed(0)
    for align in (False, True):
        x = torch.randn(2, 3, 5, 7)
        gy = torch.randn(2, 3, 9, 4)
        xr = x.clone().requires_grad_(True)
        ref = nnk.resize_bilinear_cpu(xr, 9, 4, align)
        ref.backward(gy)
        xg = x.cuda().requires_grad_(True)
        y = nnk.resize_bilinear(xg, 9, 4, align)
        y.backward(gy.cuda())
        assert torch.allclose(y.cpu(), ref.detach(), atol=1e-5)
        assert torch.allclose(xg.grad.cpu(), xr.grad, atol=1e-5)
    x = torch.randn(37, 1000) * 4
    gy = torch.randn(37, 1000)
    xr = x.clone().requires_grad_(True)
    torch.log_softmax(xr, -1).backward(gy)
    xg = x.cuda().requires_grad_(True)
    y = nnk.log_softmax(xg)
    y.backward(gy.cuda())
    assert torch.allclose(y.cpu(), torch.log_softmax(x, -1), atol=1e-5)
    assert torch.allclose(xg.grad.cpu(), xr.grad, atol=1e-5)


def test_bf16_truncation_kernel():
    from bigdl_amd.ops import nnk

    x = torch.randn(4099) * 100
    ref = nnk.f32_to_bf16_rtz(x)
    got = nnk.f32_to_bf16_rtz(x.cuda()).cpu()
    assert torch.equal(got.view(torch.int16), ref.view(torch.int16))
    assert torch.all(got.float().abs() <= x.abs())         # toward zero


@pytest.mark.parametrize("K,C,R", [(64, 8, 7), (200, 72, 3), (1000, 2048, 1), (3, 5, 2)])
def test_transpose_krsc_exact(K, C, R):
    from bigdl_amd.ops import conv as cv

    dev = _dev()
    w = torch.randn(K, C, R, R, device=dev).to(BF, memory_format=CL)
    wt = cv.transpose_w(w)
    ref = w.permute(1, 2, 3, 0).contiguous()      # (C, R, S, K)
    assert torch.equal(wt, ref)


@pytest.mark.parametrize("shape", [(3, 3, 17, 19), (2, 12, 5, 7), (4, 3, 224, 224)])
def test_nchw_to_nhwc_bf16_exact(shape):
    from bigdl_amd.ops import conv as cv

    dev = _dev()
    x = torch.randn(*shape, device=dev)
    y = cv.to_nhwc_bf16(x)
    C = shape[1]
    assert y.shape[1] % 8 == 0 and y.is_contiguous(memory_format=CL)
    assert torch.equal(y[:, :C].float(), x.to(BF).float())
    assert not y[:, C:].float().any()


@pytest.mark.parametrize("P,K,C,bias", [(16384, 1000, 1024, True), (300, 2048, 512, False), (4096, 4096, 1024, False)])
def test_gemm_shaped_wgrad_on_nt_kernel_matches_fp32(P, K, C, bias):
    """Large 1x1 / Linear weight gradients run as an NT MFMA GEMM over transposed operands with an fp32
    accumulating epilogue (ops/conv.gemm_wgrad_nt); compare against the fp32 torch product."""
    from bigdl_amd.ops import conv as cv

    torch.manual_seed(0)
    dy = torch.randn(P, K, device="cuda").to(torch.bfloat16)
    x = torch.randn(P, C, device="cuda").to(torch.bfloat16)
    dw = torch.randn(K, C, 1, 1, device="cuda")
    db = torch.randn(K, device="cuda") if bias else None
    ref = dw.view(K, C) + dy.float().t() @ x.float()
    refb = db + dy.float().sum(0) if bias else None
    cv.conv2d_wgrad(dy.view(P, K, 1, 1), x.view(P, C, 1, 1), dw, db, (1, 1), (0, 0))
    err = ((dw.view(K, C) - ref).norm() / ref.norm()).item()
    assert err < 1e-3, err
    if bias:
        assert torch.allclose(db, refb, rtol=1e-3, atol=1e-2)


def test_batched_weight_transpose_matches_per_layer():
    """transpose_krsc_batched (one launch for every conv of a step) equals the per-layer transpose."""
    from bigdl_amd.ops import conv as cv

    class _Fake:
        _w16_managed = True

        def __init__(self, w):
            self.w = w
            self.weight = w

        def _w16_padded(self):
            return self.w

    torch.manual_seed(0)
    mods = [_Fake(torch.randn(k, c, r, r, device=_dev()).to(BF, memory_format=CL))
            for k, c, r in [(64, 8, 7), (256, 64, 1), (64, 64, 3), (512, 1024, 1), (40, 24, 3)]]
    n = cv.prepare_dgrad_weights(mods)
    assert n == 5
    for m in mods:
        assert m._wt_stamp == cv.WT_STAMP[0]
        assert torch.equal(m._wt_cache, cv.transpose_w(m.w))
    cv.end_dgrad_weights()
    assert all(m._wt_stamp != cv.WT_STAMP[0] for m in mods)


def test_train_step_with_batched_transposes_matches_per_layer(monkeypatch):
    """A ResNet training step gives the same weight gradients whether the dgrad weights come from the batched
    pre-transpose or from per-layer transposes."""
    import copy

    from bigdl_amd import nn
    from bigdl_amd.models.resnet import ResNet
    from bigdl_amd.ops import conv as cv
    from bigdl_amd.optim.sgd import SGD
    from bigdl_amd.optim.train_step import TrainStep
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(3)
    base = ResNet(10, 20, dataSet="CIFAR10")
    x = torch.randn(16, 3, 32, 32, device=_dev())
    y = torch.randint(1, 11, (16,), device=_dev()).float()
    grads = {}
    for mode in ("batched", "per_layer"):
        if mode == "per_layer":
            monkeypatch.setattr(cv, "prepare_dgrad_weights", lambda convs: cv.WT_STAMP.__setitem__(0, cv.WT_STAMP[0] + 1))
        step = TrainStep(copy.deepcopy(base), nn.CrossEntropyCriterion(), SGD(learningRate=0.0), device=_dev())
        builds = cv.DESC_BUILDS[0]
        for _ in range(3):
            step.zero_grad()
            step.forward_backward(x, y)
        torch.cuda.synchronize()
        grads[mode] = step.g.clone()
        if mode == "batched":
            assert cv.DESC_BUILDS[0] - builds == 1      # one descriptor table for all steps (graph-capture safe)
    assert _rel(grads["batched"], grads["per_layer"]) < 1e-6


W8_CASES = [
    # N, C, H, K, R, stride, pad -> routed to the 256 x 256 8-wave kernel (Cs % 32 == 0, Ncol >= 256)
    (16, 256, 56, 256, 1, 1, 0),     # 196 tiles x 8 K-steps: one pass, no split
    (16, 256, 28, 512, 3, 1, 1),     # 98 tiles x 72 K-steps: split-K 4 + split-K epilogue
    (4, 512, 7, 2048, 1, 1, 0),      # 8 tiles: split-K 2
    (8, 128, 28, 320, 3, 1, 1),      # Ncol tail (320 % 256 != 0)
    (16, 256, 28, 256, 3, 2, 1),     # stride 2: dgrad phases write a strided output placement
    (66, 256, 28, 256, 1, 1, 0),     # >= 200 tiles, M tail
]


@pytest.mark.parametrize("case", W8_CASES)
def test_conv_w8_kernel_fwd_dgrad_bnred(case):
    """256 x 256 8-wave LDS-DMA kernel (4 stages, counted vmcnt) and its split-K path vs fp32 torch: forward with
    bias + BN statistics and with bias + ReLU, data gradient with a residual addend and the fused backward
    reduction of the consumer BatchNorm (sum dy, sum dy * (x - mean) under the ReLU mask)."""
    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import conv as cv

    N, C, H, K, R, st, pd = case
    torch.manual_seed(5)
    dev = _dev()
    x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
    w = (torch.randn(K, C, R, R, device=dev) * (1.0 / (C * R * R) ** 0.5)).to(BF, memory_format=CL)
    b32 = torch.randn(K, device=dev)
    stats = bnops.new_stats(K, dev)
    y = cv.conv2d_fwd(x, w, b32, (st, st), (pd, pd), stats=stats)
    yr = F.conv2d(x.float(), w.float(), b32, stride=st, padding=pd)
    assert _rel(y, yr) < 1e-2
    st2 = stats.view(bnops.stat_slots(), 2, K).sum(0)
    assert _rel(st2[0], y.float().sum(dim=(0, 2, 3))) < 1e-3
    assert _rel(st2[1], (y.float() ** 2).sum(dim=(0, 2, 3))) < 1e-3
    y2 = cv.conv2d_fwd(x, w, b32, (st, st), (pd, pd), relu=True)
    assert _rel(y2, torch.relu(yr)) < 1e-2
    # data gradient (+ residual addend, + consumer-BN backward reduction with the ReLU mask from x*scale+shift)
    gy = torch.randn_like(yr).to(BF, memory_format=CL)
    add = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
    bx = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
    mean = torch.randn(C, device=dev) * 0.1
    aff = torch.cat([torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.2])
    red = bnops.new_stats(C, dev)
    bn = {"x": bx, "z": None, "mean": mean, "aff": aff, "red": red}
    dx = cv.conv2d_dgrad(gy, cv.transpose_w(w), x.shape, (st, st), (pd, pd), addend=add, bn=bn)
    dxr = torch.nn.grad.conv2d_input(x.shape, w.float(), gy.float(), stride=st, padding=pd) + add.float()
    assert _rel(dx, dxr) < 1e-2
    if bn.get("done"):
        d = dx.float()
        xf = bx.float()
        mask = (xf * aff[:C].view(1, C, 1, 1) + aff[C:].view(1, C, 1, 1)) > 0
        dm = d * mask
        r2 = red.view(bnops.stat_slots(), 2, C).sum(0)
        assert _rel(r2[0], dm.sum(dim=(0, 2, 3))) < 1e-3
        assert _rel(r2[1], (dm * (xf - mean.view(1, C, 1, 1))).sum(dim=(0, 2, 3))) < 1e-3


G4_CASES = [
    # N, C, H, K, R, stride, pad -> 128 x BN 4-wave multi-stage kernel (Cs % 32 == 0, aligned output)
    (16, 64, 56, 256, 1, 1, 0),      # 1x1, 2 K-steps (fewer steps than stages)
    (8, 64, 56, 64, 3, 1, 1),        # 3x3, BN = 64 tile, padding taps
    (8, 256, 28, 256, 3, 2, 1),      # stride 2: dgrad phases
    (6, 128, 28, 320, 1, 1, 0),      # Ncol tail, M tail
    (4, 96, 14, 128, 3, 1, 1),       # Cs = 96: 32-channel steps across tap edges
    (4, 48, 14, 128, 3, 1, 1),       # Cs % 32 != 0: per-lane taps (slow-K), K tail
    (2, 80, 9, 200, 1, 1, 0),        # slow-K 1x1, Ncol tail
    (3, 40, 11, 64, 3, 2, 1),        # slow-K, BN = 64 tile, stride 2
    (8, 64, 28, 64, 1, 1, 0),        # Kdim 64, Ncol 64: the two-stage short-K variant (stages 2) in both passes
    (5, 64, 13, 40, 1, 1, 0),        # short-K, Ncol tail, M tail
]


@pytest.mark.parametrize("stages", [4, 3, 7, 2])
@pytest.mark.parametrize("case", G4_CASES)
def test_conv_g4_kernel_fwd_dgrad(case, stages):
    """128 x BN 4-wave kernel with 3 / 4 counted-vmcnt LDS-DMA stages (BIGDL_CONV_G4; 7 = the 256 x 128 tile for
    Ncol > 64; 2 = BIGDL_CONV_G4=3 with the two-stage short-K variant, BIGDL_CONV_SHORTK=1) vs fp32 torch: forward with
    bias + BN statistics, forward + ReLU, data gradient with a residual addend."""
    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import conv as cv
    from bigdl_amd.ops import native

    C_ = native.get()
    old = C_.get_conv_g4()
    C_.set_conv_g4(3 if stages == 2 else stages)
    C_.set_conv_shortk(1 if stages == 2 else 0)
    try:
        N, C, H, K, R, st, pd = case
        torch.manual_seed(7)
        dev = _dev()
        x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
        w = (torch.randn(K, C, R, R, device=dev) * (1.0 / (C * R * R) ** 0.5)).to(BF, memory_format=CL)
        b32 = torch.randn(K, device=dev)
        stats = bnops.new_stats(K, dev)
        y = cv.conv2d_fwd(x, w, b32, (st, st), (pd, pd), stats=stats)
        yr = F.conv2d(x.float(), w.float(), b32, stride=st, padding=pd)
        assert _rel(y, yr) < 1e-2
        st2 = stats.view(bnops.stat_slots(), 2, K).sum(0)
        assert _rel(st2[0], y.float().sum(dim=(0, 2, 3))) < 1e-3
        assert _rel(st2[1], (y.float() ** 2).sum(dim=(0, 2, 3))) < 1e-3
        y2 = cv.conv2d_fwd(x, w, b32, (st, st), (pd, pd), relu=True)
        assert _rel(y2, torch.relu(yr)) < 1e-2
        gy = torch.randn_like(yr).to(BF, memory_format=CL)
        add = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
        dx = cv.conv2d_dgrad(gy, cv.transpose_w(w), x.shape, (st, st), (pd, pd), addend=add)
        dxr = torch.nn.grad.conv2d_input(x.shape, w.float(), gy.float(), stride=st, padding=pd) + add.float()
        assert _rel(dx, dxr) < 1e-2
        torch.cuda.synchronize()
    finally:
        C_.set_conv_g4(old)
        C_.set_conv_shortk(0)


WGRAD_G3_CASES = WGRAD_CASES + [
    (8, 256, 28, 512, 1, 1, 0),      # many tiles, few splits
    (4, 512, 7, 512, 3, 1, 1),       # 3x3 over a small grid: short splits (stage count below the pipeline depth)
    (6, 128, 28, 136, 3, 2, 1),      # stride 2, Ncol tail
]


@pytest.mark.parametrize("case", WGRAD_G3_CASES)
def test_conv_wgrad_g3_kernel(case):
    """3-stage counted-vmcnt weight-gradient kernel (BIGDL_WGRAD_G3) vs fp32 torch, weight and bias gradients."""
    from bigdl_amd.ops import conv as cv
    from bigdl_amd.ops import native

    C_ = native.get()
    old = C_.get_wgrad_g3()
    C_.set_wgrad_g3(1)
    try:
        N, C, H, K, R, st, pd = case
        torch.manual_seed(4)
        dev = _dev()
        x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
        w = (torch.randn(K, C, R, R, device=dev) * (1.0 / (C * R * R) ** 0.5)).to(BF, memory_format=CL)
        yr = F.conv2d(x.float(), w.float(), None, stride=st, padding=pd)
        gy = torch.randn_like(yr).to(BF, memory_format=CL)
        dw = torch.zeros(K, C, R, R, device=dev).contiguous(memory_format=CL)
        db = torch.zeros(K, device=dev)
        cv.conv2d_wgrad(gy, x, dw, db, (st, st), (pd, pd))
        dwr = torch.nn.grad.conv2d_weight(x.float(), w.shape, gy.float(), stride=st, padding=pd)
        assert _rel(dw, dwr) < 1e-2
        assert _rel(db, gy.float().sum(dim=(0, 2, 3))) < 1e-2
        torch.cuda.synchronize()
    finally:
        C_.set_wgrad_g3(old)


@pytest.mark.parametrize("K,RS,C", [(1000, 1, 1032), (2048, 9, 264), (32768, 1, 1024), (1032, 1, 10000)])
def test_transpose_krsc_v8_matches_permute(K, RS, C):
    """16-byte 64x64-tile transpose (K % 8 == 0, C % 8 == 0, >= 1M elements): [K][RS][C] -> [C][RS][K], tails on
    both tile edges."""
    from bigdl_amd.ops import native

    w = torch.randn(K, RS, C, device=_dev()).to(BF)
    out = torch.empty(C, RS, K, device=_dev(), dtype=BF)
    native.get().transpose_krsc(w, out, K, RS, C)
    torch.cuda.synchronize()
    assert torch.equal(out, w.permute(2, 1, 0).contiguous())


P8_CASES = [
    # N, C, H, K, R, stride, pad -> 256 x 256 phase-interleaved 8-wave kernel (Cs % 64 == 0)
    (16, 256, 56, 256, 1, 1, 0),     # 196 tiles x 4 K-tiles: one pass
    (16, 256, 14, 256, 3, 1, 1),     # 13 tiles x 36 K-tiles: split-K + split-K epilogue, padding taps
    (4, 512, 7, 2048, 1, 1, 0),      # 8 tiles: split-K 2
    (8, 128, 28, 320, 3, 1, 1),      # Ncol tail (320 % 256 != 0)
    (16, 256, 28, 256, 3, 2, 1),     # stride 2: dgrad phases write a strided output placement
    (66, 256, 28, 256, 1, 1, 0),     # >= 192 tiles, M tail
    (3, 64, 10, 512, 3, 1, 1),       # tiny M (one tile), Cs = 64
    (8, 200, 14, 256, 1, 1, 0),      # 1x1 with Cs % 64 != 0: one-tap K-tail mode (forward)
    (4, 256, 9, 520, 1, 1, 0),       # K-tail on the data gradient (its Cs = 520)
]


@pytest.mark.parametrize("case", P8_CASES)
def test_conv_p8_kernel_fwd_dgrad(case):
    """256 x 256 phase-interleaved LDS-DMA kernel (BIGDL_CONV_P8=2 forces it wherever Cs % 64 == 0) and its split-K
    path vs fp32 torch: forward + bias + BN statistics, forward + ReLU, data gradient + residual addend + the consumer
    BN's fused backward reduction."""
    from bigdl_amd.ops import native

    C_ = native.get()
    C_.set_conv_p8(2)
    try:
        test_conv_w8_kernel_fwd_dgrad_bnred.__wrapped__(case) if hasattr(test_conv_w8_kernel_fwd_dgrad_bnred, "__wrapped__") \
            else test_conv_w8_kernel_fwd_dgrad_bnred(case)
        torch.cuda.synchronize()
    finally:
        C_.set_conv_p8(1)


WGRAD_P8_CASES = [
    # N, C, H, K, R, stride, pad -> 256 x 256 phase-interleaved weight-gradient kernel (no bias, Ncol, Kdim >= 256)
    (16, 64, 56, 256, 1, 1, 0),      # Kdim 64 < 256: stays on the older kernels (dispatch check)
    (16, 256, 56, 256, 1, 1, 0),     # 1 tile, deep pixel split
    (8, 128, 28, 256, 3, 1, 1),      # Kdim 1152 (4.5 tiles: kk tail), padding taps
    (8, 256, 28, 512, 3, 2, 1),      # stride 2, M tail
    (4, 512, 7, 512, 3, 1, 1),       # few pixels: one split, dw += directly
    (6, 264, 14, 320, 1, 1, 0),      # Ncol and Kdim tails (320, 264)
]


@pytest.mark.parametrize("case", WGRAD_P8_CASES)
@pytest.mark.parametrize("offset", [0, 1])
def test_conv_wgrad_p8_kernel(case, offset):
    """Phase-interleaved 256 x 256 weight-gradient kernel vs fp32 torch, accumulating into an existing gradient;
    offset 0 also checks the fused bias gradient, offset 1 places dW at a 4-byte (not 16-byte) aligned view of a
    flat buffer with no bias."""
    from bigdl_amd.ops import native

    N, C, H, K, R, st, pd = case
    torch.manual_seed(5)
    dev = _dev()
    x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
    OH = (H + 2 * pd - R) // st + 1
    gy = torch.randn(N, K, OH, OH, device=dev).to(BF, memory_format=CL)
    n = K * C * R * R
    flat = torch.randn(n + offset, device=dev)
    base = flat[offset:].clone()
    pre = flat[:offset].clone()
    dw = flat[offset:]                       # (K, R, S, C) = channels_last (K, C, R, S) storage
    geo = [N, H, H, C, OH, OH, R, R, st, st, pd, pd, 1, 1, N * OH * OH, K, R * R * C, K]
    db = torch.randn(K, device=dev) if offset == 0 else None
    db0 = db.clone() if db is not None else None
    native.get().set_wgrad_p8(2)             # every layer with Ncol, Kdim >= 256 (default 1 picks by measured wins)
    try:
        native.get().conv_wgrad(gy, x, dw, db, geo)
        torch.cuda.synchronize()
    finally:
        native.get().set_wgrad_p8(1)
    if db is not None:
        assert _rel(db - db0, gy.float().sum(dim=(0, 2, 3))) < 1e-2
    dwr = torch.nn.grad.conv2d_weight(x.float(), (K, C, R, R), gy.float(), stride=st, padding=pd)
    got = (dw - base).view(K, R, R, C).permute(0, 3, 1, 2)
    assert _rel(got, dwr) < 1e-2
    assert torch.equal(flat[:offset], pre)


S1_CASES = [
    # N, C, H, K (1x1, stride 1): the streaming 1x1 kernel takes fwd when C in {64, 128} and dgrad when K in {64, 128}
    (16, 64, 56, 256),     # fwd K 64 -> 256 (ResNet layer 3 shape at batch 16), 4 channel groups
    (8, 256, 28, 64),      # dgrad 64 -> 256 with addend + consumer-BN reduction (fwd on the other kernels)
    (6, 128, 28, 512),     # fwd K 128 -> 512, two channel blocks of 256
    (5, 64, 13, 64),       # one channel group, M tail (845 rows)
    (3, 128, 11, 192),     # Ncol 192: three one-group channel blocks, M tail
    (4, 192, 9, 128),      # dgrad 128 -> 192
    (7, 128, 10, 128),     # two channel groups both ways
    (8, 256, 14, 1024),    # fwd K 256 -> 1024 (layer 13 shape: one workgroup per CU, 128 weight VGPRs per wave)
    (6, 1024, 14, 256),    # dgrad 256 -> 1024 with addend + consumer-BN reduction (layer 15 data gradient)
    (5, 256, 13, 64),      # fwd K 256 -> 64 with an M tail; dgrad 64 -> 256
]


@pytest.mark.parametrize("zmask", [False, True])
@pytest.mark.parametrize("case", S1_CASES)
def test_conv_s1_stream_kernel(case, zmask):
    """Streaming 1x1 kernel (conv_nt_s1_kernel: persistent, weights in VGPRs, register-prefetched operand tiles,
    statistics accumulated across tiles) vs fp32 torch: forward + BN statistics, forward + bias + ReLU, data gradient
    + residual addend + consumer-BN backward reduction under the affine (or z) ReLU mask; and bit-equal outputs with
    the kernel switched off where the per-tile kernels round the same fp32 sums (forward without bias)."""
    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import conv as cv
    from bigdl_amd.ops import native

    C_ = native.get()
    N, C, H, K = case
    torch.manual_seed(11)
    dev = _dev()
    x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
    w = (torch.randn(K, C, 1, 1, device=dev) * (1.0 / C ** 0.5)).to(BF, memory_format=CL)
    b32 = torch.randn(K, device=dev)
    yr0 = F.conv2d(x.float(), w.float())
    res = {}
    for s1 in (2, 0):
        C_.set_conv_s1(s1)
        try:
            stats = bnops.new_stats(K, dev)
            y = cv.conv2d_fwd(x, w, None, (1, 1), (0, 0), stats=stats)
            y2 = cv.conv2d_fwd(x, w, b32, (1, 1), (0, 0), relu=True)
            gy = (torch.randn(N, K, H, H, device=dev, generator=torch.Generator(dev).manual_seed(3))).to(
                BF, memory_format=CL)
            add = torch.randn(N, C, H, H, device=dev, generator=torch.Generator(dev).manual_seed(4)).to(
                BF, memory_format=CL)
            bx = torch.randn(N, C, H, H, device=dev, generator=torch.Generator(dev).manual_seed(5)).to(
                BF, memory_format=CL)
            bz = torch.relu(torch.randn(N, C, H, H, device=dev, generator=torch.Generator(dev).manual_seed(6))).to(
                BF, memory_format=CL)
            mean = torch.linspace(-0.1, 0.1, C, device=dev)
            aff = torch.cat([torch.linspace(0.5, 1.5, C, device=dev), torch.linspace(-0.2, 0.2, C, device=dev)])
            red = bnops.new_stats(C, dev)
            bn = {"x": bx, "z": bz if zmask else None, "mean": mean, "aff": aff, "red": red}
            dx = cv.conv2d_dgrad(gy, cv.transpose_w(w), x.shape, (1, 1), (0, 0), addend=add, bn=bn)
            torch.cuda.synchronize()
            res[s1] = (y, stats, y2, dx, red, bool(bn.get("done")))
        finally:
            C_.set_conv_s1(2)
    y, stats, y2, dx, red, done = res[2]
    assert _rel(y, yr0) < 1e-2
    st2 = stats.view(bnops.stat_slots(), 2, K).sum(0)
    assert _rel(st2[0], y.float().sum(dim=(0, 2, 3))) < 1e-4
    assert _rel(st2[1], (y.float() ** 2).sum(dim=(0, 2, 3))) < 1e-4
    assert _rel(y2, torch.relu(yr0 + b32.view(1, K, 1, 1))) < 1e-2
    assert torch.equal(y, res[0][0])                   # same fp32 sums, same rounding
    gy = res[2][3]  # placeholder to keep names short below
    gyr = (torch.randn(N, K, H, H, device=dev, generator=torch.Generator(dev).manual_seed(3))).to(BF).float()
    addr = torch.randn(N, C, H, H, device=dev, generator=torch.Generator(dev).manual_seed(4)).to(BF).float()
    dxr = torch.nn.grad.conv2d_input(x.shape, w.float(), gyr) + addr
    assert _rel(dx, dxr) < 1e-2
    assert _rel(dx, res[0][3]) < 1e-2
    if done:
        d = dx.float()
        xf = torch.randn(N, C, H, H, device=dev, generator=torch.Generator(dev).manual_seed(5)).to(BF).float()
        if zmask:
            zf = torch.relu(torch.randn(N, C, H, H, device=dev, generator=torch.Generator(dev).manual_seed(6))).to(BF).float()
            mask = zf > 0
        else:
            mask = (xf * torch.linspace(0.5, 1.5, C, device=dev).view(1, C, 1, 1)
                    + torch.linspace(-0.2, 0.2, C, device=dev).view(1, C, 1, 1)) > 0
        dm = d * mask
        r2 = red.view(bnops.stat_slots(), 2, C).sum(0)
        assert _rel(r2[0], dm.sum(dim=(0, 2, 3))) < 1e-3
        assert _rel(r2[1], (dm * (xf - torch.linspace(-0.1, 0.1, C, device=dev).view(1, C, 1, 1))).sum(dim=(0, 2, 3))) < 1e-3


SK_CASES = [
    # N, C, H, K, R, stride, pad -> stream-K P8 (BIGDL_CONV_SK=2: wherever the 256 x 256 kernel applies)
    (16, 256, 14, 256, 3, 1, 1),     # 13 tiles x 36 K-tiles over the CUs: multi-segment tiles, padding taps
    (4, 512, 7, 512, 3, 1, 1),       # 2 x 2 tiles x 72 K-tiles, M tail
    (16, 256, 28, 256, 3, 2, 1),     # stride 2: dgrad phases with 1-4 taps
    (8, 1024, 14, 512, 1, 1, 0),     # 1x1, Ncol 512
    (3, 64, 10, 512, 3, 1, 1),       # tiny M, Cs = 64
]


@pytest.mark.parametrize("case", SK_CASES)
def test_conv_p8_stream_k(case):
    """Stream-K 256 x 256 kernel (persistent, segments of the tiles x K-tiles space, last-arriver fixup over
    write-through partial slots) vs fp32 torch: forward + bias + BN statistics, + ReLU, data gradient + addend + the
    consumer BN reduction; and run-to-run bit equality (the fixup sums the slots in segment order)."""
    from bigdl_amd.ops import conv as cv
    from bigdl_amd.ops import native

    C_ = native.get()
    C_.set_conv_sk(2)
    try:
        test_conv_w8_kernel_fwd_dgrad_bnred(case)
        N, C, H, K, R, st, pd = case
        torch.manual_seed(9)
        x = torch.randn(N, C, H, H, device=_dev()).to(BF, memory_format=CL)
        w = (torch.randn(K, C, R, R, device=_dev()) * (1.0 / (C * R * R) ** 0.5)).to(BF, memory_format=CL)
        y1 = cv.conv2d_fwd(x, w, None, (st, st), (pd, pd))
        y2 = cv.conv2d_fwd(x, w, None, (st, st), (pd, pd))
        torch.cuda.synchronize()
        assert torch.equal(y1, y2)
        C_.set_conv_sk(0)
        y0 = cv.conv2d_fwd(x, w, None, (st, st), (pd, pd))
        assert _rel(y1, y0) < 1e-2
    finally:
        C_.set_conv_sk(1)


# 3x3 / stride 1 / pad 1 weight gradients on the halo-tile kernel (csrc/wgrad_halo.hip): every supported width, both
# output-channel blocks (64 / 128), a single split (direct add into dW) and many splits (workspace + reduce), a
# non-zero starting dW (the kernel accumulates), and the same shapes with the kernel switched off as a control.
HALO_CASES = [
    (4, 64, 56, 64), (2, 64, 56, 128), (8, 128, 28, 128), (3, 64, 28, 64), (16, 256, 14, 256), (5, 64, 14, 192),
    (32, 512, 7, 512), (1, 64, 7, 64), (256, 64, 7, 128),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", HALO_CASES)
def test_conv_wgrad_halo_matches_fp32(case):
    from bigdl_amd.ops import conv as cv
    from bigdl_amd.ops import native

    N, C, H, K = case
    torch.manual_seed(5)
    dev = _dev()
    x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
    gy = torch.randn(N, K, H, H, device=dev).to(BF, memory_format=CL)
    dw0 = torch.randn(K, C, 3, 3, device=dev).contiguous(memory_format=CL)
    db0 = torch.randn(K, device=dev)
    ref = dw0 + torch.nn.grad.conv2d_weight(x.float(), (K, C, 3, 3), gy.float(), stride=1, padding=1)
    refb = db0 + gy.float().sum(dim=(0, 2, 3))
    outs = []
    try:
        for on in (1, 0):
            native.get().set_wgrad_halo(on)
            dw, db = dw0.clone(), db0.clone()
            cv.conv2d_wgrad(gy, x, dw, db, (1, 1), (1, 1))      # with the bias gradient (the ResNet convs have one)
            dw2 = dw0.clone()
            cv.conv2d_wgrad(gy, x, dw2, None, (1, 1), (1, 1))
            torch.cuda.synchronize()
            outs.append((dw, db, dw2))
    finally:
        native.get().set_wgrad_halo(1)
    for dw, db, dw2 in outs:
        assert torch.isfinite(dw).all()
        assert _rel(dw, ref) < 5e-3, _rel(dw, ref)
        assert _rel(dw2, ref) < 5e-3, _rel(dw2, ref)
        assert _rel(db, refb) < 1e-3, _rel(db, refb)
    assert _rel(outs[0][0], outs[1][0]) < 5e-3


HALO_FWD_CASES = [
    # N, C, H, K (3x3, stride 1, pad 1): conv_halo_kernel takes fwd / dgrad when H in {56, 28, 14, 7}, C % 32 == 0 and
    # the output channels are a multiple of its channel tile (64 at H 56, 128 below)
    (4, 64, 56, 64),       # ResNet-50 layer 2 shape (RB 4 row segments, top / bottom halo variants)
    (3, 128, 28, 128),     # layer 10 shape (RB 7)
    (2, 128, 28, 256),     # fwd: two channel tiles; dgrad: 256 -> 128 (8 chunks)
    (5, 256, 14, 256),     # layer 16 shape (one whole image per tile)
    (4, 512, 7, 512),      # layer 22 shape (3 stacked images per tile, last tile past the batch)
    (7, 64, 7, 128),       # stacked images, fwd two chunks; dgrad falls back (64 output channels)
    (3, 96, 14, 128),      # odd chunk count (3 x 32 channels)
]


def _sign_mask(z):
    """[P][C/8] uint8 sign bytes of an NHWC bf16 tensor (bit e of byte (p, g): z[p][8g + e] > 0)."""
    N, C, H, W = z.shape
    b = (z.permute(0, 2, 3, 1).reshape(-1, C // 8, 8) > 0).to(torch.int32)
    w = (1 << torch.arange(8, device=z.device, dtype=torch.int32))
    return (b * w).sum(-1).to(torch.uint8).reshape(-1).contiguous()


@pytest.mark.parametrize("zmask", [False, True, "zm"])
@pytest.mark.parametrize("case", HALO_FWD_CASES)
def test_conv_halo_kernel(case, zmask):
    """3x3 / stride-1 / pad-1 halo-tile kernel (conv_halo.hip: one staged input halo per 32-channel chunk, 9 shifted
    LDS windows, weight ring) vs fp32 torch: forward + BN statistics, forward + bias + ReLU, data gradient + residual
    addend + consumer-BN backward reduction under the affine (or z) ReLU mask; and against the im2col kernels
    (BIGDL_CONV_HALO off)."""
    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import conv as cv
    from bigdl_amd.ops import native

    C_ = native.get()
    N, C, H, K = case
    torch.manual_seed(13)
    dev = _dev()
    x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
    w = (torch.randn(K, C, 3, 3, device=dev) * (1.0 / (9 * C) ** 0.5)).to(BF, memory_format=CL)
    b32 = torch.randn(K, device=dev)
    yr0 = F.conv2d(x.float(), w.float(), padding=1)
    g = lambda s: torch.Generator(dev).manual_seed(s)  # noqa: E731
    gy = torch.randn(N, K, H, H, device=dev, generator=g(3)).to(BF, memory_format=CL)
    add = torch.randn(N, C, H, H, device=dev, generator=g(4)).to(BF, memory_format=CL)
    bx = torch.randn(N, C, H, H, device=dev, generator=g(5)).to(BF, memory_format=CL)
    bz = torch.relu(torch.randn(N, C, H, H, device=dev, generator=g(6))).to(BF, memory_format=CL)
    mean = torch.linspace(-0.1, 0.1, C, device=dev)
    aff = torch.cat([torch.linspace(0.5, 1.5, C, device=dev), torch.linspace(-0.2, 0.2, C, device=dev)])
    res = {}
    for halo in (1, 0):
        C_.set_conv_halo(halo)
        try:
            stats = bnops.new_stats(K, dev)
            y = cv.conv2d_fwd(x, w, None, (1, 1), (1, 1), stats=stats)
            y2 = cv.conv2d_fwd(x, w, b32, (1, 1), (1, 1), relu=True)
            red = bnops.new_stats(C, dev)
            bn = {"x": bx, "z": bz if zmask is True else None, "zm": _sign_mask(bz) if zmask == "zm" else None,
                  "mean": mean, "aff": aff, "red": red}
            dx = cv.conv2d_dgrad(gy, cv.transpose_w(w), x.shape, (1, 1), (1, 1), addend=add, bn=bn)
            # without the addend: the lean epilogue's consumer-BN reduction (the ResNet 3x3 data gradient)
            red2 = bnops.new_stats(C, dev)
            bn2 = dict(bn, red=red2)
            dx2 = cv.conv2d_dgrad(gy, cv.transpose_w(w), x.shape, (1, 1), (1, 1), bn=bn2)
            torch.cuda.synchronize()
            res[halo] = (y, stats, y2, dx, red, bool(bn.get("done")), dx2, red2)
        finally:
            C_.set_conv_halo(1)
    y, stats, y2, dx, red, done, dx2, red2 = res[1]
    assert torch.isfinite(y.float()).all() and torch.isfinite(dx.float()).all()
    assert _rel(y, yr0) < 1e-2
    st2 = stats.view(bnops.stat_slots(), 2, K).sum(0)
    assert _rel(st2[0], y.float().sum(dim=(0, 2, 3))) < 1e-4
    assert _rel(st2[1], (y.float() ** 2).sum(dim=(0, 2, 3))) < 1e-4
    assert _rel(y2, torch.relu(yr0 + b32.view(1, K, 1, 1))) < 1e-2
    assert _rel(y, res[0][0]) < 1e-2
    dxr = torch.nn.grad.conv2d_input(x.shape, w.float(), gy.float(), padding=1) + add.float()
    assert _rel(dx, dxr) < 1e-2
    assert _rel(dx, res[0][3]) < 1e-2
    assert done
    d = dx.float()
    mask = (bz.float() > 0) if zmask else (bx.float() * aff[:C].view(1, C, 1, 1) + aff[C:].view(1, C, 1, 1)) > 0
    dm = d * mask
    r2 = red.view(bnops.stat_slots(), 2, C).sum(0)
    assert _rel(r2[0], dm.sum(dim=(0, 2, 3))) < 1e-3
    assert _rel(r2[1], (dm * (bx.float() - mean.view(1, C, 1, 1))).sum(dim=(0, 2, 3))) < 1e-3
    assert _rel(dx2, dxr - add.float()) < 1e-2
    dm2 = dx2.float() * mask
    r3 = red2.view(bnops.stat_slots(), 2, C).sum(0)
    assert _rel(r3[0], dm2.sum(dim=(0, 2, 3))) < 1e-3
    assert _rel(r3[1], (dm2 * (bx.float() - mean.view(1, C, 1, 1))).sum(dim=(0, 2, 3))) < 1e-3
