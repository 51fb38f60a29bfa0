"""Native TensorMath backend (csrc/tensor_math.hip via ops/tensor_math.py): the 1-based Tensor API on fp32 GPU tensors
vs the same calls on CPU tensors (torch). torch's element / BLAS / reduction entry points are patched to raise while
the GPU calls run, so a pass proves the native kernels computed the results."""
import contextlib

import pytest
import torch

from bigdl_amd.tensor import Tensor

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def no_aten(monkeypatch):
    def boom(name):
        def f(*a, **k):
            raise AssertionError(f"aten {name} called on the native TensorMath path")
        return f
    with monkeypatch.context() as mp:
        for name in ("addmm", "addmv", "addr", "baddbmm", "bmm", "matmul", "exp", "log", "sqrt", "tanh", "abs", "clamp",
                     "maximum", "minimum"):
            mp.setattr(torch, name, boom(name))
        for name in ("add_", "sub_", "mul_", "div_", "addcmul_", "addcdiv_", "clamp_", "fill_", "zero_", "reciprocal_",
                     "pow_", "copy_", "sum", "prod", "max", "min", "mean", "__matmul__"):
            mp.setattr(torch.Tensor, name, boom(name))
        yield


def _pair(*shape, seed=0, positive=False):
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(*shape, generator=g)
    if positive:
        t = t.abs() + 0.1
    return Tensor(t.clone()), Tensor(t.clone().cuda())


def _close(gpu, cpu, tol=1e-5):
    g = gpu._t.cpu() if isinstance(gpu, Tensor) else torch.as_tensor(gpu)
    c = cpu._t if isinstance(cpu, Tensor) else torch.as_tensor(cpu)
    assert g.shape == c.shape, (g.shape, c.shape)
    assert torch.allclose(g.float(), c.float(), rtol=tol, atol=tol), float((g.float() - c.float()).abs().max())


def test_element_ops_native(monkeypatch):
    c1, g1 = _pair(5, 7, seed=1)
    c2, g2 = _pair(5, 7, seed=2, positive=True)
    c3, g3 = _pair(5, 7, seed=3, positive=True)
    steps = [
        lambda t, o, p: t.fill(2.5),
        lambda t, o, p: t.add(3.0),
        lambda t, o, p: t.add(o),
        lambda t, o, p: t.add(0.5, o),
        lambda t, o, p: t.add(o, p),
        lambda t, o, p: t.add(o, -2.0, p),
        lambda t, o, p: t.sub(o),
        lambda t, o, p: t.mul(1.5),
        lambda t, o, p: t.div(3.0),
        lambda t, o, p: t.cmul(o),
        lambda t, o, p: t.cdiv(o, p),
        lambda t, o, p: t.cmax(0.2),
        lambda t, o, p: t.cmin(o),
        lambda t, o, p: t.addcmul(0.3, o, p),
        lambda t, o, p: t.addcdiv(0.3, o, p),
        lambda t, o, p: t.clamp(-0.5, 0.5),
        lambda t, o, p: t.abs(),
        lambda t, o, p: t.exp(o),
        lambda t, o, p: t.log(p),
        lambda t, o, p: t.sqrt(p),
        lambda t, o, p: t.tanh(o),
        lambda t, o, p: t.negative(o),
        lambda t, o, p: t.inv(),
        lambda t, o, p: t.pow(2.0),
        lambda t, o, p: t.copy(o),
    ]
    for i, step in enumerate(steps):
        step(c1, c2, c3)
        with no_aten(monkeypatch):
            step(g1, g2, g3)
        torch.cuda.synchronize()
        _close(g1, c1, 1e-4)


def test_strided_and_broadcast_views_native(monkeypatch):
    ca, ga = _pair(6, 8, seed=4)
    cb, gb = _pair(8, 6, seed=5)
    # transposed operand (non-contiguous) into a column slice of the output
    c_out, g_out = _pair(6, 10, seed=6)
    cv = Tensor(c_out._t[:, 1:9])
    gv = Tensor(g_out._t[:, 1:9])
    cv.add(ca, Tensor(cb._t.t()))
    with no_aten(monkeypatch):
        gv.add(ga, Tensor(gb._t.t()))
    _close(g_out, c_out)
    # outer product (addr): broadcast strides
    cx, gx = _pair(6, seed=7)
    cy, gy = _pair(10, seed=8)
    c_out.addr(0.5, c_out, 2.0, cx, cy)
    with no_aten(monkeypatch):
        g_out.addr(0.5, g_out, 2.0, gx, gy)
    _close(g_out, c_out, 1e-4)


@pytest.mark.parametrize("m,k,n", [(17, 33, 9), (64, 64, 64), (130, 70, 200), (5, 1, 3)])
def test_blas_native(monkeypatch, m, k, n):
    ca, ga = _pair(m, k, seed=9)
    cb, gb = _pair(k, n, seed=10)
    cm, gm = _pair(m, n, seed=11)
    cv, gv = _pair(k, seed=12)
    cw, gw = _pair(m, seed=13)
    co, go = Tensor(m, n), Tensor(torch.zeros(m, n, device="cuda"))
    co.addmm(0.5, cm, 2.0, ca, cb)
    cmv = Tensor(m)
    cmv.addmv(0.25, cw, 1.5, ca, cv)
    cmm = Tensor(m, n)
    cmm.mm(ca, Tensor(cb._t.t().contiguous().t()))
    with no_aten(monkeypatch):
        go.addmm(0.5, gm, 2.0, ga, gb)
        gmv = Tensor(torch.zeros(m, device="cuda"))
        gmv.addmv(0.25, gw, 1.5, ga, gv)
        gmm = Tensor(torch.zeros(m, n, device="cuda"))
        gmm.mm(ga, Tensor(gb._t.t().contiguous().t()))      # column-major B through strides
    torch.cuda.synchronize()
    tol = 2e-4 * max(1.0, k ** 0.5)
    _close(go, co, tol)
    _close(gmv, cmv, tol)
    _close(gmm, cmm, tol)
    # batched
    cA, gA = _pair(3, m, k, seed=14)
    cB, gB = _pair(3, k, n, seed=15)
    cC, gC = Tensor(3, m, n), Tensor(torch.zeros(3, m, n, device="cuda"))
    cC.bmm(cA, cB)
    with no_aten(monkeypatch):
        gC.bmm(gA, gB)
    _close(gC, cC, tol)
    # dot
    assert abs(ga.dot(ga) - ca.dot(ca)) <= 1e-4 * abs(ca.dot(ca))


@pytest.mark.parametrize("shape,dim", [((7, 13), 2), ((7, 13), 1), ((4, 5, 6), 2), ((3, 20000), 2), ((50000,), None)])
def test_reductions_native(monkeypatch, shape, dim):
    c, g = _pair(*shape, seed=16)
    if dim is None:
        with no_aten(monkeypatch):
            s, mx, mn, sq = g.sum(), g.max(), g.min(), g.sumSquare()
        assert abs(s - c.sum()) < 1e-3 * max(1.0, abs(c.sum())) + 5e-2
        assert mx == c.max() and mn == c.min()
        assert abs(sq - c.sumSquare()) < 1e-4 * c.sumSquare()
        return
    with no_aten(monkeypatch):
        gs = g.sum(dim)
        gm = g.mean(dim)
        gv, gi = g.max(dim)
        nv, ni = g.min(dim)
    cs, cm = c.sum(dim), c.mean(dim)
    cv, ci = c.max(dim)
    cnv, cni = c.min(dim)
    _close(gs, cs, 1e-4)
    _close(gm, cm, 1e-5)
    _close(gv, cv, 0)
    _close(gi, ci, 0)
    _close(nv, cnv, 0)
    _close(ni, cni, 0)


def test_softmax_layer_native_matches_torch(monkeypatch):
    """nn.SoftMax / SoftMin on the GPU engine: exp(native log-softmax) forward, TensorMath backward."""
    from bigdl_amd import nn

    torch.manual_seed(0)
    x = torch.randn(6, 37)
    gy = torch.randn(6, 37)
    for layer, ref in ((nn.SoftMax(), torch.softmax(x, 1)), (nn.SoftMin(), torch.softmax(-x, 1))):
        m = layer.to("cuda") if hasattr(layer, "to") else layer
        with monkeypatch.context() as mp:
            mp.setattr(torch, "softmax", lambda *a, **k: (_ for _ in ()).throw(AssertionError("aten softmax")))
            y = m.forward(x.cuda())
            gx = m.backward(x.cuda(), gy.cuda())
        torch.cuda.synchronize()
        assert torch.allclose(y.cpu(), ref, atol=1e-6)
        xr = x.clone().requires_grad_(True)
        (torch.softmax(xr if isinstance(layer, nn.SoftMax) else -xr, 1) * gy).sum().backward()
        assert torch.allclose(gx.cpu(), xr.grad, atol=1e-5)


@contextlib.contextmanager
def no_aten_index(monkeypatch):
    """torch's index / sort / mask entry points raise: a pass proves csrc/index_ops.hip ran."""
    def boom(name):
        def f(*a, **k):
            raise AssertionError(f"aten {name} called on the native index path")
        return f
    with monkeypatch.context() as mp:
        for name in ("topk", "gather", "sort"):
            mp.setattr(torch, name, boom(name))
        for name in ("index_select", "index_add_", "scatter_", "masked_fill_", "masked_select", "topk", "gather",
                     "__setitem__"):
            mp.setattr(torch.Tensor, name, boom(name))
        yield


def test_index_sort_mask_ops_native(monkeypatch):
    """TensorMath gather (:199), scatter (:209), topk (:622), masked* (:700-719), index (:739), indexAdd (:751):
    fp32 GPU results vs the torch CPU path of the same Tensor calls (1-based T-typed indices)."""
    g = torch.Generator().manual_seed(7)
    x = torch.randn(6, 300, 5, generator=g)
    idx = torch.randint(1, 301, (40,), generator=g).float()
    gidx = torch.randint(1, 301, (6, 17, 5), generator=g).float()
    sidx = torch.stack([torch.randperm(300, generator=g)[:17] + 1 for _ in range(30)]).float().reshape(6, 5, 17) \
        .transpose(1, 2).contiguous()
    src = torch.randn(6, 17, 5, generator=g)
    mask = (torch.rand(6, 300, 5, generator=g) > 0.6).float()
    addsrc = torch.randn(6, 40, 5, generator=g)
    cpu = {"x": Tensor(x.clone())}
    gpu = {"x": Tensor(x.clone().cuda())}
    res = {}
    for name, T, dev in (("cpu", cpu, "cpu"), ("gpu", gpu, "cuda")):
        d = lambda t: Tensor(t.clone().to(dev))  # noqa: E731
        ctx = no_aten_index(monkeypatch) if dev == "cuda" else contextlib.nullcontext()
        with ctx:
            out = {}
            out["index"] = Tensor().index(2, d(idx), T["x"])
            out["gather"] = Tensor().gather(2, d(gidx), T["x"])
            sc = d(x)
            out["scatter"] = sc.scatter(2, d(sidx), d(src))
            ia = d(x)
            out["indexAdd"] = ia.indexAdd(2, d(idx), d(addsrc))
            for k, inc in ((1, True), (7, False), (300, True)):
                v, i = T["x"].topk(k, 2, inc)
                out[f"topk{k}{inc}_v"], out[f"topk{k}{inc}_i"] = v, i
            mf = d(x)
            out["maskedFill"] = mf.maskedFill(d(mask), -3.5)
            out["maskedSelect"] = T["x"].maskedSelect(d(mask), Tensor())
            mc = d(x)
            out["maskedCopy"] = mc.maskedCopy(d(mask), d(torch.arange(float(mask.numel()))))
            vmax, imax = T["x"].max(2)
            out["max_i"] = imax
        res[name] = out
    for k in res["cpu"]:
        _close(res["gpu"][k], res["cpu"][k], tol=1e-5)
        if k.endswith("_i"):
            assert res["gpu"][k]._t.dtype == res["cpu"][k]._t.dtype == torch.float32, k   # T-typed indices


def test_index_out_of_range_raises():
    """Out-of-range 1-based indices raise IndexError on the native path (the reference's 'index out of bound'
    require), for index / gather / indexAdd / scatter; a later valid op is unaffected (the error word is cleared)."""
    x = Tensor(torch.randn(4, 10).cuda())
    bad = Tensor(torch.tensor([1.0, 11.0]).cuda())
    with pytest.raises(IndexError):
        Tensor().index(2, bad, x)
    with pytest.raises(IndexError):
        Tensor().gather(2, Tensor(torch.full((4, 2), 0.0).cuda()), x)
    with pytest.raises(IndexError):
        Tensor(torch.zeros(4, 10).cuda()).indexAdd(2, bad, Tensor(torch.ones(4, 2).cuda()))
    ok = Tensor().index(2, Tensor(torch.tensor([1.0, 10.0]).cuda()), x)
    assert torch.equal(ok._t.cpu(), x._t.cpu()[:, [0, 9]])


def test_masked_copy_short_source_raises():
    x = Tensor(torch.zeros(10).cuda())
    mask = Tensor(torch.ones(10).cuda())
    with pytest.raises(RuntimeError):
        x.maskedCopy(mask, Tensor(torch.arange(5.0).cuda()))


@pytest.mark.parametrize("R", [37, 9000])
@pytest.mark.parametrize("inc", [True, False])
def test_topk_nan_order_matches_torch(R, inc):
    """NaN orders as torch.topk does in both directions (last for smallest-k, first for largest-k), on the native
    in-LDS sort (R <= 8192) and on the torch fallback (longer rows): same values and indices, NaN positions included."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(3, R, generator=g)
    x[0, 5] = float("nan")
    x[1, R - 1] = float("nan")
    x[1, 2] = float("inf")
    x[2, 0] = float("-inf")
    k = 8
    v, i = Tensor(x.clone().cuda()).topk(k, 2, inc)
    rv, ri = torch.topk(x, k, dim=1, largest=not inc, sorted=True)
    vv = v._t.cpu()
    assert torch.equal(torch.isnan(vv), torch.isnan(rv))
    fin = ~torch.isnan(rv)
    assert torch.equal(vv[fin], rv[fin])
    # NaN positions carry the NaN's own index; finite picks match torch's (no ties in random data)
    assert torch.equal((i._t.cpu() - 1).long()[fin], ri[fin])
