"""Recurrent layers on the GPU engine: MFMA Linear input projection (bf16) + fused HIP LSTM cell kernels vs
the fp32 CPU engine."""
import copy

import pytest
import time

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
    # GPU path: bf16 MFMA recurrent GEMM (h, U rounded to bf16), fp32 cell state
    assert _rel(out, ref) < 1e-2 and _rel(c, cr) < 1e-2


@pytest.mark.parametrize("B,T,H", [(37, 6, 64), (64, 4, 1024), (5, 3, 192),
                                   (72, 4, 1024), (150, 3, 512)])     # > 256 tiles: 2 batch tiles per workgroup
def test_fused_lstm_steps_match_fp32_reference(B, T, H):
    """csrc/lstm.hip forward/backward step kernels vs the fp32 torch LSTM recurrence (gate order i, g, f, o)."""
    from bigdl_amd.nn.recurrent import _LSTMSeq

    torch.manual_seed(0)
    xg = torch.randn(B, T, 4 * H) * 0.5
    h0, c0 = torch.randn(B, H) * 0.5, torch.randn(B, H) * 0.5
    U = (torch.randn(4 * H, H) / H ** 0.5).to(torch.bfloat16).float()

    def ref(xg, h0, c0, U):
        h, c, outs = h0, c0, []
        for t in range(T):
            g = xg[:, t] + h @ U.t()
            i, gg, f, o = (torch.sigmoid(g[:, :H]), torch.tanh(g[:, H:2 * H]), torch.sigmoid(g[:, 2 * H:3 * H]),
                           torch.sigmoid(g[:, 3 * H:]))
            c = f * c + i * gg
            h = o * torch.tanh(c)
            outs.append(h)
        return torch.stack(outs, 1), h, c

    leaves = [t.clone().double().requires_grad_(True) for t in (xg, h0, c0, U)]
    ro, rh, rc = ref(*leaves)
    go, gh, gc = torch.randn_like(ro), torch.randn_like(rh), torch.randn_like(rc)
    (ro * go).sum().backward(retain_graph=True)
    (rh * gh + rc * gc).sum().backward()
    dev = [t.cuda().requires_grad_(True) for t in (xg, h0, c0, U)]
    out, hT, cT = _LSTMSeq.apply(*dev)
    torch.autograd.backward([out, hT, cT], [go.float().cuda(), gh.float().cuda(), gc.float().cuda()])
    assert _rel(out, ro) < 1e-2 and _rel(hT, rh) < 1e-2 and _rel(cT, rc) < 1e-2
    for d, r in zip(dev, leaves):
        assert _rel(d.grad, r.grad) < 2e-2, (d.shape, _rel(d.grad, r.grad))


@pytest.mark.parametrize("B,T,H", [(37, 6, 64), (64, 5, 1024), (5, 3, 192)])
def test_fused_gru_steps_match_fp32_reference(B, T, H):
    """csrc/gru.hip forward/backward step kernels + native weight-gradient GEMMs vs the fp32 torch GRU recurrence
    (BigDL form: n = tanh(x_n + U_n (r * h)), h' = (1 - z) n + z h)."""
    from bigdl_amd.nn.recurrent import _GRUSeq

    torch.manual_seed(1)
    xg = torch.randn(B, T, 3 * H) * 0.5
    h0 = torch.randn(B, H) * 0.5
    Urz = (torch.randn(2 * H, H) / H ** 0.5).to(torch.bfloat16).float()
    Un = (torch.randn(H, H) / H ** 0.5).to(torch.bfloat16).float()

    def ref(xg, h0, Urz, Un):
        h, outs = h0, []
        for t in range(T):
            rz = torch.sigmoid(xg[:, t, :2 * H] + h @ Urz.t())
            r, z = rz[:, :H], rz[:, H:]
            n = torch.tanh(xg[:, t, 2 * H:] + (r * h) @ Un.t())
            h = (1 - z) * n + z * h
            outs.append(h)
        return torch.stack(outs, 1), h

    leaves = [t.clone().double().requires_grad_(True) for t in (xg, h0, Urz, Un)]
    ro, rh = ref(*leaves)
    go, gh = torch.randn_like(ro), torch.randn_like(rh)
    ((ro * go).sum() + (rh * gh).sum()).backward()
    dev = [t.cuda().requires_grad_(True) for t in (xg, h0, Urz, Un)]
    out, hT = _GRUSeq.apply(*dev)
    torch.autograd.backward([out, hT], [go.float().cuda(), gh.float().cuda()])
    assert _rel(out, ro) < 1e-2 and _rel(hT, rh) < 1e-2
    for d, r in zip(dev, leaves):
        assert _rel(d.grad, r.grad) < 2e-2, (d.shape, _rel(d.grad, r.grad))


@pytest.mark.parametrize("cellname", ["LSTM", "GRU"])
def test_bidirectional_two_layer_rnn_gpu_matches_cpu(cellname):
    """Multi-layer bi-directional stacks run the fused sequence kernels per layer and direction."""
    from bigdl_amd import nn
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(3)
    cell = getattr(nn, cellname)
    cpu = (nn.Sequential().add(nn.BiRecurrent(nn.JoinTable(3, 3)).add(cell(32, 64)))
           .add(nn.Recurrent().add(cell(128, 64))))
    gpu = copy.deepcopy(cpu).to("cuda")
    x = torch.randn(6, 9, 32).to(torch.bfloat16).float()
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


@pytest.mark.parametrize("B,T,H", [(128, 16, 1024), (100, 7, 512), (9, 5, 256), (64, 3, 1024), (256, 8, 1024),
                                   (200, 5, 512), (137, 4, 256)])
def test_persistent_lstm_sequence_matches_step_kernels(B, T, H):
    """csrc/lstm_seq.hip (one persistent launch per direction, W resident in VGPRs, per-step group hand-off) vs the
    per-step kernels of csrc/lstm.hip and the fp64 torch recurrence: outputs, final state and all four gradients;
    the launch's error word (set by a timed-out spin) stays 0."""
    from bigdl_amd.nn.recurrent import _LSTMSeq
    from bigdl_amd.ops import native

    C = native.get()
    torch.manual_seed(1)
    xg = torch.randn(B, T, 4 * H) * 0.5
    h0, c0 = torch.randn(B, H) * 0.5, torch.randn(B, H) * 0.5
    U = (torch.randn(4 * H, H) / H ** 0.5).to(torch.bfloat16).float()
    go = torch.randn(B, T, H)
    gh, gc = torch.randn(B, H), torch.randn(B, H)
    res = {}
    try:
        for seq in (1, 0):
            C.set_lstm_seq(seq)
            assert bool(C.lstm_seq_supported(B, H)) == bool(seq)
            dev = [t.cuda().requires_grad_(True) for t in (xg, h0, c0, U)]
            out, hT, cT = _LSTMSeq.apply(*dev)
            torch.autograd.backward([out, hT, cT], [go.cuda(), gh.cuda(), gc.cuda()])
            torch.cuda.synchronize()
            res[seq] = [out.detach(), hT.detach(), cT.detach()] + [d.grad for d in dev]
    finally:
        C.set_lstm_seq(1)
    for a, b in zip(res[1], res[0]):
        assert torch.isfinite(a).all()
        assert _rel(a, b) < 1e-2, _rel(a, b)
    # direct launch: error word untouched
    W16 = U.cuda().to(torch.bfloat16)
    h16 = torch.zeros(T + 1, B, H, device="cuda", dtype=torch.bfloat16)
    h16[0] = h0.cuda().to(torch.bfloat16)
    out = torch.empty(B, T, H, device="cuda")
    cs, acts = torch.empty(T, B, H, device="cuda"), torch.empty(T, B, 4 * H, device="cuda")
    sync = torch.full((C.lstm_seq_sync_words(),), 7, dtype=torch.int32, device="cuda")
    C.lstm_seq_fwd(W16, xg.cuda(), c0.cuda(), h16, out, None, cs, acts, sync)
    torch.cuda.synchronize()
    assert int(sync[8 * 32].item()) == 0
    assert _rel(out, res[0][0]) < 1e-2


def _hogged_lstm_forward(timeout_us, hog_us=300e3, n_hog=64, B=128, T=8, H=1024):
    """Persistent LSTM forward launched while `n_hog` CUs are held (whole-LDS spinning workgroups) by a kernel on
    another stream: some of the 256 workgroups cannot be resident until the hog ends."""
    from bigdl_amd.ops import native

    C = native.get()
    torch.manual_seed(5)
    xg = (torch.randn(B, T, 4 * H) * 0.5).cuda()
    c0, h0 = (torch.randn(B, H) * 0.5).cuda(), (torch.randn(B, H) * 0.5).cuda()
    W16 = (torch.randn(4 * H, H) / H ** 0.5).cuda().to(torch.bfloat16)

    def run():
        h16 = torch.zeros(T + 1, B, H, device="cuda", dtype=torch.bfloat16)
        h16[0] = h0.to(torch.bfloat16)
        out = torch.empty(B, T, H, device="cuda")
        cs, acts = torch.empty(T, B, H, device="cuda"), torch.empty(T, B, 4 * H, device="cuda")
        sync = torch.empty(C.lstm_seq_sync_words(), dtype=torch.int32, device="cuda")
        C.lstm_seq_fwd(W16, xg, c0, h16, out, None, cs, acts, sync)
        return out, cs

    ref, ref_cs = run()
    torch.cuda.synchronize()
    native.check_persistent()
    done = torch.zeros(n_hog, dtype=torch.int32, device="cuda")
    # a high-priority stream gets a hardware queue of its own: a normal-priority side stream may share the default
    # stream's queue (GPU_MAX_HW_QUEUES = 4 and earlier tests created many streams), which serialises the two launches
    side = torch.cuda.Stream(priority=-1)
    hog_end, run_start = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    C.set_seq_timeout_us(timeout_us)
    try:
        with torch.cuda.stream(side):
            C.hog_cus(n_hog, hog_us, done)
            hog_end.record()
        time.sleep(0.05)                 # the hog is resident before the persistent launch is queued
        run_start.record()
        out, cs = run()
        torch.cuda.synchronize()
    finally:
        C.set_seq_timeout_us(0)
    assert int((done > 0).sum()) == n_hog
    if hog_end.elapsed_time(run_start) > 0:   # the persistent launch started after the hog ended, not beside it
        native.check_persistent()
        pytest.skip("the hog and the persistent launch were not concurrent (shared hardware queue)")
    return ref, ref_cs, out, cs


def test_persistent_lstm_waits_out_other_streams():
    """Workgroups held back by another stream's kernel (64 CUs hogged for 0.3 s) only delay the persistent launch:
    with the default bound the output equals an unhindered launch bit for bit and no timeout is recorded."""
    from bigdl_amd.ops import native

    ref, ref_cs, out, cs = _hogged_lstm_forward(timeout_us=0)
    native.check_persistent()
    assert torch.equal(out, ref) and torch.equal(cs, ref_cs)


def test_persistent_lstm_forced_timeout_raises():
    """With the wait bound forced below the hog's duration the launch cannot complete: the host check raises
    PersistentKernelTimeout (never a silent NaN), and the outputs are NaN-poisoned rather than partly unwritten."""
    from bigdl_amd.ops import native

    ref, ref_cs, out, cs = _hogged_lstm_forward(timeout_us=20e3)
    with pytest.raises(native.PersistentKernelTimeout):
        native.check_persistent()
    native.check_persistent()           # cleared by the raising check
    assert torch.isnan(cs).any()
    # every element is either the correct value or poisoned: nothing is left as uninitialised memory
    ok = torch.isnan(cs) | (cs == ref_cs)
    assert bool(ok.all())


@pytest.mark.parametrize("B,T,H", [(128, 12, 1024), (40, 5, 256), (256, 6, 1024)])
def test_persistent_lstm_bf16_io_matches_f32_io(B, T, H):
    """bf16 gate inputs / outputs / gradients (the projection GEMMs' dtype, no f32 round trip) vs the f32-I/O launch of
    the same kernels: outputs, final state and all four gradients within bf16 rounding of the I/O tensors."""
    from bigdl_amd.nn.recurrent import _LSTMSeq

    torch.manual_seed(3)
    xg = (torch.randn(B, T, 4 * H) * 0.5).to(torch.bfloat16).float()
    h0, c0 = torch.randn(B, H) * 0.5, torch.randn(B, H) * 0.5
    U = (torch.randn(4 * H, H) / H ** 0.5).to(torch.bfloat16).float()
    go = torch.randn(B, T, H).to(torch.bfloat16).float()
    gh, gc = torch.randn(B, H), torch.randn(B, H)
    res = {}
    for dt in (torch.float32, torch.bfloat16):
        dev = [xg.cuda().to(dt).requires_grad_(True)] + [t.cuda().requires_grad_(True) for t in (h0, c0, U)]
        out, hT, cT = _LSTMSeq.apply(*dev)
        assert out.dtype == dt and hT.dtype == torch.float32
        torch.autograd.backward([out, hT, cT], [go.cuda().to(dt), gh.cuda(), gc.cuda()])
        torch.cuda.synchronize()
        res[dt] = [out.detach().float(), hT.detach(), cT.detach()] + [d.grad.float() for d in dev]
    for a, b in zip(res[torch.bfloat16], res[torch.float32]):
        assert torch.isfinite(a).all()
        assert _rel(a, b) < 1.5e-2, _rel(a, b)


def test_recurrent_output_dtype_stable_across_batch_sizes():
    """Recurrent(LSTM) returns fp32 on the GPU whatever the batch size (persistent whole-sequence kernels at B <= 128,
    per-step kernels above): bf16 sequence I/O is an explicit opt-in (Recurrent(bf16IO=True))."""
    from bigdl_amd import nn

    for B in (16, 300):
        torch.manual_seed(0)
        m = nn.Recurrent().add(nn.LSTM(64, 256, 0)).cuda()
        x = torch.randn(B, 5, 64, device="cuda")
        y = m.forward(x)
        assert y.dtype == torch.float32, (B, y.dtype)
        g = m.backward(x, torch.randn_like(y))
        assert g.dtype == x.dtype
    m = nn.Recurrent(bf16IO=True).add(nn.LSTM(64, 256, 0)).cuda()
    y = m.forward(torch.randn(16, 5, 64, device="cuda"))
    assert y.dtype in (torch.bfloat16, torch.float32)


@pytest.mark.parametrize("B,T,H", [(128, 12, 1024), (37, 6, 512), (9, 5, 256)])
def test_persistent_gru_sequence_matches_step_kernels(B, T, H):
    """Persistent whole-sequence GRU (csrc/lstm_seq.hip gru_seq_*_kernel: one launch per direction, two group
    hand-offs per step) vs the per-step GRU kernels (csrc/gru.hip) and an fp64 torch recurrence: outputs, final state
    and all four gradients (input gates, h0, U_rz, U_n)."""
    from bigdl_amd.nn.recurrent import _GRUSeq
    from bigdl_amd.ops import native

    C = native.get()
    torch.manual_seed(2)
    xg = torch.randn(B, T, 3 * H) * 0.5
    h0 = torch.randn(B, H) * 0.5
    Urz = (torch.randn(2 * H, H) / H ** 0.5).to(torch.bfloat16).float()
    Un = (torch.randn(H, H) / H ** 0.5).to(torch.bfloat16).float()
    go, gh = torch.randn(B, T, H), torch.randn(B, H)
    res = {}
    try:
        for seq in (1, 0):
            C.set_lstm_seq(seq)
            assert bool(C.gru_seq_supported(B, H)) == bool(seq)
            dev = [t.cuda().requires_grad_(True) for t in (xg, h0, Urz, Un)]
            out, hT = _GRUSeq.apply(*dev)
            torch.autograd.backward([out, hT], [go.cuda(), gh.cuda()])
            torch.cuda.synchronize()
            res[seq] = [out.detach(), hT.detach()] + [d.grad for d in dev]
    finally:
        C.set_lstm_seq(1)
    native.check_persistent()
    for a, b in zip(res[1], res[0]):
        assert torch.isfinite(a).all()
        assert _rel(a, b) < 2e-2, _rel(a, b)
    # fp64 recurrence for the outputs
    x64, h = xg.double(), h0.double()
    outs = []
    for t in range(T):
        rz = torch.sigmoid(x64[:, t, :2 * H] + h @ Urz.double().t())
        r, z = rz[:, :H], rz[:, H:]
        n = torch.tanh(x64[:, t, 2 * H:] + (r * h) @ Un.double().t())
        h = (1 - z) * n + z * h
        outs.append(h)
    ref = torch.stack(outs, 1)
    assert _rel(res[1][0], ref) < 1e-2


def _philox_np(seed, ctr):
    """Philox-4x32-10 (csrc/lstm_drop.hip philox4) over a numpy array of 64-bit counters -> 4 uint32 arrays."""
    import numpy as np

    M = np.uint64(0xFFFFFFFF)
    ctr = ctr.astype(np.uint64)
    c0, c1 = ctr & M, ctr >> np.uint64(32)
    c2 = np.zeros_like(c0)
    c3 = np.zeros_like(c0)
    k0, k1 = np.uint64(seed & 0xFFFFFFFF), np.uint64((seed >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c0
        p1 = np.uint64(0xCD9E8D57) * c2
        n0 = (p1 >> np.uint64(32)) ^ c1 ^ k0
        n2 = (p0 >> np.uint64(32)) ^ c3 ^ k1
        c1, c3, c0, c2 = p1 & M, p0 & M, n0 & M, n2 & M
        k0, k1 = (k0 + np.uint64(0x9E3779B9)) & M, (k1 + np.uint64(0xBB67AE85)) & M
    return c0, c1, c2, c3


def _keep_mask(seed, ids, p):
    import numpy as np

    r = _philox_np(seed, ids >> 2)
    sel = np.choose((ids & 3).astype(np.int64), r)
    return ((sel >> np.uint64(8)).astype(np.float64) / 16777216.0) >= p


@pytest.mark.parametrize("B,T,I,H,p", [(5, 4, 12, 32, 0.3), (16, 6, 40, 64, 0.5)])
def test_native_lstm_dropout_matches_masked_fp32_reference(B, T, I, H, p):
    """The native p != 0 LSTM (csrc/lstm_drop.hip + bmm_nt + the fused cell) against an fp32 torch LSTM that applies
    the SAME per-gate masks, regenerated here from the kernel's Philox counters: output, final state and the
    gradients of input, initial state and all four parameter tensors."""
    import numpy as np

    from bigdl_amd.nn import recurrent as rc
    from bigdl_amd.ops import nnk

    torch.manual_seed(0)
    dev = "cuda"
    x = torch.randn(B, T, I, device=dev)
    h0 = torch.randn(B, H, device=dev) * 0.5
    c0 = torch.randn(B, H, device=dev) * 0.5
    Wi = torch.randn(4 * H, I, device=dev) / I ** 0.5
    bi = torch.randn(4 * H, device=dev) * 0.1
    U = torch.randn(4 * H, H, device=dev) / H ** 0.5
    bu = torch.randn(4 * H, device=dev) * 0.1
    seeds = []
    orig = nnk.next_seed

    def rec_seed():
        s = orig()
        seeds.append(s)
        return s

    nnk.next_seed = rec_seed
    try:
        leaves = [t.clone().requires_grad_(True) for t in (x, h0, c0, Wi, bi, U, bu)]
        out, hT, cT = rc._LSTMDropSeq.apply(*leaves, p)
        go = torch.randn_like(out)
        gh = torch.randn_like(hT)
        (out * go).sum().backward(retain_graph=True)
    finally:
        nnk.next_seed = orig
    sx, sh = seeds
    keep = 1.0 - p
    # masks: x -> id ((g*T + t)*B + b)*I + k; h at step t -> ((g*B + b)*H + k) + t*4*B*H
    g_, t_, b_, k_ = np.meshgrid(np.arange(4), np.arange(T), np.arange(B), np.arange(I), indexing="ij")
    mx = _keep_mask(sx, ((g_ * T + t_) * B + b_) * I + k_, p)                         # [4, T, B, I]
    g2, b2, k2 = np.meshgrid(np.arange(4), np.arange(B), np.arange(H), indexing="ij")
    mh = np.stack([_keep_mask(sh, (g2 * B + b2) * H + k2 + t * 4 * B * H, p) for t in range(T)])   # [T, 4, B, H]
    mx = torch.as_tensor(mx, dtype=torch.float32, device=dev) / keep
    mh = torch.as_tensor(mh, dtype=torch.float32, device=dev) / keep
    refl = [t.clone().requires_grad_(True) for t in (x, h0, c0, Wi, bi, U, bu)]
    xr, hr, cr, Wr, bir, Ur, bur = refl
    outs = []
    h, c = hr, cr
    for t in range(T):
        gx = torch.einsum("gbi,ghi->bgh", xr[:, t].unsqueeze(0) * mx[:, t], Wr.view(4, H, I)).reshape(B, 4 * H)
        gh_ = torch.einsum("gbk,ghk->bgh", h.unsqueeze(0) * mh[t], Ur.view(4, H, H)).reshape(B, 4 * H)
        g = gx + bir + gh_ + bur
        i, gg, f, o = (torch.sigmoid(g[:, :H]), torch.tanh(g[:, H:2 * H]), torch.sigmoid(g[:, 2 * H:3 * H]),
                       torch.sigmoid(g[:, 3 * H:]))
        c = f * c + i * gg
        h = o * torch.tanh(c)
        outs.append(h)
    outr = torch.stack(outs, 1)
    (outr * go).sum().backward()
    assert _rel(out, outr) < 2e-2, _rel(out, outr)
    assert _rel(hT, h) < 2e-2 and _rel(cT, c) < 2e-2
    for a, r, name in zip(leaves, refl, ["x", "h0", "c0", "Wi", "bi", "U", "bu"]):
        assert a.grad is not None, name
        assert _rel(a.grad, r.grad) < 3e-2, (name, _rel(a.grad, r.grad))


def test_lstm_dropout_module_runs_native_path_on_gpu():
    """nn.LSTM(p != 0) inside Recurrent on the GPU takes the native dropout path in training (no per-step aten
    bernoulli / bmm), and evaluation matches the CPU engine."""
    from bigdl_amd import nn
    from bigdl_amd.nn import recurrent as rc
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(7)
    cpu = nn.Recurrent().add(nn.LSTM(16, 64, p=0.25))
    gpu = copy.deepcopy(cpu).to("cuda")
    x = torch.randn(8, 5, 16)
    calls = []
    orig = rc._LSTMDropSeq.forward

    def spy(ctx, *a):
        calls.append(1)
        return orig(ctx, *a)

    rc._LSTMDropSeq.forward = staticmethod(spy)
    try:
        gpu.training()
        y = gpu.forward(x.cuda())
        gpu.backward(x.cuda(), torch.ones_like(y))
    finally:
        rc._LSTMDropSeq.forward = staticmethod(orig)
    assert calls, "native dropout LSTM path not taken"
    cpu.evaluate()
    gpu.evaluate()
    assert _rel(gpu.forward(x.cuda()), cpu.forward(x)) < 1e-2
