"""Large Linear GEMMs on hipBLASLt (nn/linear.py _use_blas): forward with bias, input gradient, fp32 weight gradient
and the bias gradient from the ones column, against the in-tree MFMA kernels and a plain fp32 PyTorch reference."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("bias", [True, False])
def test_linear_blas_route_matches(bias):
    from bigdl_amd import nn
    from bigdl_amd.nn import linear as L

    torch.manual_seed(3)
    M, K, N = 8192, 512, 2048
    x = (torch.randn(M, K) * 0.5).to(torch.bfloat16).float()
    gy = (torch.randn(M, N) * 0.1).to(torch.bfloat16).float()
    ref = nn.Linear(K, N, withBias=bias)
    res = {}
    saved = L._BLAS[0]
    try:
        for on in (True, False):
            L._BLAS[0] = on
            m = nn.Linear(K, N, withBias=bias)
            m.weight.data.copy_(ref.weight.data)
            if bias:
                m.bias.data.copy_(ref.bias.data)
            m = m.to("cuda")
            y = m.forward(x.cuda())
            assert (getattr(m, "_xe", None) is not None) == on, "route"
            gi = m.backward(x.cuda(), gy.cuda())
            torch.cuda.synchronize()
            res[on] = (y.float().cpu(), gi.float().cpu(), m.gradWeight.float().cpu().clone(),
                       m.gradBias.float().cpu().clone() if bias else None)
    finally:
        L._BLAS[0] = saved
    w = ref.weight.data.to(torch.bfloat16).float()
    y_ref = x @ w.t() + (ref.bias.data if bias else 0)
    assert _rel(res[True][0], y_ref) < 1e-2 and _rel(res[True][0], res[False][0]) < 1e-2
    assert _rel(res[True][1], gy @ w) < 1e-2 and _rel(res[True][1], res[False][1]) < 1e-2
    assert _rel(res[True][2], gy.t() @ x) < 1e-3 and _rel(res[True][2], res[False][2]) < 1e-3
    if bias:
        assert _rel(res[True][3], gy.sum(0)) < 1e-3 and _rel(res[True][3], res[False][3]) < 1e-3


def test_recurrent_weight_gradient_blas_route_matches():
    """The whole-sequence LSTM's recurrent weight gradient dU = dg^T h on hipBLASLt (accumulated in place into the
    fp32 gradient) against the in-tree weight-gradient kernel on the same inputs (only that route toggled)."""
    import copy

    from bigdl_amd import nn
    from bigdl_amd.nn import recurrent as R

    torch.manual_seed(5)
    B, T, H = 64, 128, 512
    base = nn.Recurrent().add(nn.LSTM(H, H))
    x = (torch.randn(B, T, H) * 0.5).cuda()
    gy = (torch.randn(B, T, H) * 0.1).cuda()
    res = {}
    saved = R._RWG_BLAS[0]
    try:
        for on in (True, False):
            R._RWG_BLAS[0] = on
            assert R._recurrent_wgrad_blas(B * T, H) == on
            m = copy.deepcopy(base).cuda()
            m.training()
            m.forward(x)
            gi = m.backward(x, gy)
            torch.cuda.synchronize()
            res[on] = (gi.float().cpu(), m.cell.h2g.gradWeight.float().cpu().clone())
    finally:
        R._RWG_BLAS[0] = saved
    assert torch.equal(res[True][0], res[False][0])         # the input gradient does not depend on the route
    assert _rel(res[True][1], res[False][1]) < 1e-5        # fp32 accumulation both ways: summation order only


def test_gru_recurrent_weight_gradient_blas_route_matches():
    """The whole-sequence GRU's [2H x H] recurrent weight gradient on hipBLASLt (n = 2H meets the shape rule at
    H = 1024; the [H x H] one stays on the in-tree kernel) against the in-tree kernel on the same inputs."""
    import copy

    from bigdl_amd import nn, ops
    from bigdl_amd.nn import recurrent as R

    B, T, H = 64, 128, 1024
    if not ops.native.get().gru_seq_supported(B, H):
        pytest.skip("whole-sequence GRU not available for this shape")
    torch.manual_seed(6)
    base = nn.Recurrent().add(nn.GRU(H, H))
    x = (torch.randn(B, T, H) * 0.5).cuda()
    gy = (torch.randn(B, T, H) * 0.1).cuda()
    res = {}
    saved = R._RWG_BLAS[0]
    try:
        for on in (True, False):
            R._RWG_BLAS[0] = on
            assert R._recurrent_wgrad_blas(B * T, H, 2 * H) == on and not R._recurrent_wgrad_blas(B * T, H, H)
            m = copy.deepcopy(base).cuda()
            m.training()
            m.forward(x)
            gi = m.backward(x, gy)
            torch.cuda.synchronize()
            res[on] = (gi.float().cpu(), m.cell.h2g.gradWeight.float().cpu().clone(),
                       m.cell.h2n.gradWeight.float().cpu().clone())
    finally:
        R._RWG_BLAS[0] = saved
    assert _rel(res[True][0], res[False][0]) < 1e-6
    assert _rel(res[True][1], res[False][1]) < 1e-5
    assert _rel(res[True][2], res[False][2]) < 1e-5          # (fp32 atomic order of the in-tree kernel only)
