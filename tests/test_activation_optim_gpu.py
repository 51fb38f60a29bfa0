"""Native point-wise activations (csrc/activation.hip) and adaptive optimizer updates (csrc/optim.hip) vs the fp32
torch reference of the same layer / method on the CPU."""
import copy

import pytest
import torch

from bigdl_amd import nn

pytestmark = pytest.mark.gpu

CL = torch.channels_last
ACTS = [
    lambda: nn.Tanh(), lambda: nn.Sigmoid(), lambda: nn.ELU(0.7), lambda: nn.LeakyReLU(0.05), lambda: nn.ReLU6(),
    lambda: nn.SoftPlus(1.5), lambda: nn.SoftSign(), lambda: nn.HardTanh(-0.8, 1.2), lambda: nn.HardSigmoid(),
    lambda: nn.LogSigmoid(), lambda: nn.TanhShrink(), lambda: nn.SoftShrink(0.3), lambda: nn.HardShrink(0.4),
    lambda: nn.Threshold(0.2, -1.0), lambda: nn.Exp(), lambda: nn.Square(), lambda: nn.Abs(),
    lambda: nn.Log(), lambda: nn.Sqrt(),
]


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.parametrize("make", ACTS)
@pytest.mark.parametrize("dtype,layout", [(torch.float32, "flat"), (torch.bfloat16, "nhwc")])
def test_activation_native_matches_fp32(make, dtype, layout):
    torch.manual_seed(0)
    m = make()
    x = torch.randn(3, 8, 5, 7) * 2
    if type(m).__name__ in ("Log", "Sqrt"):
        x = x.abs() + 0.1
    gy = torch.randn_like(x)
    # reference on the dtype-rounded inputs: piecewise layers (thresholds, clamps) must see the same x
    x, gy = x.to(dtype).float(), gy.to(dtype).float()
    ref_m = copy.deepcopy(m)
    yr = ref_m.forward(x.clone())
    gr = ref_m.backward(x.clone(), gy)
    xd = x.to("cuda", dtype)
    gd = gy.to("cuda", dtype)
    if layout == "nhwc":
        xd, gd = xd.contiguous(memory_format=CL), gd.contiguous(memory_format=CL)
    y = m.forward(xd)
    assert m._native_x is not None, "native kernel not used"
    g = m.backward(xd, gd)
    tol = 1e-5 if dtype == torch.float32 else 1.5e-2
    assert _rel(y, yr) < tol
    assert _rel(g, gr) < (tol if dtype == torch.float32 else 3e-2)


@pytest.mark.parametrize("method", ["Adagrad", "RMSprop", "Adadelta", "Adamax", "Ftrl", "Ftrl_p"])
def test_adaptive_optimizer_native_matches_cpu(method):
    from bigdl_amd.optim import methods as M

    def make():
        return {"Adagrad": lambda: M.Adagrad(0.1, 0.01, 1e-3), "RMSprop": lambda: M.RMSprop(0.01, 0.0, 0.9, 1e-6),
                "Adadelta": lambda: M.Adadelta(0.9, 1e-6), "Adamax": lambda: M.Adamax(0.02),
                "Ftrl": lambda: M.Ftrl(0.1, -0.5, 0.1, 0.01, 0.02, 0.03),
                "Ftrl_p": lambda: M.Ftrl(0.1, -0.6, 0.1, 0.01, 0.02, 0.0)}[method]()
    torch.manual_seed(1)
    n = 4099                                        # exercises the scalar tail path too
    x0 = torch.randn(n)
    grads = [torch.randn(n) for _ in range(4)]
    xc, oc = x0.clone(), make()
    for g in grads:
        oc.optimize(lambda w, _g=g: (0.0, _g), xc)
    xg, og = x0.clone().cuda(), make()
    w16 = torch.empty(n, dtype=torch.bfloat16, device="cuda")
    og._shadow16 = w16
    for g in grads:
        og.optimize(lambda w, _g=g.cuda(): (0.0, _g), xg)
    assert torch.allclose(xg.cpu(), xc, rtol=1e-4, atol=1e-5), (xg.cpu() - xc).abs().max()
    assert torch.equal(w16, xg.to(torch.bfloat16))
    xv = torch.randn(4096).cuda()                   # vectorised path
    og2, oc2 = make(), make()
    xc2 = xv.cpu().clone()
    og2.optimize(lambda w: (0.0, grads[0][:4096].cuda()), xv)
    oc2.optimize(lambda w: (0.0, grads[0][:4096]), xc2)
    assert torch.allclose(xv.cpu(), xc2, rtol=1e-4, atol=1e-5)
