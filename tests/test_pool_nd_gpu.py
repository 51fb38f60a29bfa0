"""N-d pooling and nearest up-sampling kernels (csrc/pool_nd.hip) against the fp32 CPU layers (torch reference).

Covers VolumetricMax/AveragePooling (overlapping windows, padding, ceil mode, count_include_pad), TemporalMaxPooling,
the 2D pooling layers on channel counts the NHWC kernels do not take (generic path), and UpSampling1D/2D/3D, in fp32
and bf16, forward and backward. torch's own pooling functions are patched to raise during the GPU calls, so a pass
means the native kernels ran.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

from bigdl_amd import nn

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


def _block_torch_pooling(monkeypatch):
    def boom(*a, **k):
        raise AssertionError("torch pooling called on the GPU path")

    for name in ("max_pool1d", "max_pool2d", "max_pool3d", "avg_pool2d", "avg_pool3d"):
        monkeypatch.setattr(F, name, boom)


CASES = [
    ("vmax", lambda: nn.VolumetricMaxPooling(3, 3, 2, 2, 2, 1, 1, 1, 0), (2, 5, 7, 11, 9)),
    ("vmax_ceil", lambda: nn.VolumetricMaxPooling(2, 2, 2, 2, 2, 2).ceil(), (2, 4, 5, 7, 9)),
    ("vavg_pad", lambda: nn.VolumetricAveragePooling(3, 3, 3, 1, 2, 2, 1, 1, 1), (2, 3, 6, 9, 8)),
    ("vavg_nopad", lambda: nn.VolumetricAveragePooling(3, 3, 3, 2, 2, 2, 1, 1, 1, countIncludePad=False,
                                                        ceilMode=True), (1, 4, 7, 8, 9)),
    ("tmax", lambda: nn.TemporalMaxPooling(3, 2), (4, 17, 24)),
    ("smax_c3", lambda: nn.SpatialMaxPooling(3, 3, 2, 2, 1, 1).ceil(), (2, 3, 15, 17)),
    ("savg_c5", lambda: nn.SpatialAveragePooling(3, 2, 2, 1, 1, 0, countIncludePad=False), (2, 5, 9, 10)),
    ("up1", lambda: nn.UpSampling1D(3), (2, 7, 12)),
    ("up2", lambda: nn.UpSampling2D((2, 3)), (2, 3, 5, 6)),
    ("up2_nhwc", lambda: nn.UpSampling2D((3, 2), format="NHWC"), (2, 5, 6, 16)),
    ("up3", lambda: nn.UpSampling3D((2, 2, 3)), (1, 3, 4, 5, 6)),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("name,make,shape", CASES, ids=[c[0] for c in CASES])
def test_pool_nd_native_matches_fp32(name, make, shape, dtype, monkeypatch):
    torch.manual_seed(0)
    m = make()
    x = torch.randn(*shape).to(dtype).float()      # the reference sees the same (rounded) input
    ref = copy.deepcopy(m)
    yr = ref.forward(x.clone())
    gy = torch.randn(yr.shape).to(dtype).float()
    gr = ref.backward(x.clone(), gy)
    _block_torch_pooling(monkeypatch)              # from here on only the native kernels may pool
    xd = x.to("cuda", dtype)
    y = m.forward(xd)
    g = m.backward(xd, gy.to("cuda", dtype))
    assert y.shape == yr.shape and g.shape == x.shape
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert _rel(y, yr) < tol
    assert _rel(g, gr) < (tol if dtype == torch.float32 else 2e-2)


def test_max_pool_ties_and_overlap_sum_gradients():
    """Overlapping max windows that share a winner must add their gradients (gather form, no atomics)."""
    x = torch.zeros(1, 1, 1, 5, 5)
    x[0, 0, 0, 2, 2] = 5.0
    m = nn.VolumetricMaxPooling(1, 3, 3, 1, 1, 1)
    xd = x.cuda()
    y = m.forward(xd)
    g = m.backward(xd, torch.ones_like(y))
    assert float(y.max()) == 5.0
    assert float(g[0, 0, 0, 2, 2]) == 9.0            # all 9 windows pick the centre
    assert float(g.sum()) == 9.0
