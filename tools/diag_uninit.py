"""Uninitialised-memory probe: one ResNet training forward + backward (TrainStep.forward_backward, fused GPU path,
no update) repeated on identical inputs; before each trial the caching allocator's free blocks are poisoned
(large NaN / 1e30 / zero tensors allocated and released), so any kernel that reads memory it did not write shows up
as a per-module difference between trials. Prints the first modules (forward order) whose output / gradInput
differs, and the flat-gradient difference."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bigdl_amd  # noqa: E402,F401
from bigdl_amd import nn  # noqa: E402
from bigdl_amd import optim as O  # noqa: E402
from bigdl_amd.models.resnet import DatasetType, ResNet  # noqa: E402
from bigdl_amd.optim.train_step import TrainStep  # noqa: E402
from bigdl_amd.utils.random_generator import RNG  # noqa: E402

depth = int(sys.argv[1]) if len(sys.argv) > 1 else 20
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 16
dev = torch.device("cuda:0")
RNG.setSeed(42)
if depth in (20, 32, 56):
    model = ResNet(10, depth, dataSet=DatasetType.CIFAR10)
    shape = (batch, 3, 32, 32)
else:
    model = ResNet(1000, depth, dataSet=DatasetType.ImageNet)
    shape = (batch, 3, 224, 224)
step = TrainStep(model, nn.CrossEntropyCriterion(), O.SGD(0.05), device=dev)
g = torch.Generator().manual_seed(0)
x = torch.randn(*shape, generator=g).to(dev)
y = torch.randint(1, 11, (batch,), generator=g).float().to(dev)
mods = [m for m in model.flattened_layers() if not m.modules_list()]


def snap():
    out = []
    for m in mods:
        o = getattr(m, "output", None)
        gi = getattr(m, "gradInput", None)
        out.append((o.detach().float().clone() if isinstance(o, torch.Tensor) else None,
                    gi.detach().float().clone() if isinstance(gi, torch.Tensor) else None))
    return out, step.g.detach().clone()


def poison(val):
    free, _ = torch.cuda.mem_get_info()
    n = min(int(free * 0.5) // 4, 1 << 30)
    chunks = []
    for sz in (n // 2, n // 4, n // 8, 1 << 24, 1 << 22, 1 << 20, 1 << 16):
        chunks.append(torch.full((sz,), val, device=dev))
    torch.cuda.synchronize()
    del chunks


res = []
for trial, val in enumerate([0.0, float("nan"), 1e30, -7.0]):
    poison(val)
    step.zero_grad()
    step.forward_backward_step(x, y)
    torch.cuda.synchronize()
    res.append(snap())
ref, gref = res[0]
for t, (r, gr) in enumerate(res[1:], 1):
    bad = []
    for i, (m, (o0, g0), (o1, g1)) in enumerate(zip(mods, ref, r)):
        for kind, a, b in (("out", o0, o1), ("gradIn", g0, g1)):
            if a is None or b is None or a.shape != b.shape:
                continue
            d = (a - b).abs().max().item() if a.numel() else 0.0
            if not (d == 0.0):
                bad.append(f"{i}:{type(m).__name__}.{kind} maxdiff={d:.3e} nan={bool(torch.isnan(b).any())}")
    dg = (gr - gref).abs().max().item()
    print(f"trial {t}: flat grad maxdiff {dg:.3e} nan={bool(torch.isnan(gr).any())}; {len(bad)} differing tensors; "
          f"first: {bad[:6]}", flush=True)
