"""Fused vs unfused vs fp32-CPU gradients for the Sequential and Graph forms of ResNet-20 (per parameter tensor)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


def run(build, x, y, fused):
    from bigdl_amd import nn
    from bigdl_amd.nn.fusion import fuse_for_training

    m = copy.deepcopy(build)
    if fused is not None:
        m = m.to("cuda")
        if fused:
            fuse_for_training(m)
        x, y = x.cuda(), y.cuda()
    crit = nn.CrossEntropyCriterion()
    out = m.forward(x)
    crit.forward(out, y)
    m.backward(x, crit.backward(out, y))
    return [t.float().cpu().reshape(-1).clone() for t in m.parameters()[1]]


def main():
    from bigdl_amd.models.resnet import DatasetType, ResNet, ResNetGraph
    from bigdl_amd.utils.random_generator import RNG

    torch.manual_seed(0)
    x = torch.randn(16, 3, 32, 32).to(torch.bfloat16).float()
    y = torch.randint(1, 11, (16,)).float()
    for name, fn in (("seq", ResNet), ("graph", ResNetGraph)):
        RNG.setSeed(5)
        base = fn(10, 20, dataSet=DatasetType.CIFAR10)
        c = run(base, x, y, None)
        u = run(base, x, y, False)
        u2 = run(base, x, y, False)
        f = run(base, x, y, True)
        cat = torch.cat
        print(f"{name}: fused-unfused {rel(cat(f), cat(u)):.4f} unfused-unfused {rel(cat(u2), cat(u)):.4f} "
              f"fused-cpu {rel(cat(f), cat(c)):.4f} unfused-cpu {rel(cat(u), cat(c)):.4f}", flush=True)
        for i, (a, b, cc) in enumerate(zip(f, u, c)):
            print(f"  p{i:02d} n={a.numel():6d} f-u {rel(a, b):.4f} f-c {rel(a, cc):.4f} u-c {rel(b, cc):.4f}")


if __name__ == "__main__":
    main()
