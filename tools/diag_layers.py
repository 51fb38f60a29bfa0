"""Per-layer GPU-vs-CPU diagnostic: run a model on the fp32 CPU engine and on the GPU engine (optionally
fused), then report the relative error of every leaf module's output and gradInput in execution order."""
import argparse
import copy
import sys

import torch

sys.path.insert(0, ".")
from bigdl_amd import nn  # noqa: E402
from bigdl_amd.models.resnet import ResNet  # noqa: E402
from bigdl_amd.nn.fusion import fuse_for_training  # noqa: E402


def rel(a, b):
    if a is None or b is None or not isinstance(a, torch.Tensor) or not isinstance(b, torch.Tensor):
        return float("nan")
    if a.shape != b.shape:
        return float("nan")
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth", type=int, default=20)
    ap.add_argument("--dataset", default="CIFAR10")
    ap.add_argument("--img", type=int, default=32)
    ap.add_argument("--fuse", type=int, default=1)
    a = ap.parse_args()
    torch.manual_seed(0)
    cpu = ResNet(10 if a.dataset == "CIFAR10" else 1000, a.depth, dataSet=a.dataset)
    g = torch.Generator().manual_seed(3)
    for m in cpu.flattened_layers():
        if isinstance(m, nn.BatchNormalization) and m.affine:
            m.weight.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
            m.bias.copy_(torch.randn(m.bias.shape, generator=g) * 0.1)
    gpu = copy.deepcopy(cpu).to("cuda")
    if a.fuse:
        fuse_for_training(gpu)
    x = torch.randn(4, 3, a.img, a.img)
    y = torch.randint(1, 11, (4,)).float()
    cc, cg = nn.CrossEntropyCriterion(), nn.CrossEntropyCriterion()
    oc = cpu.forward(x)
    og = gpu.forward(x.cuda())
    cc.forward(oc, y)
    cg.forward(og, y.cuda())
    cpu.backward(x, cc.backward(oc, y))
    gpu.backward(x.cuda(), cg.backward(og, y.cuda()))
    lc = [m for m in cpu.flattened_layers() if not m.modules_list()]
    lg = [m for m in gpu.flattened_layers() if not m.modules_list()]
    for i, (mc, mg) in enumerate(zip(lc, lg)):
        gw = ""
        p = mc.parameters()
        if p is not None:
            gw = " ".join(f"{rel(b, a2):.3g}" for a2, b in zip(p[1], mg.parameters()[1]))
        print(f"{i:3d} {type(mc).__name__:28s} out {rel(mg.output, mc.output):8.3g}  gin {rel(mg.gradInput, mc.gradInput):8.3g}  "
              f"gparams [{gw}]")


if __name__ == "__main__":
    main()
