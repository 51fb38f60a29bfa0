"""Which Python call sites issue device copies / fills in one ResNet-50 training step (torch.profiler stacks).

    python tools/find_copies.py [--batch 64]
"""
import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    args = ap.parse_args()
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import DatasetType, ResNet
    from bigdl_amd.optim.sgd import SGD
    from bigdl_amd.optim.train_step import TrainStep
    from bigdl_amd.utils.engine import Engine

    Engine.init(master="local[1]", dist=False)
    dev = torch.device("cuda", 0)
    step = TrainStep(ResNet(1000, 50, dataSet=DatasetType.ImageNet), nn.CrossEntropyCriterion(),
                     SGD(learningRate=0.1, momentum=0.9, dampening=0.0), device=dev)
    x = torch.randn(args.batch, 3, 224, 224, device=dev)
    y = torch.randint(1, 1001, (args.batch,), device=dev).float()
    for _ in range(3):
        step.step(x, y)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step.step(x, y)
        torch.cuda.synchronize()
    sites = collections.Counter()
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::clone", "aten::contiguous", "aten::to",
                       "aten::cat", "aten::zeros", "aten::zeros_like"):
            st = [f for f in (ev.stack or []) if "bigdl_amd" in f or "bench" in f][:3]
            sites[(ev.name, " <- ".join(st))] += 1
    for (name, st), n in sites.most_common(40):
        print(f"{n:5d}  {name:18s} {st}")
    Engine.shutdown()


if __name__ == "__main__":
    main()
