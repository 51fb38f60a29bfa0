"""Deterministic-mode check on the GPU (bigdl.deterministic): ResNet-20 (CIFAR-10 shape, BatchNorm, SGD + momentum)
trained for --iters iterations twice from the same seed must end with bitwise-equal weights; the same two runs without
the mode show how far the default (fp32-atomic) reductions drift. Also times a ResNet-50 batch-256 step in both modes
(--r50) to record the mode's cost.

    python tools/det_check.py [--iters 10] [--r50]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from bigdl_amd.ops import native  # noqa: E402


def run(iters, det, depth=20, batch=128, classes=10, image=32, dataset="CIFAR10", seed=3):
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import DatasetType, ResNet
    from bigdl_amd.optim.sgd import SGD
    from bigdl_amd.optim.train_step import TrainStep
    from bigdl_amd.utils.random_generator import RNG

    native.set_deterministic(det)
    RNG.setSeed(seed)
    torch.manual_seed(seed)
    dev = torch.device("cuda")
    model = ResNet(classes, depth, dataSet=getattr(DatasetType, dataset))
    step = TrainStep(model, nn.CrossEntropyCriterion(), SGD(learningRate=0.1, momentum=0.9, dampening=0.0,
                                                             weightDecay=1e-4), device=dev)
    g = torch.Generator(device="cpu").manual_seed(seed)
    xs = [torch.randn(batch, 3, image, image, generator=g).to(dev) for _ in range(2)]
    ys = [torch.randint(1, classes + 1, (batch,), generator=g).float().to(dev) for _ in range(2)]
    torch.cuda.synchronize()
    t0 = None
    for it in range(iters):
        if it == 2:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        step.step(xs[it % 2], ys[it % 2])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / max(1, iters - 2) if t0 is not None else float("nan")
    step.flush() if hasattr(step, "flush") else None
    w = step.w[:step.total].detach().clone()
    native.set_deterministic(False)
    return w, ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--r50", action="store_true")
    a = ap.parse_args()
    for det in (True, False):
        w1, _ = run(a.iters, det)
        w2, _ = run(a.iters, det)
        d = (w1 - w2).abs().max().item()
        print(f"ResNet-20 x{a.iters} iterations, deterministic={det}: bitwise equal {torch.equal(w1, w2)}, "
              f"max |dw| {d:.3e}", flush=True)
    if a.r50:
        for det in (False, True, False, True):
            _, ms = run(8, det, depth=50, batch=256, classes=1000, image=224, dataset="ImageNet")
            print(f"ResNet-50 b256 step, deterministic={det}: {ms:.2f} ms/step (eager, 6 timed)", flush=True)


if __name__ == "__main__":
    main()
