"""Model throughput on the GPU engine: training steps (forward + backward + SGD) or fused inference.

Reference: S/nn/mkldnn/Perf.scala (ResNet-50 / VGG-16 / Inception-v1 with random inputs, training or inference,
batch size and iteration count from the command line, images/second per iteration) and the LocalOptimizerPerf /
DistriOptimizerPerf harnesses. Training runs the same TrainStep as bench.py (HIP-graph captured when
``--graph 1``); inference runs the model lowered to the fused engine (``ConversionUtils.convert(..., "dnn")``).

    python -m bigdl_amd.examples perf --model resnet50 --batchSize 64 --iteration 10 [--training 0]
"""
import argparse
import time

import torch

from ._common import device_of


def build(name, classes):
    from ..models.inception import Inception_v1_NoAuxClassifier, Inception_v3
    from ..models.resnet import DatasetType, ResNet
    from ..models.vgg import Vgg_16

    if name == "resnet50":
        return ResNet(classes, 50, dataSet=DatasetType.ImageNet), 224
    if name == "vgg16":
        return Vgg_16(classes, False), 224
    if name == "inception_v1":
        return Inception_v1_NoAuxClassifier(classes), 224
    if name == "inception_v3":
        return Inception_v3(classes), 299
    raise ValueError(name)


def run(args):
    from .. import nn
    from ..optim.sgd import SGD
    from ..optim.train_step import TrainStep
    from ..utils.intermediate import ConversionUtils
    from ..utils.random_generator import RNG

    dev = device_of(args.device)
    RNG.setSeed(1)
    model, side = build(args.model, args.classNum)
    B = args.batchSize
    x = torch.randn(B, 3, side, side, device=dev)
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    times = []
    if args.training:
        y = torch.randint(1, args.classNum + 1, (B,), device=dev).float()
        step = TrainStep(model, nn.CrossEntropyCriterion(), SGD(learningRate=0.01, momentum=0.9, dampening=0.0),
                         device=dev)
        run_step = lambda: step.step(x, y)          # noqa: E731
        if args.graph and dev.type == "cuda":
            from ..optim.graphed import GraphedTrainStep

            graphed = GraphedTrainStep(step, x, y, warmup=2)
            run_step = graphed.replay
    else:
        model.evaluate()
        fused = ConversionUtils.convert(model, "dnn", device=dev, train=False) if dev.type == "cuda" else model
        run_step = lambda: fused.forward(x)          # noqa: E731
    with torch.no_grad() if not args.training else torch.enable_grad():
        for _ in range(2):
            run_step()
        sync()
        for _ in range(args.iteration):
            t0 = time.perf_counter()
            run_step()
            sync()
            times.append(time.perf_counter() - t0)
    ms = sorted(times)[len(times) // 2] * 1e3
    return {"model": args.model, "training": bool(args.training), "batch": B, "median_ms": round(ms, 3),
            "images_per_s": round(B / ms * 1e3, 1)}


def build_parser():
    p = argparse.ArgumentParser(prog="perf")
    p.add_argument("--model", choices=["resnet50", "vgg16", "inception_v1", "inception_v3"], default="resnet50")
    p.add_argument("--batchSize", type=int, default=32)
    p.add_argument("--iteration", type=int, default=5)
    p.add_argument("--training", type=int, default=1)
    p.add_argument("--graph", type=int, default=1)
    p.add_argument("--classNum", type=int, default=1000)
    p.add_argument("--device", default="auto")
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
