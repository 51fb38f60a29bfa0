"""cProfile of the host side of one eager ResNet-50 training iteration (enqueue only: the in-flight throttle is
lifted so the host never waits for the device). Prints the top functions by own time."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from bigdl_amd import nn
    from bigdl_amd.models.resnet import DatasetType, ResNet
    from bigdl_amd.optim.sgd import SGD
    from bigdl_amd.optim.train_step import TrainStep
    from bigdl_amd.utils.engine import Engine

    Engine.init(master="local[1]", dist=False)
    dev = torch.device("cuda", 0)
    model = ResNet(1000, 50, dataSet=DatasetType.ImageNet)
    step = TrainStep(model, nn.CrossEntropyCriterion(), SGD(0.1, momentum=0.9, dampening=0.0), device=dev)
    B = int(os.environ.get("BATCH", "64"))
    x = torch.randn(B, 3, 224, 224, device=dev)
    y = torch.randint(1, 1001, (B,), device=dev).float()
    for _ in range(3):
        step.step(x, y)
    torch.cuda.synchronize()
    step.MAX_INFLIGHT = 1 << 20
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(3):
        step.step(x, y)
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()
