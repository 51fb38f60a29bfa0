"""Calibration only: pure-PyTorch (MIOpen) ResNet-50 v1.5 bf16 channels_last training step throughput.

Not part of the framework; used to see where the vendor-library path sits on this box so the native
bigdl_amd kernels have a concrete number to beat.
"""
import argparse
import json
import time

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    def __init__(self, cin, n, stride):
        super().__init__()
        self.c1 = nn.Conv2d(cin, n, 1, bias=False)
        self.b1 = nn.BatchNorm2d(n)
        self.c2 = nn.Conv2d(n, n, 3, stride, 1, bias=False)
        self.b2 = nn.BatchNorm2d(n)
        self.c3 = nn.Conv2d(n, n * 4, 1, bias=False)
        self.b3 = nn.BatchNorm2d(n * 4)
        self.sc = None
        if stride != 1 or cin != n * 4:
            self.sc = nn.Sequential(nn.Conv2d(cin, n * 4, 1, stride, bias=False), nn.BatchNorm2d(n * 4))

    def forward(self, x):
        y = torch.relu(self.b1(self.c1(x)))
        y = torch.relu(self.b2(self.c2(y)))
        y = self.b3(self.c3(y))
        return torch.relu(y + (self.sc(x) if self.sc is not None else x))


def resnet50():
    layers = [nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(), nn.MaxPool2d(3, 2, 1)]
    cin = 64
    for n, cnt, st in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for i in range(cnt):
            layers.append(Bottleneck(cin, n, st if i == 0 else 1))
            cin = n * 4
    layers += [nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Linear(2048, 1000)]
    return nn.Sequential(*layers)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda")
    m = resnet50().to(dev).to(memory_format=torch.channels_last).to(torch.bfloat16)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(args.batch, 3, 224, 224, device=dev).to(torch.bfloat16, memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (args.batch,), device=dev)
    lossf = nn.CrossEntropyLoss()

    def step():
        opt.zero_grad(set_to_none=True)
        loss = lossf(m(x).float(), y)
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / args.steps
    print(json.dumps({"torch_miopen_resnet50_img_s": round(args.batch / dt, 1), "ms_per_step": round(dt * 1e3, 2)}))


if __name__ == "__main__":
    main()
