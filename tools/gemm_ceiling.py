"""Ceiling of the implicit-GEMM conv kernels on plain GEMM shapes (1x1 convs) and ResNet-50 3x3 shapes: TF/s per
kernel variant (select with the BIGDL_CONV_* environment knobs; each process reads them once).
    python tools/gemm_ceiling.py   -> one line per shape: M K N us TF/s"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bigdl_amd  # noqa: E402,F401
from bigdl_amd.ops import conv as cv  # noqa: E402

CL, BF = torch.channels_last, torch.bfloat16
# (N, C, H, K, R, stride, pad)
SHAPES = [(1, 4096, 64, 4096, 1, 1, 0), (4, 2048, 64, 2048, 1, 1, 0), (256, 512, 7, 2048, 1, 1, 0),
          (256, 256, 14, 256, 3, 1, 1), (256, 512, 7, 512, 3, 1, 1), (256, 128, 28, 128, 3, 1, 1),
          (256, 64, 56, 256, 1, 1, 0)]


def main():
    dev = torch.device("cuda")
    tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("BIGDL_CONV"))
    for (N, C, H, K, R, st, pd) in SHAPES:
        x = (torch.rand(N, C, H, H, device=dev) * 2 - 1).to(BF, memory_format=CL)
        w = ((torch.rand(K, C, R, R, device=dev) * 2 - 1) * 0.05).to(BF, memory_format=CL)
        OH = cv.out_size(H, R, st, pd)
        fl = 2.0 * N * OH * OH * K * C * R * R
        fn = lambda: cv.conv2d_fwd(x, w, None, (st, st), (pd, pd))  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(15):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        us = statistics.median(ts)
        print(f"[{tag or 'default'}] M={N * OH * OH:>7} K={C * R * R:>5} N={K:>5} ({R}x{R}) {us:8.1f} us "
              f"{fl / us / 1e6:7.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
