"""Weight-gradient kernels on GEMM-shaped (1x1) problems, for timing and PMC passes:
dW[K][C] += sum_p dy[p][K] x[p][C] with P pixels, through conv2d_wgrad (kernel choice by BIGDL_WGRAD_P8)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bigdl_amd.ops import conv as cv  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="32768x4096x1024,32768x10000x1024,50176x1024x256")
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
CL, BF = torch.channels_last, torch.bfloat16
for s in a.shapes.split(","):
    P, K, C = (int(v) for v in s.split("x"))
    dy = torch.randn(P, K, 1, 1, device="cuda").to(BF)
    x = torch.randn(P, C, 1, 1, device="cuda").to(BF)
    dw = torch.zeros(K, C, 1, 1, device="cuda")
    db = torch.zeros(K, device="cuda")
    fn = lambda: cv.conv2d_wgrad(dy, x, dw, db, (1, 1), (0, 0))  # noqa: E731
    fn()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(a.iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    ms = st.elapsed_time(en) / a.iters
    print(json.dumps({"P": P, "K": K, "C": C, "p8": os.environ.get("BIGDL_WGRAD_P8", "1"), "ms": round(ms, 4),
                      "tflops": round(2.0 * P * K * C / ms / 1e9, 1)}), flush=True)
