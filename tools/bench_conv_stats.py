"""Cost of the BatchNorm-statistics epilogue: conv forward with and without per-channel (sum, sumsq) accumulation
on ResNet-50 shapes (batch 256)."""
import json

import torch

from bigdl_amd.ops import conv as cv
from bigdl_amd.ops import native

CL, BF = torch.channels_last, torch.bfloat16


def t(fn, it=20):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for C, H, K, R in [(64, 56, 256, 1), (64, 56, 64, 3), (256, 56, 64, 1), (128, 28, 512, 1), (256, 14, 256, 3)]:
    x = torch.randn(256, C, H, H, device="cuda").to(BF, memory_format=CL)
    w = (torch.randn(K, C, R, R, device="cuda") * 0.05).to(BF, memory_format=CL)
    st = torch.zeros(native.get().STAT_SLOTS, 2, K, device="cuda")
    p = R // 2
    a = t(lambda: cv.conv2d_fwd(x, w, None, (1, 1), (p, p)))
    b = t(lambda: cv.conv2d_fwd(x, w, None, (1, 1), (p, p), stats=st))
    print(json.dumps({"C": C, "H": H, "K": K, "R": R, "plain_ms": round(a, 4), "stats_ms": round(b, 4)}))
