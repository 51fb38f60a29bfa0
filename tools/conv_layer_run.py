"""Run ONE conv layer (fwd or dgrad) of the ResNet-50 shape table N times: a short, single-kernel program for
rocprofv3 --pmc passes (tools/bench_conv.py SHAPES index)."""
import argparse
import torch
from bigdl_amd.ops import conv as cv
from bigdl_amd.ops import bn as bnops
import sys, os
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from bench_conv import SHAPES

ap = argparse.ArgumentParser()
ap.add_argument("--idx", type=int, required=True)
ap.add_argument("--op", default="fwd")
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--batch", type=int, default=256)
a = ap.parse_args()
C, H, K, R, st, pd, _ = SHAPES[a.idx]
N = a.batch
dev = torch.device("cuda")
CL, BF = torch.channels_last, torch.bfloat16
x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
w = (torch.randn(K, C, R, R, device=dev) * 0.05).to(BF, memory_format=CL)
OH = cv.out_size(H, R, st, pd)
gy = torch.randn(N, K, OH, OH, device=dev).to(BF, memory_format=CL)
wt = cv.transpose_w(w)
stats = bnops.new_stats(K, dev)
dw = torch.zeros(K, C, R, R, device=dev).contiguous(memory_format=CL)
for _ in range(a.iters):
    if a.op == "wgrad":
        cv.conv2d_wgrad(gy, x, dw, None, (st, st), (pd, pd))
    elif a.op == "fwd":
        cv.conv2d_fwd(x, w, None, (st, st), (pd, pd), stats=stats)
    else:
        cv.conv2d_dgrad(gy, wt, x.shape, (st, st), (pd, pd))
torch.cuda.synchronize()
print("done", a.idx, a.op, (C, H, K, R, st))
