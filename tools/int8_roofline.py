"""Per-layer int8 vs bf16 inference forward on the ResNet-50 (224x224) conv shapes at batch 256 (GPU).

For every distinct conv shape (tools/bench_conv.py SHAPES, counted as in the network) it times the int8 conv
(i8 MFMA, requantizing int8 epilogue with ReLU — what the static int8 plan runs) and the bf16 conv (bias + ReLU
epilogue), with the bytes bound of each (operands read once, result written once, at --hbm TB/s) and the
FLOP bound at the dense i8 / bf16 MFMA peaks, and prints the int8 / bf16 speedup per layer and count-weighted.

    python tools/int8_roofline.py [--batch 256] [--iters 20] [--only IDX]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import bigdl_amd  # noqa: F401,E402
from bench_conv import SHAPES  # noqa: E402
from bigdl_amd.ops import conv as cv  # noqa: E402
from bigdl_amd.ops import native  # noqa: E402
from bigdl_amd.ops.conv import _fwd_taps, out_size  # noqa: E402

PEAK_BF16, PEAK_I8 = 2.5e15, 5.0e15


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--hbm", type=float, default=8.0)
    ap.add_argument("--only", type=int, default=-1, help="time one shape index (PMC passes)")
    a = ap.parse_args()
    N, dev, hbm = a.batch, torch.device("cuda"), a.hbm * 1e12
    C_ = native.get()
    print(f"{'#':>2} {'C':>5} {'HxW':>7} {'K':>5} {'RxS/s':>6} {'cnt':>3} {'i8 us':>8} {'i8 bnd':>7} {'bf16 us':>8} "
          f"{'bf bnd':>7} {'i8/bf16':>7}", flush=True)
    tot_i8 = tot_bf = 0.0
    for si, (C, H, K, R, st, pd, cnt) in enumerate(SHAPES):
        if si == 0 or (a.only >= 0 and si != a.only):
            continue                      # the stem runs as a width-im2col int8 conv in the plan (own kernel)
        OH = out_size(H, R, st, pd)
        g = torch.Generator(device=dev).manual_seed(si)
        x8 = torch.randint(-127, 128, (N, H, H, C), device=dev, generator=g, dtype=torch.int8)
        w8 = torch.randint(-127, 128, (K, R, R, C), device=dev, generator=g, dtype=torch.int8)
        out8 = torch.empty(N * OH * OH, K, device=dev, dtype=torch.int8)
        bias = torch.zeros(K, device=dev)
        xs, ws = torch.full((N,), 1e-3, device=dev), torch.full((K,), 1e-3, device=dev)
        geo = [N, H, H, C, OH, OH, st, st, R * R * C, K, K, OH, OH, 1, 1, 0, 0]
        taps = _fwd_taps(R, R, pd, pd, 1, 1)
        i8 = lambda: C_.conv_i8(x8, w8, out8, bias, xs, ws, geo, taps, True, 1.0, 0.05, None, 1.0)  # noqa: E731
        xb = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16, memory_format=torch.channels_last)
        wb = (torch.randn(K, C, R, R, device=dev) * 0.05).to(torch.bfloat16, memory_format=torch.channels_last)
        bf = lambda: cv.conv2d_fwd(xb, wb, bias, (st, st), (pd, pd), relu=True)  # noqa: E731
        fl = 2.0 * N * OH * OH * K * C * R * R
        b8 = N * H * H * C + K * C * R * R + N * OH * OH * K
        us8, usb = timed(i8, a.iters), timed(bf, a.iters)
        bnd8 = max(fl / PEAK_I8, b8 / hbm) * 1e6
        bndb = max(fl / PEAK_BF16, 2 * b8 / hbm) * 1e6
        tot_i8 += us8 * cnt
        tot_bf += usb * cnt
        print(f"{si:2d} {C:5d} {H:3d}x{H:<3d} {K:5d} {R}x{R}/{st:<2d} {cnt:3d} {us8:8.1f} {bnd8:7.1f} {usb:8.1f} {bndb:7.1f} "
              f"{usb / us8:7.2f}", flush=True)
    print(f"# count-weighted (stem excluded): int8 {tot_i8 / 1e3:.3f} ms, bf16 {tot_bf / 1e3:.3f} ms, "
          f"speedup {tot_bf / tot_i8:.2f}x")


if __name__ == "__main__":
    main()
