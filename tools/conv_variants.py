"""A/B of conv kernel choices on single ResNet-50 layers, interleaved in one process (GPU).

For each selected layer (tools/bench_conv.py SHAPES index) and pass (fwd with the BN-statistics epilogue, fwd without
statistics, dgrad, dgrad with the BN-backward epilogue, wgrad), every variant (a set of runtime switches: set_conv_impl / set_conv_g4 / set_conv_p8 / set_conv_nt2)
is timed over --rounds interleaved rounds of --iters launches; the table prints the median per variant and the
output's max abs difference against the first variant (so a variant that computes something else shows).

    python tools/conv_variants.py --layers 3,4,7,13 --variants "base:;g4=4:g4=4;nt2:nt2=1"
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bench_conv import SHAPES  # noqa: E402
from bigdl_amd.ops import bn as bnops  # noqa: E402
from bigdl_amd.ops import conv as cv  # noqa: E402
from bigdl_amd.ops import native  # noqa: E402

SETTERS = {"impl": "set_conv_impl", "g4": "set_conv_g4", "p8": "set_conv_p8", "nt2": "set_conv_nt2",
           "shortk": "set_conv_shortk", "s1": "set_conv_s1", "sk": "set_conv_sk",
           "halo": "set_wgrad_halo", "chalo": "set_conv_halo"}
DEFAULTS = {"impl": 1, "g4": 3, "p8": 1, "nt2": 0, "shortk": 0, "s1": 1, "sk": 0, "halo": 1, "chalo": 1}


def parse_variants(spec):
    out = []
    for item in spec.split(";"):
        name, _, kv = item.partition(":")
        sw = dict(DEFAULTS)
        for p in filter(None, kv.split(",")):
            k, v = p.split("=")
            sw[k] = int(v)
        out.append((name, sw))
    return out


def apply(sw):
    C = native.get()
    for k, v in sw.items():
        fn = getattr(C, SETTERS[k], None)
        if fn is not None:
            fn(v)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="3,4,7,13")
    ap.add_argument("--ops", default="fwd,fwd_nostats,dgrad,dgrad_bn")
    ap.add_argument("--variants", default="base:")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    variants = parse_variants(a.variants)
    N, dev = a.batch, torch.device("cuda")
    CL, BF = torch.channels_last, torch.bfloat16
    print(f"{'#':>2} {'C':>5} {'HxW':>7} {'K':>5} {'RxS/s':>6} {'pass':>11} " +
          " ".join(f"{n:>12}" for n, _ in variants) + "   max|d| vs first", flush=True)
    for li in [int(i) for i in a.layers.split(",")]:
        C, H, K, R, st, pd, _ = SHAPES[li]
        OH = cv.out_size(H, R, st, pd)
        torch.manual_seed(li)
        x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
        w = (torch.randn(K, C, R, R, device=dev) * 0.05).to(BF, memory_format=CL)
        gy = torch.randn(N, K, OH, OH, device=dev).to(BF, memory_format=CL)
        wt = cv.transpose_w(w)
        stats = bnops.new_stats(K, dev)
        add = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
        bx = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
        bz = torch.relu(torch.randn(N, C, H, H, device=dev)).to(BF, memory_format=CL)
        red = bnops.new_stats(C, dev)
        dw = torch.zeros(K, C, R, R, device=dev).contiguous(memory_format=CL)
        bnarg = {"x": bx, "z": bz, "mean": torch.zeros(C, device=dev), "aff": None, "red": red}
        passes = {
            "fwd": lambda: cv.conv2d_fwd(x, w, None, (st, st), (pd, pd), stats=stats),
            "fwd_nostats": lambda: cv.conv2d_fwd(x, w, None, (st, st), (pd, pd)),
            "dgrad": lambda: cv.conv2d_dgrad(gy, wt, x.shape, (st, st), (pd, pd)),
            # training form: residual-gradient addend + the consumer BN's fused backward reduction (z mask)
            "dgrad_bn": lambda: cv.conv2d_dgrad(gy, wt, x.shape, (st, st), (pd, pd), addend=add, bn=dict(bnarg)),
            # weight gradient into a zeroed fp32 dW (the memset is inside the timed launches)
            "wgrad": lambda: cv.conv2d_wgrad(gy, x, dw.zero_(), None, (st, st), (pd, pd)) or dw,
        }
        for op in a.ops.split(","):
            if op.startswith("dgrad") and li == 0:
                continue
            fn = passes[op]
            times = {n: [] for n, _ in variants}
            outs = {}
            for n, sw in variants:
                apply(sw)
                outs[n] = fn().float().clone()
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for n, sw in variants:
                    apply(sw)
                    fn()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        fn()
                    e1.record()
                    e1.synchronize()
                    times[n].append(e0.elapsed_time(e1) * 1e3 / a.iters)
            apply(DEFAULTS)
            ref = outs[variants[0][0]]
            diffs = " ".join(f"{(outs[n] - ref).abs().max().item():.2e}" for n, _ in variants[1:])
            print(f"{li:>2} {C:>5} {H:>3}x{H:<3} {K:>5} {R}x{R}/{st:<2} {op:>11} " +
                  " ".join(f"{statistics.median(times[n]):>12.1f}" for n, _ in variants) + "   " + diffs, flush=True)


if __name__ == "__main__":
    main()
