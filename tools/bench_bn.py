"""Per-kernel microbenchmark of the BatchNorm streaming passes on the ResNet-50 b256 shapes (GPU).

    python tools/bench_bn.py [--batch 256] [--iters 20]

For every BN of ResNet-50 v1.5 (NHWC, P = N*H*W rows x C channels) it times the three passes the training step runs —
bn_apply (affine [+ residual] + ReLU), bn_bwd_reduce (sum dy, sum dy*(x-mean) with the ReLU mask recomputed from
x) and bn_bwd_apply (dx [+ residual-branch gradient]) — and prints, per pass, the per-step total and the achieved
HBM bandwidth (logical bytes / time). BIGDL_BN_UNROLL selects the row unroll of the kernels (A/B in one run).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bigdl_amd.ops import native  # noqa: E402


def resnet50_bn_shapes(n):
    """(P, C, count, residual) of every BN in ResNet-50 v1.5 at batch n."""
    s = [(n * 112 * 112, 64, 1, False)]
    hw = {1: 56, 2: 28, 3: 14, 4: 7}
    for stage, (blocks, w) in enumerate([(3, 64), (4, 128), (6, 256), (3, 512)], start=1):
        p = n * hw[stage] ** 2
        pin = n * hw[max(stage - 1, 1)] ** 2 if stage > 1 else p
        # first block: BN1 at the input resolution (stride on the 3x3), shortcut BN at the output
        s.append((pin, w, 1, False))
        s.append((p, w, 2 * blocks - 1, False))
        s.append((p, 4 * w, blocks, True))
        s.append((p, 4 * w, 1, False))  # projection shortcut BN
    return s


def timeit(fn, iters):
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    st.record()
    for _ in range(iters):
        fn()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    C_ = native.get()
    dev = torch.device("cuda:0")
    tot = {"apply": [0.0, 0.0], "bwd_reduce": [0.0, 0.0], "bwd_apply": [0.0, 0.0]}
    slots = C_.STAT_SLOTS
    for P, C, cnt, res in resnet50_bn_shapes(args.batch):
        x = torch.randn(P, C, device=dev).to(torch.bfloat16)
        dz = torch.randn(P, C, device=dev).to(torch.bfloat16)
        r = torch.randn(P, C, device=dev).to(torch.bfloat16) if res else None
        y = torch.empty_like(x)
        aff = torch.randn(2 * C, device=dev)
        mean = torch.randn(C, device=dev)
        inv = torch.rand(C, device=dev) + 0.5
        gamma = torch.randn(C, device=dev)
        red = torch.zeros(slots * 2 * C, device=dev)
        coef = torch.empty(3 * C, device=dev)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if res else None
        dg = torch.zeros(C, device=dev)
        db = torch.zeros(C, device=dev)
        sz = P * C * 2
        t_app = timeit(lambda: C_.bn_apply(x, aff[:C], aff[C:], r, y, P, C, True), args.iters)
        t_red = timeit(lambda: C_.bn_bwd_reduce(dz, None, x, mean, red, P, C, aff), args.iters)
        t_bwd = timeit(lambda: C_.bn_bwd_apply(dz, None, x, mean, inv, gamma, red, slots, coef, dx, dres, dg, db, P, C, aff),
                                               args.iters)
        b_app = sz * (3 if res else 2)
        b_red = sz * 2
        b_bwd = sz * (4 if res else 3)
        for k, t, b in (("apply", t_app, b_app), ("bwd_reduce", t_red, b_red), ("bwd_apply", t_bwd, b_bwd)):
            tot[k][0] += t * cnt
            tot[k][1] += b * cnt
        print(json.dumps({"P": P, "C": C, "cnt": cnt, "res": res,
                          "apply_us": round(t_app * 1e3, 1), "apply_TBs": round(b_app / t_app / 1e9, 2),
                          "red_us": round(t_red * 1e3, 1), "red_TBs": round(b_red / t_red / 1e9, 2),
                          "bwd_us": round(t_bwd * 1e3, 1), "bwd_TBs": round(b_bwd / t_bwd / 1e9, 2)}), flush=True)
        del x, dz, r, y, dx, dres
    print("TOTAL_PER_STEP", json.dumps({k: {"ms": round(v[0], 3), "TBs": round(v[1] / v[0] / 1e9, 2)}
                                        for k, v in tot.items()}), flush=True)


if __name__ == "__main__":
    main()
