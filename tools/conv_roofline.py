"""Per-layer roofline of the ResNet-50 (224x224) convolutions at batch 256 on one MI355X.

For every distinct conv shape (tools/bench_conv.py SHAPES, with its count in the network) and every pass — fwd (with
the conv bias and the BN-statistics epilogue, as in training), dgrad, wgrad (fp32 weight gradient + bias gradient incl.
any split reduce) — through the paths the training step takes (the stem as the pixel-pair view from the fp32 image,
ops/conv.py conv2d_pairs_*; the data gradients without the fused consumer-BN epilogue) — it prints
FLOPs, the minimum HBM bytes (every operand read once, the result written once), the measured device time (CUDA
events, median of --iters launches), the bound max(FLOP / 2.5 PF, bytes / 8 TB/s) and measured / bound. Totals are
weighted by the layer counts. ``--hbm`` prices bytes at another bandwidth (6.3 TB/s = the measured copy rate).

    python tools/conv_roofline.py [--batch 256] [--iters 20] [--json out.jsonl]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import bigdl_amd  # noqa: F401,E402
from bench_conv import SHAPES  # noqa: E402
from bigdl_amd.ops import bn as bnops  # noqa: E402
from bigdl_amd.ops import conv as cv  # noqa: E402

PEAK = 2.5e15


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
    ap.add_argument("--hbm", type=float, default=8.0, help="TB/s used for the byte bound")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    N, dev = a.batch, torch.device("cuda")
    CL, BF = torch.channels_last, torch.bfloat16
    hbm = a.hbm * 1e12
    rows = []
    hdr = (f"{'#':>2} {'C':>5} {'HxW':>7} {'K':>5} {'RxS/s':>6} {'cnt':>3} {'pass':>5} {'GFLOP':>7} {'MB':>7} "
           f"{'us':>8} {'bound_us':>8} {'x_bound':>7} {'TF/s':>6} {'TB/s':>5}")
    print(hdr, flush=True)
    tot = {"fwd": [0.0, 0.0], "dgrad": [0.0, 0.0], "wgrad": [0.0, 0.0]}
    for si, (C, H, K, R, st, pd, cnt) in enumerate(SHAPES):
        OH = cv.out_size(H, R, st, pd)
        x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
        w = (torch.randn(K, C, R, R, device=dev) * 0.05).to(BF, memory_format=CL)
        gy = torch.randn(N, K, OH, OH, device=dev).to(BF, memory_format=CL)
        wt = cv.transpose_w(w)
        dw = torch.zeros(K, C, R, R, device=dev).contiguous(memory_format=CL)
        db = torch.zeros(K, device=dev)
        stats = bnops.new_stats(K, dev)
        bias = torch.zeros(K, device=dev)
        fl = 2.0 * N * OH * OH * K * C * R * R
        bx, bw, by = N * H * H * C * 2, K * C * R * R * 2, N * OH * OH * K * 2
        passes = {
            "fwd": (lambda: cv.conv2d_fwd(x, w, bias, (st, st), (pd, pd), stats=stats), bx + bw + by),
            "dgrad": (lambda: cv.conv2d_dgrad(gy, wt, x.shape, (st, st), (pd, pd)), by + bw + bx),
            "wgrad": (lambda: cv.conv2d_wgrad(gy, x, dw, db, (st, st), (pd, pd)), by + bx + K * C * R * R * 4),
        }
        if si == 0:
            # the stem as the step runs it: 3-channel fp32 image -> pixel-pair view (8 channels per 2 columns), the
            # pair-view kernels for fwd / wgrad; its input gradient is never computed
            img = torch.randn(N, 3, H, H, device=dev)
            OHp, OWp, S2, _, _ = cv.pair_geometry(H, H, R, R, st, pd, pd)
            xp = cv.to_pairs_bf16(img, R, R, st, pd, pd)
            wp = cv.pair_weight((torch.randn(K, 3, R, R, device=dev) * 0.05).to(BF, memory_format=CL))
            dwp = torch.zeros(K, R * S2 * 8, device=dev)
            fl = 2.0 * N * OH * OH * K * 3 * R * R
            bx = N * H * H * 3 * 4
            passes = {
                "fwd": (lambda: cv.conv2d_pairs_fwd(xp, wp, bias, K, OHp, OWp, R, S2, st, stats=stats),
                        bx + bw + by),
                "wgrad": (lambda: cv.conv2d_pairs_wgrad(gy, xp, R, S2, st, dwp, db), by + bx + K * 3 * R * R * 4),
            }
        for name, (fn, byt) in passes.items():
            us = timed(fn, a.iters)
            bound = max(fl / PEAK, byt / hbm) * 1e6
            r = dict(idx=si, C=C, H=H, K=K, R=R, stride=st, count=cnt, op=name, gflop=round(fl / 1e9, 2),
                     mbytes=round(byt / 1e6, 1), us=round(us, 1), bound_us=round(bound, 1),
                     x_bound=round(us / bound, 2), tflops=round(fl / us / 1e6, 1), tbps=round(byt / us / 1e6, 2))
            rows.append(r)
            tot[name][0] += us * cnt
            tot[name][1] += bound * cnt
            print(f"{si:>2} {C:>5} {H:>3}x{H:<3} {K:>5} {R}x{R}/{st:<2} {cnt:>3} {name:>5} {r['gflop']:>7} "
                  f"{r['mbytes']:>7} {r['us']:>8} {r['bound_us']:>8} {r['x_bound']:>7} {r['tflops']:>6} "
                  f"{r['tbps']:>5}", flush=True)
    print("# totals over the network (count-weighted): measured ms / bound ms / ratio")
    for k, (m, b) in tot.items():
        print(f"# {k:>5}: {m / 1e3:7.3f} ms  bound {b / 1e3:7.3f} ms  x{m / b:5.2f}")
    m_all, b_all = sum(v[0] for v in tot.values()), sum(v[1] for v in tot.values())
    print(f"#   all: {m_all / 1e3:7.3f} ms  bound {b_all / 1e3:7.3f} ms  x{m_all / b_all:5.2f}")
    if a.json:
        with open(a.json, "w") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
