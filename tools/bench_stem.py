"""Time the training stem (7x7/2 over 3 channels, 64 outputs, batch 256 x 224 x 224) on the GPU: forward (pixel-pair
packing + implicit GEMM, the BN-statistics epilogue on), weight gradient, and the two forward formulations
(BIGDL_STEM_WINDOW=1: one 32-element overlapping window per row tap; 0: four 8-element pair taps per row tap).

    python tools/bench_stem.py [--batch 256] [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from bigdl_amd.ops import bn as bnops
    from bigdl_amd.ops import conv as cv

    dev = torch.device("cuda")
    x = torch.randn(a.batch, 3, 224, 224, device=dev)
    w16 = (torch.randn(64, 3, 7, 7, device=dev) * 0.1).to(torch.bfloat16)
    R, S, sh, ph, pw = 7, 7, 2, 3, 3
    OH, OW, S2, _, _ = cv.pair_geometry(224, 224, R, S, sh, ph, pw)
    wp = cv.pair_weight(w16)
    stats = bnops.new_stats(64, dev)
    xp = cv.to_pairs_bf16(x, R, S, sh, ph, pw)
    gy = torch.randn(a.batch, 64, OH, OW, device=dev).to(torch.bfloat16, memory_format=torch.channels_last)
    dwp = torch.zeros(64, R * S2 * 8, device=dev)
    res = {}
    res["pack_us"] = timed(lambda: cv.to_pairs_bf16(x, R, S, sh, ph, pw), a.iters)
    outs = {}
    for mode in ("1", "0"):
        os.environ["BIGDL_STEM_WINDOW"] = mode
        res[f"fwd_window{mode}_us"] = timed(lambda: cv.conv2d_pairs_fwd(xp, wp, None, 64, OH, OW, R, S2, sh,
                                                                        stats=stats), a.iters)
        outs[mode] = cv.conv2d_pairs_fwd(xp, wp, None, 64, OH, OW, R, S2, sh).float()
    os.environ["BIGDL_STEM_WINDOW"] = "1"
    res["fwd_window_vs_pairs_maxdiff"] = (outs["1"] - outs["0"]).abs().max().item()
    res["wgrad_us"] = timed(lambda: cv.conv2d_pairs_wgrad(gy, xp, R, S2, sh, dwp.zero_(), None), a.iters)
    print({k: round(v, 4) for k, v in res.items()}, flush=True)


if __name__ == "__main__":
    main()
