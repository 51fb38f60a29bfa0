"""HBM ceilings on this MI355X for the shapes of the streaming-bound ResNet-50 layers (GPU).

Times a pure write (bigdl fill_bytes kernel), a read+write copy (torch copy_) and a read-mostly reduction (torch sum)
over the byte counts of the one-K-step 1x1 convs (layer 3: 51 MB int8 in, 205 MB int8 out at batch 256), so the
per-layer roofline's "x_bound" can be read against what a trivial kernel reaches rather than the 8 TB/s peak.

    python tools/hbm_probe.py [--iters 20]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bigdl_amd.ops import native  # noqa: E402


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
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C_ = native.get()
    for mb in (51, 205, 411):
        n = mb * 2**20
        dst = torch.empty(n, dtype=torch.uint8, device="cuda")
        src = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda")
        us_w = timed(lambda: C_.fill_bytes(dst, 0), a.iters)
        us_c = timed(lambda: dst.copy_(src), a.iters)
        f = src.view(torch.float32)
        us_r = timed(lambda: f.sum(), a.iters)
        print(f"{mb:4d} MiB  write {us_w:8.1f} us {n / us_w / 1e6:6.2f} TB/s | copy {us_c:8.1f} us "
              f"{2 * n / us_c / 1e6:6.2f} TB/s (r+w) | read(sum) {us_r:8.1f} us {n / us_r / 1e6:6.2f} TB/s", flush=True)


if __name__ == "__main__":
    main()
