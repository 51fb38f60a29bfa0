"""How HIP stream priorities schedule on this GPU: a 200 ms one-wave spin kernel on stream A, then a tiny kernel on
stream B; prints how long B's kernel took to complete (host wall time from its launch), for A / B priority pairs.
A B stream that has to wait for the spin is reported as ~200 ms.
    python tools/stream_prio_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bigdl_amd.ops import native  # noqa: E402


def probe(pa, pb, work_on_a=False):
    C = native.get()
    a = torch.cuda.Stream(priority=pa)
    b = torch.cuda.Stream(priority=pb)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    x = torch.zeros(1 << 20, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.stream(a):
        C.spin_us(200_000.0, flag)
        if work_on_a:                    # queued behind the spin on A (in-order)
            x.add_(1.0)
    time.sleep(0.01)
    t0 = time.perf_counter()
    with torch.cuda.stream(b):
        x.mul_(2.0)
        ev = torch.cuda.Event()
        ev.record()
    ev.synchronize()
    dt = (time.perf_counter() - t0) * 1e3
    torch.cuda.synchronize()
    return dt


def main():
    print("priority range", torch.cuda.Stream.priority_range())
    for pa, pb in ((0, 0), (-1, 0), (0, -1), (-1, -1)):
        for w in (False, True):
            print(f"A prio {pa:2d} (spin{' + queued work' if w else ''}), B prio {pb:2d}: "
                  f"B done after {probe(pa, pb, w):7.2f} ms", flush=True)


if __name__ == "__main__":
    main()
