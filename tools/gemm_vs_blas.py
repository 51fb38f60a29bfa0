"""ResNet-50 b256 1x1 stride-1 layers as plain GEMMs: the in-tree conv kernel (with and without the BN-statistics
epilogue) against torch.matmul (hipBLASLt) on the same [M, K] x [K, N] bf16 problem.
    python tools/gemm_vs_blas.py   -> one line per shape: M K N  ours / ours+stats / blas  (us)"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bigdl_amd  # noqa: E402,F401
from bigdl_amd.ops import bn as bnops  # noqa: E402
from bigdl_amd.ops import conv as cv  # noqa: E402

CL, BF = torch.channels_last, torch.bfloat16
# (C_in, H, C_out, count) for the stride-1 1x1 layers of ResNet-50 (fwd; dgrad swaps C_in / C_out)
LAYERS = [(64, 56, 64, 1), (64, 56, 256, 4), (256, 56, 64, 2), (256, 56, 128, 1), (128, 28, 512, 4),
          (512, 28, 128, 3), (512, 28, 256, 1), (256, 14, 1024, 6), (1024, 14, 256, 5), (1024, 14, 512, 1),
          (512, 7, 2048, 3), (2048, 7, 512, 2)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    dev = torch.device("cuda")
    N = 256
    tot = [0.0, 0.0, 0.0]
    for (C, H, K, cnt) in LAYERS:
        for (ci, co, tag) in ((C, K, "fwd"), (K, C, "dgr")):
            x = (torch.rand(N, ci, H, H, device=dev) * 2 - 1).to(BF, memory_format=CL)
            w = ((torch.rand(co, ci, 1, 1, device=dev) * 2 - 1) * 0.05).to(BF, memory_format=CL)
            st = bnops.new_stats(co, dev)
            t0 = timeit(lambda: cv.conv2d_fwd(x, w, None, (1, 1), (0, 0)))
            t1 = timeit(lambda: cv.conv2d_fwd(x, w, None, (1, 1), (0, 0), stats=st))
            a2 = x.permute(0, 2, 3, 1).reshape(-1, ci)
            b2 = w.reshape(co, ci).t()
            t2 = timeit(lambda: torch.matmul(a2, b2))
            M = N * H * H
            bytes_ = (M * ci + M * co) * 2
            print(f"{tag} M={M:>7} K={ci:>5} N={co:>5} x{cnt}: ours {t0:7.1f} +stats {t1:7.1f} blas {t2:7.1f} us"
                  f"  (HBM@6TB/s {bytes_ / 6e6:6.1f} us, MFMA@2.5PF {2.0 * M * ci * co / 2.5e9:6.1f} us)", flush=True)
            tot[0] += t0 * cnt
            tot[1] += t1 * cnt
            tot[2] += t2 * cnt
    print(f"count-weighted totals: ours {tot[0] / 1e3:.3f} ms, +stats {tot[1] / 1e3:.3f} ms, blas {tot[2] / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
