"""The LSTM LM's (config 5: B 128 x T 256, hidden 1024, vocab 10000) non-recurrent GEMMs, fwd / dgrad / wgrad: the
in-tree kernels the Linear layers run (1x1-conv forms: conv_nt p8 / g4, conv_wgrad p8) against torch.matmul
(hipBLASLt) on the same bf16 problems, fp32 accumulate.
    python tools/lm_gemm_vs_blas.py   -> one line per GEMM: us and TF/s for both"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bigdl_amd  # noqa: E402,F401
from bigdl_amd.ops import conv as cv  # noqa: E402

CL, BF = torch.channels_last, torch.bfloat16


def timeit(fn, reps=10):
    for _ in range(2):
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
    M = 128 * 256
    tot = [0.0, 0.0]
    for (K, N, name) in ((1024, 10000, "vocab"), (1024, 4096, "lstm-in")):
        Np = -(-N // 8) * 8
        x = (torch.randn(M, K, device=dev) * 0.5).to(BF)
        w = (torch.randn(Np, K, device=dev) * 0.03).to(BF)
        gy = (torch.randn(M, Np, device=dev) * 0.1).to(BF)
        x4, w4, g4 = x.view(M, K, 1, 1), w.view(Np, K, 1, 1), gy.view(M, Np, 1, 1)
        wt = cv.transpose_w(w4)
        dw = torch.zeros(Np, K, 1, 1, device=dev)
        fl = 2.0 * M * K * N
        b32 = torch.randn(Np, device=dev) * 0.1
        b16 = b32.to(BF)
        dw2 = torch.zeros(Np, K, device=dev)
        cases = [
            ("fwd", lambda: cv.conv2d_fwd(x4, w4, b32, (1, 1), (0, 0)), lambda: torch.addmm(b16, x, w.t())),
            ("dgrad", lambda: cv.conv2d_dgrad(g4, wt, (M, K, 1, 1), (1, 1), (0, 0)), lambda: gy @ w),
            ("wgrad", lambda: cv.conv2d_wgrad(g4, x4, dw, None, (1, 1), (0, 0)),
             lambda: dw2.add_(torch.mm(gy.t(), x, out_dtype=torch.float32))),
        ]
        for tag, ours, blas in cases:
            t0, t1 = timeit(ours), timeit(blas)
            tot[0] += t0
            tot[1] += t1
            print(f"{name:8s} {tag:5s} M={M} K={K} N={N}: ours {t0:8.1f} us {fl / t0 / 1e6:7.1f} TF/s | "
                  f"hipBLASLt {t1:8.1f} us {fl / t1 / 1e6:7.1f} TF/s", flush=True)
    print(f"totals: ours {tot[0] / 1e3:.3f} ms, hipBLASLt {tot[1] / 1e3:.3f} ms (one LSTM layer's projections + vocab)")


if __name__ == "__main__":
    main()
