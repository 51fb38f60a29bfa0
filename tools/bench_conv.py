"""Per-layer conv kernel benchmark on ResNet-50 shapes: bigdl_amd implicit GEMM vs MIOpen (torch)."""
import argparse, json, time
import torch
import torch.nn.functional as F
from bigdl_amd.ops import conv as cv

CL, BF = torch.channels_last, torch.bfloat16
# (C, H, K, R, stride, pad, count)  -- ResNet-50 v1.5 distinct conv shapes (224x224, count = occurrences)
SHAPES = [
    (8, 224, 64, 7, 2, 3, 1),
    (64, 56, 64, 1, 1, 0, 1), (64, 56, 64, 3, 1, 1, 3), (64, 56, 256, 1, 1, 0, 4), (256, 56, 64, 1, 1, 0, 2),
    (256, 56, 128, 1, 1, 0, 1), (128, 56, 128, 3, 2, 1, 1), (128, 28, 512, 1, 1, 0, 4), (256, 56, 512, 1, 2, 0, 1),
    (512, 28, 128, 1, 1, 0, 3), (128, 28, 128, 3, 1, 1, 3),
    (512, 28, 256, 1, 1, 0, 1), (256, 28, 256, 3, 2, 1, 1), (256, 14, 1024, 1, 1, 0, 6), (512, 28, 1024, 1, 2, 0, 1),
    (1024, 14, 256, 1, 1, 0, 5), (256, 14, 256, 3, 1, 1, 5),
    (1024, 14, 512, 1, 1, 0, 1), (512, 14, 512, 3, 2, 1, 1), (512, 7, 2048, 1, 1, 0, 3), (1024, 14, 2048, 1, 2, 0, 1),
    (2048, 7, 512, 1, 1, 0, 2), (512, 7, 512, 3, 1, 1, 2),
]


def timeit(fn, iters=10):
    fn(); torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", type=str, default="", help="comma-separated shape indices")
    ap.add_argument("--no-miopen", action="store_true")
    ap.add_argument("--ops", type=str, default="fwd,dgrad,wgrad")
    args = ap.parse_args()
    only = {int(i) for i in args.only.split(",") if i}
    ops = set(args.ops.split(","))
    N = args.batch
    dev = torch.device("cuda")
    tot = {"ours_fwd": 0, "ours_dgrad": 0, "ours_wgrad": 0, "miopen_fwd": 0, "miopen_dgrad": 0, "miopen_wgrad": 0}
    flops_total = 0
    rows = []
    for si, (C, H, K, R, st, pd, cnt) in enumerate(SHAPES):
        if only and si not in only:
            continue
        x = torch.randn(N, C, H, H, device=dev).to(BF, memory_format=CL)
        w = (torch.randn(K, C, R, R, device=dev) * 0.05).to(BF, memory_format=CL)
        b = torch.zeros(K, device=dev)
        OH = cv.out_size(H, R, st, pd)
        gy = torch.randn(N, K, OH, OH, device=dev).to(BF, memory_format=CL)
        wt = cv.transpose_w(w)
        dw = torch.zeros(K, C, R, R, device=dev).contiguous(memory_format=CL)
        db = torch.zeros(K, device=dev)
        fl = 2.0 * N * OH * OH * K * C * R * R
        nan = float("nan")
        t_f = timeit(lambda: cv.conv2d_fwd(x, w, b, (st, st), (pd, pd)), args.iters) if "fwd" in ops else nan
        t_d = timeit(lambda: cv.conv2d_dgrad(gy, wt, x.shape, (st, st), (pd, pd)), args.iters) if "dgrad" in ops else nan
        t_w = timeit(lambda: (dw.zero_(), cv.conv2d_wgrad(gy, x, dw, db, (st, st), (pd, pd))), args.iters) \
            if "wgrad" in ops else nan
        if args.no_miopen:
            m_f = m_d = m_w = nan
        else:
          m_f = timeit(lambda: F.conv2d(x, w, None, st, pd), args.iters)
          m_d = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, (st, st), (pd, pd), (1, 1), False, (0, 0), 1, (True, False, False)), args.iters)
          m_w = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, (st, st), (pd, pd), (1, 1), False, (0, 0), 1, (False, True, False)), args.iters)
        row = dict(C=C, H=H, K=K, R=R, s=st, cnt=cnt, fwd_ms=round(t_f, 3), dgrad_ms=round(t_d, 3), wgrad_ms=round(t_w, 3),
                   miopen_fwd=round(m_f, 3), miopen_dgrad=round(m_d, 3), miopen_wgrad=round(m_w, 3),
                   fwd_tflops=round(fl / t_f / 1e9, 1), dgrad_tflops=round(fl / t_d / 1e9, 1), wgrad_tflops=round(fl / t_w / 1e9, 1))
        rows.append(row)
        print(json.dumps(row), flush=True)
        for k, v in (("ours_fwd", t_f), ("ours_dgrad", t_d), ("ours_wgrad", t_w), ("miopen_fwd", m_f), ("miopen_dgrad", m_d), ("miopen_wgrad", m_w)):
            tot[k] += v * cnt
        flops_total += fl * cnt
    tot = {k: round(v, 2) for k, v in tot.items()}
    tot["conv_fwd_gflop"] = round(flops_total / 1e9, 1)
    print("TOTAL_MS", json.dumps(tot))


if __name__ == "__main__":
    main()
