"""Micro-benchmark of the fused LSTM step kernels (csrc/lstm.hip): per-step time of the forward / backward step
at the LM shape, with and without the recurrent GEMM, launched back to back like the sequence loop."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, n=256, reps=3):
    """Per-call device time of n back-to-back calls captured in one HIP graph (no host launch overhead)."""
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for t in range(n):
            fn(t)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for t in range(n):
            fn(t)
    g.replay()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3 / n)
    return best


def main():
    from bigdl_amd.ops import native

    C = native.get()
    B, T, H = int(os.environ.get("B", 64)), 256, int(os.environ.get("H", 1024))
    dev = "cuda"
    W16 = (torch.randn(4 * H, H, device=dev) / H ** 0.5).to(torch.bfloat16)
    WT16 = W16.t().contiguous()
    xg = torch.randn(B, T, 4 * H, device=dev)
    out = torch.empty(B, T, H, device=dev)
    cs = torch.zeros(T, B, H, device=dev)
    acts = torch.rand(T, B, 4 * H, device=dev)
    h16 = torch.zeros(2, B, H, device=dev, dtype=torch.bfloat16)
    dxg = torch.empty(B, T, 4 * H, device=dev)
    dg16 = torch.zeros(2, B, 4 * H, device=dev, dtype=torch.bfloat16)
    dc = torch.zeros(B, H, device=dev)
    dout = torch.randn(B, T, H, device=dev)

    def fwd(t=0, gemm=True):
        t = t % T
        C.lstm_fwd_step(W16, h16[t & 1] if gemm else None, xg[:, t], cs[t - 1] if t else None, cs[t], out[:, t],
                        h16[(t + 1) & 1], acts[t])

    def bwd(t=0, gemm=True):
        t = t % T
        C.lstm_bwd_step(WT16, dg16[(t + 1) & 1] if gemm else None, dout[:, t], None, acts[t],
                        cs[t - 1] if t else None, cs[t], dc, dxg[:, t], dg16[t & 1])

    empty = torch.empty(1, device=dev)
    print(f"B={B} H={H}")
    print(f"empty fill launch      {timeit(lambda t=0: empty.fill_(1.0)):7.2f} us")
    print(f"fwd step (gemm+cell)   {timeit(lambda t=0: fwd(t)):7.2f} us")
    print(f"fwd step (cell only)   {timeit(lambda t=0: fwd(t, False)):7.2f} us")
    print(f"bwd step (gemm+cell)   {timeit(lambda t=0: bwd(t)):7.2f} us")
    print(f"bwd step (cell only)   {timeit(lambda t=0: bwd(t, False)):7.2f} us")
    # same-t (no strided walk over the sequence): isolates TLB / first-touch effects of the [B, T, *] layouts
    print(f"fwd step fixed t       {timeit(lambda t=0: fwd(5)):7.2f} us")
    print(f"bwd step fixed t       {timeit(lambda t=0: bwd(5)):7.2f} us")


if __name__ == "__main__":
    main()
