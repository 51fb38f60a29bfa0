"""Does HIP graph replay run a long-kernel branch concurrently with a short-kernel chain (truly asynchronous
branches), or does it synchronise per topological level? Main: 200 short GEMMs; side: 20 long GEMMs, each forked from
the main chain at a different point (as the per-conv weight-gradient forks of a training step), joined at the end."""
import time

import torch


def main():
    dev = torch.device("cuda")
    s = [torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16) for _ in range(3)]
    L = [torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16) for _ in range(3)]
    side = torch.cuda.Stream()

    def work(n_short, n_long, forks=True):
        cur = torch.cuda.current_stream()
        every = max(1, n_short // max(n_long, 1))
        k = 0
        for i in range(n_short):
            torch.mm(s[0], s[1], out=s[2])
            if forks and k < n_long and i % every == 0:
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    torch.mm(L[0], L[1], out=L[2])
                k += 1
        if not forks:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                for _ in range(n_long):
                    torch.mm(L[0], L[1], out=L[2])
        cur.wait_stream(side)

    def graph_of(fn):
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            fn()
        torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        return g

    def timed(fn, n=10):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    short_only = timed(graph_of(lambda: work(200, 0)).replay)
    long_only = timed(graph_of(lambda: work(0, 20, forks=False)).replay)
    interleaved = timed(graph_of(lambda: work(200, 20)).replay)
    eager = timed(lambda: work(200, 20), 5)
    print(f"graph: short chain {short_only:.3f} ms, long kernels {long_only:.3f} ms, interleaved forks "
          f"{interleaved:.3f} ms (async ~{max(short_only, long_only):.3f}); eager interleaved {eager:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
