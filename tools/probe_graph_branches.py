"""Do the parallel branches of a captured HIP graph run concurrently on replay? Two independent chains of small,
latency-bound GEMMs (main stream, and a side stream forked at the start and joined at the end): replay time of the
graph of each chain alone vs the graph of both (concurrent if ~max, serialized if ~sum)."""
import time

import torch


def main():
    dev = torch.device("cuda")
    x = [torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16) for _ in range(4)]
    side = torch.cuda.Stream()

    def work(n_main, n_side):
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        for _ in range(n_main):
            torch.mm(x[0], x[1], out=x[2])
        with torch.cuda.stream(side):
            for _ in range(n_side):
                torch.mm(x[1], x[0], out=x[3])
        cur.wait_stream(side)

    def graph_of(fn):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        return g

    def timed(fn, n=20):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    N = 200
    gm, gs, gb = graph_of(lambda: work(N, 0)), graph_of(lambda: work(0, N)), graph_of(lambda: work(N, N))
    tm, ts, tb = timed(gm.replay), timed(gs.replay), timed(gb.replay)
    print(f"graph replay: main chain {tm:.3f} ms, side chain {ts:.3f} ms, both {tb:.3f} ms "
          f"(concurrent ~{max(tm, ts):.3f}, serialized ~{tm + ts:.3f})", flush=True)
    te = timed(lambda: work(N, N), 5)
    print(f"eager two streams: {te:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
