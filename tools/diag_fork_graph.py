"""Root-cause probe for the side-stream HIP-graph discrepancy (parallel/graph_segments.py docstring).

Part 1 (pure PyTorch, no bigdl_amd code): a chain of bf16 GEMMs on the capture stream with a side-stream branch
forked in the middle and joined at the end, captured as ONE graph and replayed; compared with eager execution.
Part 2 (the training step, 1 rank, one graph, no segmentation): the bucket reduce-scatter replaced by a side-stream
branch that (A) runs no kernel, (B) scales an unrelated tensor, (C) scales the bucket's gradient range in place
(the r2 "graph_ov_fake" case), (D) like C but every branch tensor is also record_stream()'d on the side stream,
(E) B with every zero_() as a kernel instead of a memset node, (H) B but only the bucket completed last (end of
backward) forks, so no backward kernel runs beside the branch, (J) B with the compute stream waiting on an event of
its own just before the fork, (K) B forked through a second stream that runs no kernel.
Each variant vs eager after the same number of steps. Prints one line per variant."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def part1():
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    Ws = [torch.randn(1024, 1024, device=dev, generator=g).to(torch.bfloat16) * 0.03 for _ in range(16)]
    x0 = torch.randn(2048, 1024, device=dev, generator=g).to(torch.bfloat16)
    z = torch.randn(1 << 20, device=dev, generator=g)
    side = torch.cuda.Stream()

    def run(xin, zz):
        y = xin
        ev = None
        for i, W in enumerate(Ws):
            y = torch.relu(y @ W)
            if i == 4:
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    zz.mul_(1.0001)
                    ev = torch.cuda.Event()
                    ev.record(side)
        torch.cuda.current_stream().wait_event(ev)
        return y

    ref = run(x0, z.clone())
    torch.cuda.synchronize()
    xs = x0.clone()
    zs = z.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run(xs, zs)   # warm-up on the capture stream
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = run(xs, zs)
    errs = []
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        errs.append(float((out.float() - ref.float()).abs().max()))
    print(f"part1 pure-torch fork/join graph: max|out - eager| per replay {errs}", flush=True)


def part1b():
    """Pure PyTorch: the side branch joins the capture stream in the MIDDLE of the chain (the training step's
    pattern: a bucket's reduce-scatter joined in the update) and the main chain continues with kernels that read
    the main branch's results. If capturing cur.wait_event(ev_side) replaced the stream's dependency set by the
    event's nodes instead of adding them, the kernels after the join would lose their edge to the main-branch
    kernels issued between fork and join."""
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(1)
    Ws = [torch.randn(2048, 2048, device=dev, generator=g).to(torch.bfloat16) * 0.02 for _ in range(24)]
    x0 = torch.randn(4096, 2048, device=dev, generator=g).to(torch.bfloat16)
    z = torch.randn(1 << 16, device=dev, generator=g)
    side = torch.cuda.Stream()

    def run(xin, zz):
        y = xin
        ev = None
        for i, W in enumerate(Ws):
            y = torch.relu(y @ W) + 0.01
            if i == 2:
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    zz.mul_(1.0001)
                    ev = torch.cuda.Event()
                    ev.record(side)
            if i == 12:
                torch.cuda.current_stream().wait_event(ev)     # join mid-chain; GEMMs 13.. read y of GEMM 12
        return y

    ref = run(x0, z.clone())
    torch.cuda.synchronize()
    xs, zs = x0.clone(), z.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run(xs, zs)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = run(xs, zs)
    errs = []
    for _ in range(3):
        graph.replay()
        torch.cuda.synchronize()
        errs.append(float((out.float() - ref.float()).abs().max()))
    print(f"part1b pure-torch fork, mid-chain join, chain continues: max|out - eager| per replay {errs}", flush=True)


def part2(variant, steps=3):
    from tests.graph_fork_cases import part2 as _p2

    return _p2(variant, steps)


def main(rank, world, variants=()):
    if not variants:
        part1()
        part1b()
    for v in variants:
        part2(v)


if __name__ == "__main__":
    from bigdl_amd.utils.testing import run_distributed

    # python tools/diag_fork_graph.py            -> parts 1 / 1b (pure PyTorch)
    # python tools/diag_fork_graph.py A B C H    -> part 2 variants (the training step as one graph)
    run_distributed(main, 1, (tuple(sys.argv[1:]),), engine="gpu", backend="nccl",
                    env={"BIGDL_FORCE_COLLECTIVES": "1"})
