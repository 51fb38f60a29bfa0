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
    from bigdl_amd import nn
    from bigdl_amd import optim as O
    from bigdl_amd.optim.graphed import GraphedTrainStep
    from bigdl_amd.optim.train_step import TrainStep
    from bigdl_amd.parallel import allreduce_parameter as AR
    from bigdl_amd.parallel import graph_segments as GS
    from tests.test_distributed_gpu import _batch, _cnn

    dev = torch.device("cuda", 0)
    X, Y = _batch(16)
    X, Y = X.to(dev), Y.to(dev)
    side = torch.cuda.Stream()
    hop = torch.cuda.Stream()
    other = torch.zeros(1 << 16, device=dev)

    class _W:
        def __init__(self, ev):
            self.ev = ev

        def wait(self):
            torch.cuda.current_stream().wait_event(self.ev)

    def rs_side(self, g, lo, hi, async_op=False, average=True):
        if variant == "H" and lo != 0:     # H: only the bucket finished LAST (at the end of backward) forks
            return None, g[lo:hi]
        if variant == "J":      # B, with the compute stream first waiting on an event it recorded itself
            ev0 = torch.cuda.Event()
            ev0.record()
            torch.cuda.current_stream().wait_event(ev0)
        if variant == "K":      # B, forked through a second side stream that runs no kernel
            hop.wait_stream(torch.cuda.current_stream())
            side.wait_stream(hop)
        else:
            side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            if variant in ("B", "E", "H", "J", "K"):
                other.mul_(1.0)
            elif variant in ("C", "D"):
                g[lo:hi].mul_(1.0)
                if variant == "D":
                    g.record_stream(side)
            ev = torch.cuda.Event()
            ev.record(side)
        return _W(ev), g[lo:hi]

    def ag_none(self, w, w16, lo, hi, async_op=False):
        return None

    orig_rs, orig_ag, orig_boundary = (AR.AllReduceParameter.reduce_scatter_range,
                                       AR.AllReduceParameter.all_gather_range, GS.SegmentedGraph.boundary)
    orig_zero = torch.Tensor.zero_
    res = {}
    if variant == "E":      # side kernel as B, every zero_() as a kernel (bitwise and 0) instead of a memset node
        def kzero(t):
            if t.is_cuda and t.is_floating_point():
                t.mul_(0.0)
                t.nan_to_num_(0.0, 0.0, 0.0)
                return t
            return orig_zero(t)
        torch.Tensor.zero_ = kzero
    try:
        AR.AllReduceParameter.reduce_scatter_range = rs_side
        AR.AllReduceParameter.all_gather_range = ag_none
        GS.SegmentedGraph.boundary = lambda self, fn: fn()          # ONE graph: no segmentation
        for name, graphed in (("eager", False), ("graph", True)):
            model = _cnn(True)
            step = TrainStep(model, nn.CrossEntropyCriterion(), O.SGD(0.05, momentum=0.9, dampening=0.0),
                             device=dev, overlap=True, bucket_elems=4096)
            if graphed:
                gs = GraphedTrainStep(step, X, Y, warmup=2)
                for _ in range(steps):
                    gs.replay()
            else:
                for _ in range(2 + 1 + steps):     # GraphedTrainStep runs warmup 2 + 1 eager step first
                    step.step(X, Y)
            torch.cuda.synchronize()
            res[name] = step.w[:step.total].clone().cpu()
    finally:
        torch.Tensor.zero_ = orig_zero
        AR.AllReduceParameter.reduce_scatter_range = orig_rs
        AR.AllReduceParameter.all_gather_range = orig_ag
        GS.SegmentedGraph.boundary = orig_boundary
    d = (res["eager"] - res["graph"]).abs()
    print(f"part2 variant {variant}: max|w_graph - w_eager| {float(d.max()):.3e} "
          f"(frac != 0: {float((d > 0).float().mean()):.4f})", flush=True)
    return float(d.max())


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
