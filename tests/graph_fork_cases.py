"""Forked-branch HIP-graph cases shared by tests/test_distributed_gpu.py and tools/diag_fork_graph.py.

``part2(variant)``: the training step (1 rank, forced collectives) captured as ONE graph (no segmentation) with the
bucket reduce-scatter replaced by a side-stream branch that (A) runs no kernel, (B) scales an unrelated tensor, (C)
scales the bucket's gradient range in place, (D) like C with record_stream, (E) B with every zero_() as a kernel, (H) B
but only the bucket completed last forks, (J) B with the compute stream first waiting on its own event, (K) B forked
through a kernel-less hop stream. Returns max |w_graph - w_eager| after the same number of steps.
"""
import torch


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
