"""Diagnose eager vs HIP-graph vs non-overlapped training steps on one GPU (1 RCCL rank, forced collectives).

Prints max |dw| between the variants after K steps; all should be (near) bit-equal."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["BIGDL_FORCE_COLLECTIVES"] = "1"


def main(rank, world):
    from bigdl_amd import nn
    from bigdl_amd import optim as O
    from bigdl_amd.optim.graphed import GraphedTrainStep
    from bigdl_amd.optim.train_step import TrainStep
    from tests.test_distributed_gpu import _batch, _cnn

    dev = torch.device("cuda", 0)
    X, Y = _batch(16)
    X, Y = X.to(dev), Y.to(dev)
    res = {}
    from bigdl_amd.parallel import bucketed as B

    orig_launch, orig_start = B.BucketedGradSync._launch, B.BucketedGradSync.start_gather

    def sync_launch(self, b):
        orig_launch(self, b)
        h = self.works[b]
        if h is not None:
            h.wait()
        self.works[b] = None

    orig_update = B.BucketedGradSync.update

    def waitall_update(self, loss):
        for b in list(self.works):
            h = self.works[b]
            if h is not None:
                h.wait()
            self.works[b] = None
        return orig_update(self, loss)

    from bigdl_amd.parallel import allreduce_parameter as AR
    import torch.distributed as dist

    orig_rs = AR.AllReduceParameter.reduce_scatter_range

    class _W:
        def __init__(self, ev):
            self.ev = ev

        def wait(self):
            torch.cuda.current_stream().wait_event(self.ev)

    side = {}

    def rs_sum(self, g, lo, hi, async_op=False, average=True):
        w = dist.reduce_scatter_tensor(g[lo:hi], g[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        return w, g[lo:hi]

    def rs_allreduce(self, g, lo, hi, async_op=False, average=True):
        w = dist.all_reduce(g[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        return w, g[lo:hi]

    def rs_fake(self, g, lo, hi, async_op=False, average=True):
        s = side.setdefault("s", torch.cuda.Stream())
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            g[lo:hi].mul_(1.0)
            ev = torch.cuda.Event()
            ev.record(s)
        return _W(ev), g[lo:hi]

    def sync_start(self):
        orig_start(self)
        for b in list(self.ag_works):
            self.ag_works.pop(b).wait()

    variants = [("eager_ov", True, False, 6, ""), ("eager_no", False, False, 6, ""),
                ("graph_ov", True, True, 3, ""), ("graph_no", False, True, 3, ""),
                ("graph_ov_syncrs", True, True, 3, "rs"), ("graph_ov_syncag", True, True, 3, "ag"),
                ("graph_ov_syncboth", True, True, 3, "rsag"), ("graph_ov_waitall", True, True, 3, "wa"),
                ("graph_ov1_waitall", True, True, 1, "wa"), ("graph_ov_sum", True, True, 3, "sum"),
                ("graph_ov_allreduce", True, True, 3, "allred"), ("graph_ov_fake", True, True, 3, "fake"),
                ("eager_ov_fake", True, False, 6, "fake"),
                ("eager_ov4", True, False, 4, ""), ("graph_ov1", True, True, 1, ""),
                ("eager_ov5", True, False, 5, ""), ("graph_ov2", True, True, 2, "")]
    for name, overlap, graphed, steps, mode in variants:
        B.BucketedGradSync._launch = sync_launch if "rs" in mode else orig_launch
        B.BucketedGradSync.start_gather = sync_start if "ag" in mode else orig_start
        B.BucketedGradSync.update = waitall_update if "wa" in mode else orig_update
        AR.AllReduceParameter.reduce_scatter_range = {"sum": rs_sum, "allred": rs_allreduce,
                                                      "fake": rs_fake}.get(mode, orig_rs)
        model = _cnn(True)
        step = TrainStep(model, nn.CrossEntropyCriterion(), O.SGD(0.05, momentum=0.9, dampening=0.0,
                                                                  learningRateDecay=0.01),
                         device=dev, overlap=overlap, bucket_elems=4096)
        if graphed:
            g = GraphedTrainStep(step, X, Y, warmup=2)
            for _ in range(steps):
                g.replay()
        else:
            for _ in range(steps):
                step.step(X, Y)
        step.gather_model()
        torch.cuda.synchronize()
        res[name] = (step.w[:step.total].clone().cpu(), step.w16[:step.total].float().cpu(), float(step.loss),
                     step.g[:step.total].clone().cpu())
        if overlap and name == "eager_ov":
            print(name, "buckets", step.bucketed.bounds, "units", [type(u).__name__ for u in step.bucketed.units],
                  "unit_off", step.bucketed.unit_off, "total", step.total, flush=True)
    pairs = [("eager_ov", "eager_no"), ("eager_ov", "graph_ov"), ("eager_ov", "graph_no"),
             ("eager_ov", "graph_ov_syncrs"), ("eager_ov", "graph_ov_syncag"), ("eager_ov", "graph_ov_syncboth"),
             ("eager_ov4", "graph_ov1"), ("eager_ov5", "graph_ov2"), ("eager_ov", "graph_ov_waitall"),
             ("eager_ov4", "graph_ov1_waitall"), ("eager_ov", "graph_ov_sum"), ("eager_ov", "graph_ov_allreduce"),
             ("eager_ov", "graph_ov_fake"), ("eager_ov", "eager_ov_fake")]
    for a, b in pairs:
        dw = (res[a][0] - res[b][0]).abs()
        d16 = (res[a][1] - res[b][1]).abs()
        dg = (res[a][3] - res[b][3]).abs()
        print(f"   grad diff max {dg.max():.3e} argmax {int(dg.argmax())} per-bucket "
              f"{[f'{float(dg[i:i + 4096].max()):.1e}' for i in range(0, dg.numel(), 4096)]}")
        per = [f"{float(dw[i:i + 4096].max()):.1e}" for i in range(0, dw.numel(), 4096)]
        print(f"{a:10s} vs {b:18s} max|dw| {dw.max():.3e} argmax {int(dw.argmax())} max|dw16| {d16.max():.3e} "
              f"loss {res[a][2]:.6f} {res[b][2]:.6f} per-bucket {per}", flush=True)


if __name__ == "__main__":
    from bigdl_amd.utils.testing import run_distributed

    run_distributed(main, 1, (), engine="gpu", backend="nccl", env={"BIGDL_FORCE_COLLECTIVES": "1"})
