"""Localise the graph+overlap discrepancy: per-unit outputs / gradInputs / parameter gradients after the same
number of steps, eager vs HIP-graph replay (1 RCCL rank, forced collectives)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def snap(step):
    out = {}
    for i, u in enumerate(step.bucketed.units):
        o = getattr(u, "output", None)
        gi = getattr(u, "gradInput", None)
        if torch.is_tensor(o):
            out[f"u{i}.{type(u).__name__}.output"] = o.detach().float().cpu().clone()
        if torch.is_tensor(gi):
            out[f"u{i}.{type(u).__name__}.gradInput"] = gi.detach().float().cpu().clone()
        ws, gs = u.parameters() or ([], [])
        for j, gg in enumerate(gs):
            out[f"u{i}.{type(u).__name__}.grad{j}"] = gg.detach().float().cpu().clone()
    out["g"] = step.g[:step.total].clone().cpu()
    return out


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
    for name, graphed, steps in [("eager", False, 4), ("graph", True, 1), ("graph_b", True, 1)]:
        model = _cnn(True)
        step = TrainStep(model, nn.CrossEntropyCriterion(), O.SGD(0.05, momentum=0.9, dampening=0.0),
                         device=dev, overlap=True, bucket_elems=4096)
        if graphed:
            g = GraphedTrainStep(step, X, Y, warmup=2)
            for _ in range(steps):
                g.replay()
        else:
            for _ in range(steps):
                step.step(X, Y)
        torch.cuda.synchronize()
        res[name] = snap(step)
    for other in ("graph", "graph_b"):
        print("=== eager vs", other)
        for k, v in res["eager"].items():
            w = res[other][k]
            d = (v - w).abs()
            print(f"{k:45s} shape {tuple(v.shape)} max|d| {float(d.max()):.3e} frac!=0 "
                  f"{float((d > 0).float().mean()):.3f}")
    # where inside conv1's weight gradient do the errors sit?
    k = [k for k in res["eager"] if k.startswith("u0.") and k.endswith("grad0")][0]
    d = (res["eager"][k] - res["graph"][k]).abs()
    print(k, "per-out-channel max:", [f"{float(x):.1e}" for x in d.flatten(1).max(1).values])
    print(k, "per-in-channel max:", [f"{float(x):.1e}" for x in d.transpose(0, 1).flatten(1).max(1).values])


if __name__ == "__main__":
    from bigdl_amd.utils.testing import run_distributed

    run_distributed(main, 1, (), engine="gpu", backend="nccl", env={"BIGDL_FORCE_COLLECTIVES": "1"})
