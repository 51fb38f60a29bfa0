"""Straggler drop on the GPU engine, measured on the device (reference DistriOptimizer.scala:241-278 times each
replica's real compute and drops the ones past the k-th largest time, :421-449).

Two gloo ranks share cuda:0. From iteration 7 on, rank 1's GPU is slowed by a device-side spin kernel (600 ms per
iteration, launched from a layer's forward: the host is not delayed at all). The checks:
  * rank 1 is dropped in every slowed iteration (its host enqueues on time; only device-time pacing sees it);
  * rank 0's iterations stay bounded by the threshold — far below the 600 ms rank 1's device needs — so the late
    rank's exchange does not wait for its device backlog;
  * the weights equal a replay of the same drop pattern (recorded votes forced, no clocks, no spin): every update
    was the average over the ranks that finished.
"""
import pytest
import torch

from bigdl_amd.utils.testing import run_distributed

pytestmark = pytest.mark.gpu

SPIN_FROM, SPIN_US, ITERS = 7, 600_000, 14


def _job(rank, world, votes):
    import time

    from bigdl_amd import nn
    from bigdl_amd import optim as O
    from bigdl_amd.dataset.core import DataSet, Sample
    from bigdl_amd.ops import native
    from tests.test_distributed_gpu import _batch, _cnn

    it = [0]
    flag = torch.zeros(1, dtype=torch.int32, device="cuda:0")

    class Spin(nn.Identity):
        def updateOutput(self, input):
            if votes is None and rank == 1 and it[0] >= SPIN_FROM:
                native.get().spin_us(float(SPIN_US), flag)
            return super().updateOutput(input)

    model = nn.Sequential().setName("snet")
    model.add(Spin()).add(_cnn(False))
    X, Y = _batch(64)
    ds = DataSet.rdd([Sample(X[i], Y[i]) for i in range(64)], shuffle=False)
    opt = O.Optimizer(model, ds, nn.CrossEntropyCriterion(), batchSize=16,
                      optimMethod=O.SGD(0.05, momentum=0.9, dampening=0.0),
                      endTrigger=O.Trigger.maxIteration(ITERS))
    opt.setDropModuleProperty(0.25, 0.5, batchsize=3, warmupIteration=5)
    if votes is not None:
        opt._forced_votes = dict(enumerate(votes))
    walls, last = {}, [time.perf_counter()]

    def hook(n):
        now = time.perf_counter()
        walls[n] = now - last[0]
        last[0] = now
        it[0] = n

    opt._iteration_hook = hook
    m = opt.optimize()
    torch.cuda.synchronize()
    w = m.getParameters()[0][:opt._step.total].detach().float().cpu().clone()
    return walls, list(opt._drop.history), opt._drop.threshold, w


def test_slow_gpu_is_dropped_on_device_time():
    res = run_distributed(_job, 2, (None,), engine="gpu", timeout=600)
    (walls0, hist0, thr0, w0), (walls1, hist1, thr1, w1) = res
    assert len(hist0) == ITERS and len(hist1) == ITERS
    slowed = range(SPIN_FROM, ITERS)            # 0-based iterations that launched the spin on rank 1
    assert all(hist1[i] == 0.0 for i in slowed), hist1
    assert thr0 < 0.3, thr0
    late = [walls0[n] for n in range(SPIN_FROM + 2, ITERS + 1) if n in walls0]
    assert late and max(late) < min(0.3, thr0 + 0.2), (late, thr0)     # a full slowed iteration needs >= 0.6 s
    assert torch.equal(w0, w1)
    for r in _replay(hist0, hist1):
        rel = float((r - w0).norm() / w0.norm())
        assert rel < 1e-5, rel


def _replay(hist0, hist1):
    """Both ranks again with their recorded votes forced (rank r replays hist_r)."""
    out = run_distributed(_forced, 2, ([hist0, hist1],), engine="gpu", timeout=600)
    return [o[3] for o in out]


def _forced(rank, world, hists):
    return _job(rank, world, hists[rank])
