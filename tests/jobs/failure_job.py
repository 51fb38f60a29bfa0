"""A 4-rank gloo training job for tests/test_failure_recovery_cpu.py, launched with torch.distributed.run.

    python -m torch.distributed.run --nproc-per-node 4 --max-restarts 1 ... failure_job.py CKPT_DIR OUT FAIL_RANK FAIL_AT

Optimizer (DistriOptimizer) over 4 ranks, checkpoint every 2 iterations, 8 iterations. On the launcher's first attempt
(TORCHELASTIC_RESTART_COUNT 0) rank FAIL_RANK raises at iteration FAIL_AT (FAIL_RANK < 0: no failure); the launcher
tears the job down and restarts every rank, which resume from the newest checkpoint through bigdl.failure.resume
(reference DistriOptimizer.scala:881-963 retries from the checkpoint; here the retry is the restarted job). Rank 0
writes the final weights to OUT (torch.save of a plain tensor)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ckpt, out, fail_rank, fail_at = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    from bigdl_amd import nn
    from bigdl_amd import optim as O
    from bigdl_amd.dataset.core import DataSet, Sample
    from bigdl_amd.utils.engine import Engine
    from bigdl_amd.utils.random_generator import RNG

    world = int(os.environ["WORLD_SIZE"])
    Engine.init(master=f"local[{world}]", dist=True)
    rank = Engine.rank()
    attempt = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
    Engine.setProperty("bigdl.failure.resume", "true")
    Engine.setProperty("bigdl.compress", "fp32")
    RNG.setSeed(7)
    model = nn.Sequential().setName("net")
    model.add(nn.Linear(6, 24).setName("fc1")).add(nn.Tanh()).add(nn.Linear(24, 3).setName("fc2"))
    g = torch.Generator().manual_seed(3)
    X, Y = torch.randn(128, 6, generator=g), torch.randn(128, 3, generator=g)
    ds = DataSet.rdd([Sample(X[i], Y[i]) for i in range(128)], shuffle=False)
    opt = O.Optimizer(model, ds, nn.MSECriterion(), batchSize=32,
                      optimMethod=O.SGD(0.05, momentum=0.9, dampening=0.0), endTrigger=O.Trigger.maxIteration(8))
    opt.setCheckpoint(ckpt, O.Trigger.severalIteration(2))

    def hook(n):
        if attempt == 0 and rank == fail_rank and n == fail_at:
            raise RuntimeError(f"injected failure on rank {rank} at iteration {n}")
    opt._iteration_hook = hook
    m = opt.optimize()
    w = m.getParameters()[0][:opt._step.total].detach().clone()
    if rank == 0:
        torch.save({"w": w, "attempt": attempt, "neval": int(opt.state["neval"])}, out)
    Engine.shutdown()


if __name__ == "__main__":
    main()
