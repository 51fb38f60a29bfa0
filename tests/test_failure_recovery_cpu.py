"""Multi-rank failure recovery (reference DistriOptimizer.scala:881-963 retry-from-checkpoint, tested there with an
injected ExceptionTest layer, T/optim/DistriOptimizerSpec.scala:588-656): a 4-rank gloo job under
``torch.distributed.run --max-restarts 1`` where one rank raises at iteration 5. The launcher restarts the job, every
rank resumes from the iteration-4 checkpoint through ``bigdl.failure.resume``, and the final weights equal those of an
uninterrupted run."""
import os
import socket
import subprocess
import sys

import torch

JOB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "jobs", "failure_job.py")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp, tag, fail_rank, fail_at, restarts):
    ckpt = os.path.join(tmp, f"ckpt_{tag}")
    os.makedirs(ckpt)
    out = os.path.join(tmp, f"w_{tag}.pt")
    env = {k: v for k, v in os.environ.items()            # a clean launcher environment: no rendezvous left over
           if k not in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")
           and not k.startswith("TORCHELASTIC")}
    env.update(OMP_NUM_THREADS="1", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
           f"--max-restarts={restarts}", "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           JOB, ckpt, out, str(fail_rank), str(fail_at)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
    return p, out, ckpt


def test_rank_failure_restarts_and_resumes_to_the_same_weights(tmp_path):
    straight, out_s, _ = _run(str(tmp_path), "straight", -1, 0, 0)
    assert straight.returncode == 0, straight.stderr[-3000:]
    failed, out_f, ckpt_f = _run(str(tmp_path), "failed", 2, 5, 1)
    assert failed.returncode == 0, failed.stderr[-3000:]
    assert "injected failure on rank 2 at iteration 5" in failed.stderr + failed.stdout
    s = torch.load(out_s, weights_only=True)
    f = torch.load(out_f, weights_only=True)
    assert s["attempt"] == 0 and f["attempt"] == 1          # the second run finished on the launcher's restart
    assert s["neval"] == f["neval"] == 9
    assert "model.4" in os.listdir(ckpt_f)                  # the restart resumed from this snapshot
    assert torch.allclose(f["w"], s["w"], atol=1e-6), (f["w"] - s["w"]).abs().max()


def test_failure_without_restart_budget_fails_the_job(tmp_path):
    """No restart left: the injected error ends the job with a non-zero status (no silent partial training)."""
    p, out, _ = _run(str(tmp_path), "norestart", 1, 3, 0)
    assert p.returncode != 0
    assert not os.path.exists(out)
