"""Host placement / liveness helpers (utils/affinity.py): NUMA-local CPU lists from a fake sysfs, the per-rank
split, and the step watchdog (reference Engine.scala:569-593 thread binding, DistriOptimizer retry/timeouts)."""
import os
import time

from bigdl_amd.utils.affinity import StepWatchdog, gpu_local_cpus, parse_cpulist, rank_cpu_slice


def test_parse_cpulist():
    assert parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert parse_cpulist("") == []


def test_gpu_local_cpus_from_sysfs(tmp_path):
    d = tmp_path / "bus" / "pci" / "devices" / "0000:05:00.0"
    d.mkdir(parents=True)
    (d / "local_cpulist").write_text("0-7,64-71\n")
    assert gpu_local_cpus(bdf="0000:05:00.0", sysfs=str(tmp_path)) == list(range(8)) + list(range(64, 72))
    assert gpu_local_cpus(bdf="0000:06:00.0", sysfs=str(tmp_path)) is None


def test_rank_cpu_slice_splits_evenly():
    cpus = list(range(16))
    parts = [rank_cpu_slice(cpus, r, 4) for r in range(4)]
    assert parts == [list(range(4 * r, 4 * r + 4)) for r in range(4)]
    assert sorted(sum(parts, [])) == cpus
    assert rank_cpu_slice(list(range(5)), 1, 2) == [2, 3, 4]


def test_step_watchdog_fires_only_without_progress():
    fired = []
    wd = StepWatchdog(0.3, on_timeout=fired.append, poll=0.05).start()
    for _ in range(8):            # steady progress: never fires
        time.sleep(0.05)
        wd.kick()
    assert not fired
    time.sleep(0.6)               # stall
    assert fired and "no training step" in fired[0]
    wd.stop()


def test_optimizer_runs_with_watchdog_property():
    import torch

    from bigdl_amd import nn
    from bigdl_amd.dataset.core import DataSet, Sample
    from bigdl_amd.optim import SGD, Optimizer, Trigger
    from bigdl_amd.utils.engine import Engine

    Engine.setProperty("bigdl.step.timeout", 60)
    try:
        torch.manual_seed(0)
        x = torch.randn(32, 4)
        samples = [Sample(x[i], torch.tensor([float(i % 2 + 1)])) for i in range(32)]
        model = nn.Sequential().add(nn.Linear(4, 2)).add(nn.LogSoftMax())
        opt = Optimizer(model=model, dataset=DataSet.array(samples), criterion=nn.ClassNLLCriterion(), batchSize=8)
        opt.setOptimMethod(SGD(learningRate=0.1)).setEndWhen(Trigger.maxIteration(3))
        opt.optimize()
        assert opt.state["neval"] == 4
    finally:
        Engine.properties.pop("bigdl.step.timeout", None)
