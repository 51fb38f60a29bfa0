"""Host-side placement and liveness for one-process-per-GPU jobs.

Reference: S/utils/Engine.scala:569-593 (binding the MKL / computing threads to cores) and
S/utils/DistriParameterSynchronizer.scala:128-144 (dedicated, pinned communication threads), plus the
``retryTimes`` / per-task timeouts of S/optim/DistriOptimizer.scala:881-963 that keep a stuck task from hanging
the job.

MI355X mapping:
  * ``bind_to_gpu_numa(local_rank)``: a rank's host threads (data loader pool, C++ batch assembler, the Python
    main thread that launches kernels and RCCL calls) are pinned to the CPU cores of the NUMA node its GPU hangs
    off — read from sysfs (``/sys/bus/pci/devices/<bdf>/local_cpulist``) — and split evenly among the ranks that
    share that node, so launches and host<->device copies never cross the socket interconnect.
  * ``StepWatchdog``: a daemon thread that the training loop ``kick()``s every step; when no step completes for
    ``timeout`` seconds (a rank stuck in a collective whose peer died, a hung kernel) it dumps every thread's
    stack and exits the process with a non-zero code, so the launcher (torchrun) tears the job down and a
    restart policy can resume from the last checkpoint instead of the job hanging forever. RCCL's own
    collective timeout (``init_process_group(timeout=...)`` with async error handling) covers the same failure
    from the communicator side.
"""
import faulthandler
import logging
import os
import sys
import threading
import time

logger = logging.getLogger("bigdl_amd.affinity")

SYSFS = "/sys"


def parse_cpulist(s):
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out = []
    for part in s.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def _pci_bdf(device_index):
    """PCI address 'dddd:bb:dd.f' of a visible GPU, or None."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device_index)
        dom = getattr(p, "pci_domain_id", 0)
        bus, dev = getattr(p, "pci_bus_id", None), getattr(p, "pci_device_id", None)
        if bus is None or dev is None:
            return None
        return f"{dom:04x}:{bus:02x}:{dev:02x}.0"
    except Exception:
        return None


def gpu_local_cpus(device_index=None, bdf=None, sysfs=None):
    """CPU ids local to the GPU's NUMA node (from sysfs), or None when unknown."""
    root = sysfs or SYSFS
    bdf = bdf or (_pci_bdf(device_index) if device_index is not None else None)
    if bdf is None:
        return None
    path = os.path.join(root, "bus", "pci", "devices", bdf, "local_cpulist")
    try:
        with open(path) as f:
            cpus = parse_cpulist(f.read())
    except OSError:
        return None
    return cpus or None


def rank_cpu_slice(cpus, local_rank, ranks_on_node):
    """The share of ``cpus`` for the ``local_rank``-th of ``ranks_on_node`` ranks that share one NUMA node."""
    if not cpus:
        return []
    n = max(1, ranks_on_node)
    k = local_rank % n
    per = max(1, len(cpus) // n)
    part = cpus[k * per:(k + 1) * per] if k < n - 1 else cpus[k * per:]
    return part or cpus


def bind_to_gpu_numa(local_rank, device_index=None, local_world=None, sysfs=None):
    """Pin this process to the CPUs of its GPU's NUMA node (shared evenly with the node's other ranks).
    Returns the CPU list applied, or None when the topology is unknown or pinning is unavailable."""
    if not hasattr(os, "sched_setaffinity"):
        return None
    dev = local_rank if device_index is None else device_index
    cpus = gpu_local_cpus(dev, sysfs=sysfs)
    if not cpus:
        return None
    allowed = set(os.sched_getaffinity(0))
    cpus = [c for c in cpus if c in allowed]
    if not cpus:
        return None
    local_world = local_world or int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    # ranks whose GPUs share this NUMA node (same local_cpulist) split its cores
    same = [r for r in range(local_world) if gpu_local_cpus(r, sysfs=sysfs) == gpu_local_cpus(dev, sysfs=sysfs)]
    idx = same.index(local_rank) if local_rank in same else 0
    mine = rank_cpu_slice(cpus, idx, len(same) or 1)
    os.sched_setaffinity(0, mine)
    logger.info("rank %d bound to CPUs %s (GPU %d NUMA-local)", local_rank, mine, dev)
    return mine


class StepWatchdog:
    """Abort a stuck rank: ``kick()`` once per completed step; after ``timeout`` seconds without one, dump all
    thread stacks to stderr and ``os._exit(exit_code)`` (or call ``on_timeout`` instead, for tests)."""

    def __init__(self, timeout, on_timeout=None, exit_code=75, poll=None):
        self.timeout = float(timeout)
        self.on_timeout = on_timeout
        self.exit_code = exit_code
        self.poll = poll if poll is not None else min(5.0, max(0.05, self.timeout / 10))
        self._last = time.monotonic()
        self._stop = threading.Event()
        self._fired = False
        self._t = threading.Thread(target=self._run, name="bigdl-step-watchdog", daemon=True)

    def start(self):
        self._last = time.monotonic()
        self._t.start()
        return self

    def kick(self):
        self._last = time.monotonic()

    def stop(self):
        self._stop.set()
        if self._t.is_alive():
            self._t.join(timeout=self.poll * 2 + 1)

    @property
    def fired(self):
        return self._fired

    def _run(self):
        while not self._stop.wait(self.poll):
            idle = time.monotonic() - self._last
            if idle > self.timeout:
                self._fired = True
                msg = f"[bigdl watchdog] no training step completed for {idle:.0f}s (limit {self.timeout:.0f}s)"
                if self.on_timeout is not None:
                    self.on_timeout(msg)
                    return
                print(msg + "; dumping stacks and exiting", file=sys.stderr, flush=True)
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
                os._exit(self.exit_code)


__all__ = ["parse_cpulist", "gpu_local_cpus", "rank_cpu_slice", "bind_to_gpu_numa", "StepWatchdog"]
