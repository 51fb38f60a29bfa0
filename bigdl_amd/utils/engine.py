"""Engine: process/device topology and runtime configuration.

Reference: S/utils/Engine.scala:41-600 (``init`` :106-119, ``parseExecutorAndCore`` :485-567 which maps
``local[N]`` → 1 node × N cores, engine type :210-216, thread pools :349-380).

MI355X-native mapping: the unit of parallelism is a *device rank* — one process per GPU, wired together
with ``torch.distributed`` over RCCL/xGMI (backend ``nccl``). ``local[N]`` therefore means N ranks on this
node (launched by torchrun), not N CPU threads. With no GPU the engine runs the fp32 CPU path and uses the
``gloo`` backend for multi-process jobs (that is how the distributed code is tested in CI).
"""
import os
import re
import threading

import torch


class EngineType:
    GPU = "gpu"        # bf16 NHWC compute on gfx950 HIP kernels (the default when a GPU is present)
    CPU = "cpu"        # fp32 torch CPU path (reference "MklBlas"-like local engine)


class _Engine:
    def __init__(self):
        self._initialized = False
        self.node_number = 1
        self.core_number = 1
        self.engine_type = None
        self.master = None
        self._lock = threading.Lock()
        self.properties = {}
        self._pg_owned = False

    # ------------------------------------------------------------------ init
    def init(self, master=None, node_number=None, core_number=None, engine_type=None, dist=None):
        """Initialise the engine.

        master: ``local[N]`` / ``local[*]`` string (Spark-master syntax, kept for API parity).
        dist: force (True/False) initialising ``torch.distributed`` from the torchrun environment.
        """
        with self._lock:
            if master is None:
                master = os.environ.get("BIGDL_MASTER", None)
            self.master = master
            world = int(os.environ.get("WORLD_SIZE", "1"))
            if master is not None:
                n, c = parse_master(master)
                self.node_number = n
                self.core_number = c if c is not None else max(world, 1)
            if node_number is not None:
                self.node_number = node_number
            if core_number is not None:
                self.core_number = core_number
            if engine_type is None:
                engine_type = os.environ.get("BIGDL_ENGINE_TYPE")
            if engine_type is None:
                engine_type = EngineType.GPU if torch.cuda.is_available() else EngineType.CPU
            self.engine_type = engine_type
            if dist is None:
                dist = world > 1
            if (engine_type == EngineType.GPU and torch.cuda.is_available()
                    and str(self.getProperty("bigdl.affinity", "1")) != "0"):
                # pin this rank's host threads to its GPU's NUMA node before any pool thread exists
                from .affinity import bind_to_gpu_numa

                try:
                    self.cpus = bind_to_gpu_numa(self.local_rank())
                except OSError:
                    self.cpus = None
            if dist:
                self._init_dist()
            self._initialized = True
        return self

    def _init_dist(self):
        import torch.distributed as td

        if td.is_initialized():
            return
        backend = "nccl" if (self.engine_type == EngineType.GPU and torch.cuda.is_available()) else "gloo"
        # test hook: BIGDL_DIST_BACKEND=gloo runs several ranks on one GPU (RCCL refuses duplicate devices)
        backend = os.environ.get("BIGDL_DIST_BACKEND", backend)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        # collective timeout (reference bigdl.network.timeout): with async error handling a rank whose peer died
        # gets an error from RCCL instead of blocking forever
        import datetime

        timeout = datetime.timedelta(seconds=float(self.getProperty("bigdl.network.timeout", 1800)))
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        kw = {"timeout": timeout}
        attempt = os.environ.get("TORCHELASTIC_RESTART_COUNT")
        if attempt is not None and "RANK" in os.environ and "WORLD_SIZE" in os.environ:
            # under torch.distributed.run: rendezvous through the launcher's store under a key prefix of this restart
            # attempt. With the default env:// rendezvous a job restarted by --max-restarts (the failure policy of
            # optim/optimizer.py) finds the previous attempt's gloo peer addresses and fails to connect (measured on
            # torch 2.10; tests/test_failure_recovery_cpu.py)
            rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
            agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "False").lower() == "true"
            base = td.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world,
                               is_master=(not agent and rank == 0), timeout=timeout)
            kw.update(store=td.PrefixStore(f"bigdl/attempt_{attempt}", base), rank=rank, world_size=world)
        if backend == "nccl":
            torch.cuda.set_device(self.local_rank())
            # RCCL keeps its default (normal-priority) streams: a raised-priority compute stream still leaves
            # normal-priority work dispatching beside it (tools/stream_prio_probe.py: 0.3 ms behind a running
            # raised-priority kernel), while raised-priority streams could share hardware queues with the compute
            # stream and serialise the bucketed reduce-scatters behind the backward
            td.init_process_group(backend, device_id=torch.device("cuda", self.local_rank()), **kw)
        else:
            td.init_process_group(backend, **kw)
        self._pg_owned = True

    def shutdown(self):
        import torch.distributed as td

        if self._pg_owned and td.is_initialized():
            td.destroy_process_group()
            self._pg_owned = False

    # ------------------------------------------------------------------ queries
    def isInitialized(self):
        return self._initialized

    def nodeNumber(self):
        return self.node_number

    def coreNumber(self):
        return self.core_number

    def getEngineType(self):
        if self.engine_type is None:
            return EngineType.GPU if torch.cuda.is_available() else EngineType.CPU
        return self.engine_type

    def setEngineType(self, t):
        self.engine_type = t

    def rank(self):
        import torch.distributed as td

        return td.get_rank() if td.is_available() and td.is_initialized() else int(os.environ.get("RANK", "0"))

    def world_size(self):
        import torch.distributed as td

        return td.get_world_size() if td.is_available() and td.is_initialized() else 1

    def local_rank(self):
        return int(os.environ.get("LOCAL_RANK", "0"))

    def device(self):
        if self.getEngineType() == EngineType.GPU and torch.cuda.is_available():
            return torch.device("cuda", self.local_rank() if torch.cuda.device_count() > 1 else 0)
        return torch.device("cpu")

    def checkSingleton(self):
        return True

    def setProperty(self, k, v):
        self.properties[k] = v
        if k == "bigdl.deterministic":
            from ..ops import native

            native.set_deterministic(str(v).lower() in ("1", "true", "yes"))
        elif k == "bigdl.module.deviceTiming":      # getTimes in device time (HIP events) for GPU modules
            from ..nn import abstractnn

            abstractnn.DEVICE_TIMING[0] = str(v).lower() in ("1", "true", "yes")

    def getProperty(self, k, default=None):
        return self.properties.get(k, os.environ.get(k, default))


def parse_master(master):
    """Reference Engine.parseExecutorAndCore (S/utils/Engine.scala:485-567).

    ``local`` → (1, 1); ``local[N]`` → (1, N); ``local[*]`` → (1, #GPUs or #CPUs);
    ``spark://…``/``yarn``/``k8s`` style masters are accepted with an explicit core count from env.
    """
    m = re.fullmatch(r"local(?:\[(\*|\d+)\])?", master.strip())
    if m:
        g = m.group(1)
        if g is None:
            return 1, 1
        if g == "*":
            n = torch.cuda.device_count() if torch.cuda.is_available() else (os.cpu_count() or 1)
            return 1, n
        return 1, int(g)
    nodes = int(os.environ.get("BIGDL_NODE_NUMBER", "1"))
    cores = os.environ.get("BIGDL_CORE_NUMBER")
    return nodes, int(cores) if cores else None


Engine = _Engine()
