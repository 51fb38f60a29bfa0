"""Multi-process test harness: run a function on N local ranks over torch.distributed gloo (CPU) — the analogue
of the reference's fake multi-node cluster in one JVM (T/optim/DistriOptimizerSpec.scala:44-46)."""
import os
import pickle
import socket
import traceback

import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, args, q, engine="cpu", backend="gloo", env=None):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    os.environ.update(env or {})
    import torch.distributed as dist

    try:
        if backend == "nccl":
            import torch

            torch.cuda.set_device(0)
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        from .engine import Engine, EngineType

        Engine.init(master=f"local[{world}]", engine_type=EngineType.GPU if engine == "gpu" else EngineType.CPU,
                    dist=False)
        res = fn(rank, world, *args)
        # by value (plain pickle), not through shared-memory file descriptors that die with this process
        q.put((rank, "ok", pickle.dumps(_to_cpu(res))))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _to_cpu(v):
    import torch

    if isinstance(v, torch.Tensor):
        return v.detach().cpu().clone()
    if isinstance(v, (list, tuple)):
        return type(v)(_to_cpu(x) for x in v)
    if isinstance(v, dict):
        return {k: _to_cpu(x) for k, x in v.items()}
    return v


def run_distributed(fn, world=2, args=(), timeout=300, engine="cpu", backend="gloo", env=None):
    """Run ``fn(rank, world, *args)`` on ``world`` ranks (gloo by default; ``engine="gpu"`` puts every rank on
    cuda:0 — several ranks share the one GPU over gloo, RCCL refuses duplicate devices); returns the list of
    per-rank results."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q, engine, backend, env))
             for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, status, res = q.get(timeout=timeout)
        if status != "ok":
            for p in procs:
                p.kill()
            raise RuntimeError(f"rank {rank} failed:\n{res}")
        out[rank] = pickle.loads(res)  # noqa: S301 - produced by our own worker process
    for p in procs:
        p.join(timeout=60)
    return [out[r] for r in range(world)]
