"""Multi-process test harness: run a function on N local ranks over torch.distributed gloo (CPU) — the analogue
of the reference's fake multi-node cluster in one JVM (T/optim/DistriOptimizerSpec.scala:44-46)."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, args, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    import torch.distributed as dist

    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from .engine import Engine, EngineType

        Engine.init(master=f"local[{world}]", engine_type=EngineType.CPU, dist=False)
        res = fn(rank, world, *args)
        q.put((rank, "ok", res))
    except Exception:
        q.put((rank, "err", traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_distributed(fn, world=2, args=(), timeout=300):
    """Run ``fn(rank, world, *args)`` on ``world`` gloo ranks; returns the list of per-rank results."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, status, res = q.get(timeout=timeout)
        if status != "ok":
            for p in procs:
                p.kill()
            raise RuntimeError(f"rank {rank} failed:\n{res}")
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
    return [out[r] for r in range(world)]
