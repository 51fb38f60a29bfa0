"""Headline benchmark: ResNet-50 (224x224, bf16) synchronous data-parallel training throughput.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One process per GPU over RCCL (torch.distributed backend "nccl"). Each timed step is a full
DistriOptimizer iteration of the framework: forward + CrossEntropy + backward through the BigDL module
protocol on the native gfx950 kernels, reduce-scatter of gradients (ZeRO-1 shard), fused SGD(momentum,
folded L2 regularizers) on the shard, all-gather of bf16 weights. Batch 256 per GPU (weak scaling),
synthetic ImageNet-shaped data and random-init weights (no datasets / checkpoints are available offline).
Rank 0 prints ONE JSON line; value = whole-job images/sec; the time is the MAX over ranks.
"""
import argparse
import json
import os
import sys
import time

import torch

import bigdl_amd  # noqa: F401,E402  (HIP runtime graph settings must precede the first GPU call)

METRIC = "images/sec (whole node) ResNet-50 224x224 bf16 at 1/2/4/8 MI355X"
BASELINE = None  # BASELINE.json "published" is empty: no reference number on this metric


def dist_backend():
    import torch.distributed as dist

    if not dist.is_initialized():
        return "none"
    b = dist.get_backend()
    return "RCCL" if b == "nccl" else b


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--compress", default="auto", choices=["auto", "bf16", "fp16", "fp32"],
                    help="gradient / weight wire format: auto (default) = bf16 whenever N > 1, the reference's 16-bit "
                         "exchange; fp16 = the reference's truncating FP16CompressedTensor; fp32 = uncompressed")
    ap.add_argument("--graph", type=int, default=-1,
                    help="1: capture the training step in HIP graphs, 0: eager launches, -1 (default): time both "
                         "during warm-up and keep the faster")
    ap.add_argument("--bucket", type=int, default=8, help="gradient bucket size, M elements (N > 1)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--graph-model", action="store_true",
                    help="build the Graph-form ResNet (ResNet.graph: nn.Graph over nodes) instead of the Sequential "
                         "one; training fusion is planned on the graph's edges")
    ap.add_argument("--via-optimizer", action="store_true",
                    help="drive the step through the user-facing Optimizer(...).optimize() loop (host batches fed "
                         "through its pinned double-buffered H2D feed, iteration captured in HIP graphs)")
    return ap.parse_args()


def _via_optimizer(args, model, crit, optim, dev, world, rank):
    """Time W + K iterations of Optimizer.optimize() on a synthetic host-side DataSet of ImageNet-shaped batches;
    returns the seconds of the last K iterations (synchronised and barriered on both sides)."""
    import torch.distributed as dist

    from bigdl_amd.dataset.core import LocalDataSet, MiniBatch
    from bigdl_amd.optim.optimizer import Optimizer
    from bigdl_amd.optim.trigger import Trigger

    B = args.batch
    g = torch.Generator().manual_seed(rank)
    host = [MiniBatch(torch.randn(B, 3, args.image, args.image, generator=g).pin_memory(),
                      torch.randint(1, 1001, (B,), generator=g).float().pin_memory()) for _ in range(2)]

    class Synthetic(LocalDataSet):
        def data(self, train=True):
            i = 0
            while True:
                yield host[i & 1]
                i += 1

        def size(self):
            return B * world * 10000

    W, K = max(args.warmup, 9), args.steps     # 2 eager + capture + 3 replays decide graph-or-eager, 3 more re-warm
    marks = {}

    def hook(neval):
        if neval in (W, W + K):
            from bigdl_amd.optim.train_step import wait_event

            end = torch.cuda.Event()
            end.record()
            wait_event(end)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            marks[neval] = time.perf_counter()

    opt = Optimizer(model, Synthetic(), crit, batchSize=None, optimMethod=optim,
                    endTrigger=Trigger.maxIteration(W + K))
    opt.device = dev
    opt._iteration_hook = hook
    opt.optimize()
    return marks[W + K] - marks[W], opt


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus > 1 and world == 1:
        print("bench.py: --gpus > 1 requires torch.distributed.run (one process per GPU)", file=sys.stderr)
        sys.exit(2)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    local = local % max(1, torch.cuda.device_count())   # ranks > devices only in single-GPU rehearsals
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from bigdl_amd.utils.engine import Engine

    # BIGDL_FORCE_COLLECTIVES=1 (under torch.distributed.run) runs the full multi-GPU step on one rank: RCCL
    # reduce-scatter / all-gather, bucketed overlap and the segmented HIP graph, to price their overhead
    force = os.environ.get("BIGDL_FORCE_COLLECTIVES") == "1" and "MASTER_PORT" in os.environ
    Engine.init(master=f"local[{world}]", dist=world > 1 or force)

    from bigdl_amd import nn
    from bigdl_amd.models.resnet import DatasetType, ResNet, ResNetGraph
    from bigdl_amd.ops import side_stream
    from bigdl_amd.optim.sgd import SGD
    from bigdl_amd.optim.train_step import TrainStep, wait_event
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(1234 + rank)
    model = (ResNetGraph if args.graph_model else ResNet)(1000, args.depth, dataSet=DatasetType.ImageNet)
    crit = nn.CrossEntropyCriterion()
    optim = SGD(learningRate=0.1, momentum=0.9, dampening=0.0)
    step = None
    if not args.via_optimizer:
        step = TrainStep(model, crit, optim, device=dev, compress=args.compress, bucket_elems=args.bucket << 20)

    B = args.batch
    if args.via_optimizer:
        dt, opt = _via_optimizer(args, model, crit, optim, dev, world, rank)
        t = torch.tensor([dt], device=dev)
        if world > 1:
            import torch.distributed as dist

            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        ms = dt / args.steps * 1e3
        if rank == 0:
            print(json.dumps({
                "metric": METRIC, "value": round(B * world * args.steps / dt, 2), "unit": "images/sec",
                "n_gpus": world, "steps": args.steps, "warmup": max(args.warmup, 9), "ms_per_step": round(ms, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
                "data": "synthetic host batches (random 3x224x224 fp32, pinned) through Optimizer.optimize()",
                "config": {"model": f"ResNet-{args.depth} v1.5 (BigDL ImageNet builder{', Graph form' if args.graph_model else ''})", "global_batch": B * world,
                           "per_gpu_batch": B, "seq_len": None, "image": args.image, "parallelism": f"dp{world}",
                           "driver": "Optimizer.optimize()", "hip_graph": opt._graph is not None,
                           "graph_vs_eager": getattr(opt, "graph_decision", None),
                           "loss": float(opt.state.get("Loss", float("nan")))},
            }), flush=True)
        Engine.shutdown()
        return
    g = torch.Generator(device=dev)
    g.manual_seed(rank)
    x = torch.randn(B, 3, args.image, args.image, device=dev, generator=g)
    y = torch.randint(1, 1001, (B,), device=dev, generator=g).float()

    def barrier():
        if world > 1:
            import torch.distributed as dist

            dist.barrier()

    run = lambda: step.step(x, y)  # noqa: E731
    graph = None
    decision = None
    mode = args.graph            # 1 graph, 0 eager, -1 auto: time both during warm-up, keep the faster
    if mode and (world > 1 or force):
        import torch.distributed as dist

        if dist.get_backend() != "nccl":
            # gloo collectives (single-GPU multi-rank rehearsal) run on the host: nothing to capture
            print("[bench] non-RCCL backend: eager launches", file=sys.stderr)
            mode = 0
    for _ in range(max(args.warmup, 2)):
        run()

    def timed(fn, n=2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / n

    if mode:
        from bigdl_amd.optim.graphed import GraphedTrainStep

        eager_ms = timed(run) if mode < 0 else None
        host_ms = None
        if mode < 0:       # host cost of enqueueing one iteration (right after a sync: no throttle wait)
            torch.cuda.synchronize()
            h0 = time.perf_counter()
            run()
            host_ms = (time.perf_counter() - h0) * 1e3
            torch.cuda.synchronize()
        try:
            graph = GraphedTrainStep(step, x, y, prewarmed=True)
            graph.replay()
            graph_ms = timed(graph.replay)
            run = graph.replay  # noqa: F811
        except Exception as e:  # fall back to eager launches
            print(f"[bench] HIP graph capture failed ({type(e).__name__}: {e}); running eager", file=sys.stderr)
            side_stream.reset()
            graph = None
        if mode < 0 and graph is not None:
            t = torch.tensor([eager_ms, graph_ms, host_ms], device=dev)
            if world > 1:
                import torch.distributed as dist

                dist.all_reduce(t)
            eager_ms, graph_ms, host_ms = (float(v) / world for v in t.cpu())
            decision = {"eager_ms": round(eager_ms, 3), "graph_ms": round(graph_ms, 3), "host_ms": round(host_ms, 3)}
            # eager only when clearly faster AND the host has headroom: an eager step whose enqueue takes more than
            # half the device time turns host-bound on a busier CPU, while a replay costs ~1 ms of host time
            if eager_ms < 0.97 * graph_ms and host_ms < 0.5 * eager_ms:
                graph.release()
                graph = None
                torch.cuda.synchronize()
                torch.cuda.empty_cache()      # hand the graph's private pool back to the device
                run = lambda: step.step(x, y)  # noqa: E731
                for _ in range(3):            # re-warm the caching allocator before the timed loop: a fresh device
                    run()                     # allocation can wait on the driver (seconds, measured) mid-loop
    torch.cuda.synchronize()

    import gc

    gc.collect()
    gc.freeze()                 # setup objects out of the collector's generations: no long GC pass mid-loop
    barrier()
    torch.cuda.synchronize()
    trace = os.environ.get("BIGDL_BENCH_TRACE") == "1"
    if trace:                   # a host stall > 1 s inside the loop dumps the Python stack where it sits
        import faulthandler
    reserved = []
    t0 = time.perf_counter()
    stamps = []
    for _ in range(args.steps):
        if trace:
            faulthandler.dump_traceback_later(1.0, repeat=False, file=sys.stderr)
        run()
        stamps.append(time.perf_counter())     # host clock after each enqueue (host-only: no device sync)
        if trace:
            faulthandler.cancel_dump_traceback_later()
            reserved.append((round(torch.cuda.memory_reserved(dev) / 2**30, 2), round(torch.cuda.memory_allocated(dev) / 2**30, 2)))
    end = torch.cuda.Event()
    end.record()
    wait_event(end)             # poll until the device drained (see TrainStep.wait_event), then the contract's sync
    barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if os.environ.get("BIGDL_BENCH_TRACE") == "1":     # diagnostics after the timed region: per-step times, memory
        gaps = [round((b - a) * 1e3, 1) for a, b in zip([t0] + stamps[:-1], stamps)]
        print(f"[bench trace] host enqueue-to-enqueue gaps in the timed loop (ms): {gaps}", file=sys.stderr, flush=True)
        print(f"[bench trace] (reserved, allocated) GiB after each enqueue: {reserved}", file=sys.stderr, flush=True)
        free, total = torch.cuda.mem_get_info(dev)
        print(f"[bench trace] reserved {torch.cuda.memory_reserved(dev) / 2**30:.1f} GiB, max allocated "
              f"{torch.cuda.max_memory_allocated(dev) / 2**30:.1f} GiB, device free {free / 2**30:.1f} / "
              f"{total / 2**30:.1f} GiB", file=sys.stderr, flush=True)
        for i in range(8):
            torch.cuda.synchronize()
            a = time.perf_counter()
            run()
            torch.cuda.synchronize()
            print(f"[bench trace] step {i}: {(time.perf_counter() - a) * 1e3:.2f} ms, reserved "
                  f"{torch.cuda.memory_reserved(dev) / 2**30:.1f} GiB", file=sys.stderr, flush=True)
        if step is not None:      # host cost of enqueueing one iteration (no throttle wait): the eager-mode CPU floor
            old_if = step.MAX_INFLIGHT
            step.MAX_INFLIGHT = 1 << 20
            torch.cuda.synchronize()
            a = time.perf_counter()
            for _ in range(4):
                run()
            host = (time.perf_counter() - a) / 4 * 1e3
            torch.cuda.synchronize()
            step.MAX_INFLIGHT = old_if
            print(f"[bench trace] host enqueue time {host:.2f} ms/iteration", file=sys.stderr, flush=True)
    t = torch.tensor([dt], device=dev)
    if world > 1:
        import torch.distributed as dist

        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    loss = float(step.loss.item()) if step.loss is not None else float("nan")
    step.flush()
    # device-timed phases (optim/phase_timer.py) of the eager steps (a HIP-graph replay records none: then they come
    # from the eager warm-up steps); the exposed collective wait is the max over ranks
    phase = step.phase.summary(last=args.steps) if step.phase is not None else None
    comm_exposed = None
    if phase is not None:
        ce = torch.tensor([phase["comm_exposed_ms"]], device=dev)
        if world > 1:
            import torch.distributed as dist

            dist.all_reduce(ce, op=dist.ReduceOp.MAX)
        comm_exposed = round(float(ce.item()), 3)
        phase["source"] = "eager warm-up steps" if graph is not None else "timed steps"
    ms = dt / args.steps * 1e3
    ips = B * world * args.steps / dt
    if rank == 0:
        print(json.dumps({
            "metric": METRIC,
            "value": round(ips, 2),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(ips / BASELINE, 4) if BASELINE else None),
            "comm_exposed_ms": comm_exposed if step.comm.active else None,
            "dtype": "bf16",
            "data": "synthetic (random 3x224x224 images, random labels; random-init weights)",
            "config": {"model": f"ResNet-{args.depth} v1.5 (BigDL ImageNet builder{', Graph form' if args.graph_model else ''})", "global_batch": B * world,
                       "per_gpu_batch": B, "seq_len": None, "image": args.image, "parallelism": f"dp{world}",
                       "optimizer": "SGD momentum 0.9 + L2 1e-4" + (
                           f" (ZeRO-1: {dist_backend()} reduce-scatter / all-gather, optimizer state sharded)"
                           if step.comm.active else " (one rank: no gradient exchange)"),
                       "hip_graph": graph is not None, "graph_vs_eager": decision,
                       "wgrad_side_stream": side_stream.enabled(), "bucketed_overlap": step.bucketed is not None,
                       "grad_compress": step.comm.wire_format, "final_loss": round(loss, 4),
                       "phase_ms": phase},
        }), flush=True)
    Engine.shutdown()


if __name__ == "__main__":
    main()
