"""Distributed pieces on the CPU engine over gloo: synchronized BatchNorm (reference
T/nn/SpatialBatchNormalizationSpec / S/utils/ParameterSynchronizer.scala) and the sharded AllReduceParameter."""
import torch

from bigdl_amd.utils.testing import run_distributed


def _bn():
    from bigdl_amd import nn

    bn = nn.SpatialBatchNormalization(3)
    bn.weight.copy_(torch.tensor([0.5, 1.0, 2.0]))
    bn.bias.copy_(torch.tensor([0.1, -0.2, 0.3]))
    return bn


def _sync_bn_job(rank, world, x_full, gy_full):
    from bigdl_amd import nn
    from bigdl_amd.parallel.sync_bn import enable_sync_bn

    bn = _bn()
    seq = nn.Sequential().add(bn)
    assert enable_sync_bn(seq) == 1
    n = x_full.shape[0] // world
    x = x_full[rank * n:(rank + 1) * n]
    gy = gy_full[rank * n:(rank + 1) * n]
    y = seq.forward(x)
    gx = seq.backward(x, gy)
    return y, gx, bn.gradWeight.clone(), bn.gradBias.clone(), bn.runningMean.clone()


def test_sync_bn_matches_global_batch():
    from bigdl_amd import nn

    g = torch.Generator().manual_seed(0)
    x = torch.randn(8, 3, 4, 4, generator=g) * 2 + 1
    gy = torch.randn(8, 3, 4, 4, generator=g)
    res = run_distributed(_sync_bn_job, 2, (x, gy))
    ref = _bn()
    y = ref.forward(x)
    gx = ref.backward(x, gy)
    ys = torch.cat([res[0][0], res[1][0]])
    gxs = torch.cat([res[0][1], res[1][1]])
    assert torch.allclose(ys, y, atol=1e-5)
    assert torch.allclose(gxs, gx, atol=1e-5)
    # parameter gradients are per-replica partial sums (the optimizer all-reduces them)
    assert torch.allclose(res[0][2] + res[1][2], ref.gradWeight, atol=1e-4)
    assert torch.allclose(res[0][3] + res[1][3], ref.gradBias, atol=1e-4)
    assert torch.allclose(res[0][4], ref.runningMean, atol=1e-5)


def _arp_job(rank, world):
    from bigdl_amd.parallel.allreduce_parameter import AllReduceParameter

    arp = AllReduceParameter(1000, compress="fp32")
    w = torch.full((arp.padded,), float(rank))
    arp.init(w)
    g = torch.arange(arp.padded, dtype=torch.float32) * (rank + 1)
    shard = arp.reduce_scatter_gradients(g).clone()
    w[arp.start:arp.end] += 10 * (rank + 1)
    arp.all_gather_weights(w)
    return w.clone(), shard, arp.padded, arp.shard


def test_allreduce_parameter_shards():
    res = run_distributed(_arp_job, 2)
    padded, shard = res[0][2], res[0][3]
    assert padded % 128 == 0 and padded >= 1000 and shard * 2 == padded
    full = torch.arange(padded, dtype=torch.float32) * 1.5     # AVG of (1x, 2x)
    assert torch.allclose(res[0][1], full[:shard]) and torch.allclose(res[1][1], full[shard:])
    expect = torch.cat([torch.full((shard,), 10.0), torch.full((shard,), 20.0)])  # broadcast rank0 weights (0)
    assert torch.equal(res[0][0], expect) and torch.equal(res[1][0], expect)


def _bucketed_job(rank, world, data, iters, bucket):
    import torch as _t
    from bigdl_amd import nn as _nn
    from bigdl_amd import optim as _O
    from bigdl_amd.optim.train_step import TrainStep
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(5)
    model = _nn.Sequential().add(_nn.Linear(6, 16)).add(_nn.Tanh()) \
        .add(_nn.Sequential().add(_nn.Linear(16, 16)).add(_nn.ReLU())).add(_nn.Linear(16, 2))
    step = TrainStep(model, _nn.MSECriterion(), _O.SGD(0.05, momentum=0.9, dampening=0.0), device="cpu",
                     overlap=True, bucket_elems=bucket)
    assert step.bucketed is not None and len(step.bucketed.bounds) >= 2
    X, Y = data
    n = X.shape[0] // world
    for i in range(iters):
        step.step(X[rank * n:(rank + 1) * n], Y[rank * n:(rank + 1) * n])
    step.gather_model()      # the weight all-gather of the last update is deferred to the next forward
    w, _ = model.getParameters()
    return w[:model._flat_total].clone()


def _plain_job(rank, world, data, iters):
    from bigdl_amd import nn as _nn
    from bigdl_amd import optim as _O
    from bigdl_amd.optim.train_step import TrainStep
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(5)
    model = _nn.Sequential().add(_nn.Linear(6, 16)).add(_nn.Tanh()) \
        .add(_nn.Sequential().add(_nn.Linear(16, 16)).add(_nn.ReLU())).add(_nn.Linear(16, 2))
    step = TrainStep(model, _nn.MSECriterion(), _O.SGD(0.05, momentum=0.9, dampening=0.0), device="cpu",
                     overlap=False)
    X, Y = data
    n = X.shape[0] // world
    for i in range(iters):
        step.step(X[rank * n:(rank + 1) * n], Y[rank * n:(rank + 1) * n])
    step.comm.all_gather_weights(step.w)
    w, _ = model.getParameters()
    return w[:model._flat_total].clone()


def test_bucketed_overlap_equals_plain_zero1():
    """ParallelOptimizer-style bucketed reduce-scatter during backward == one post-backward reduce-scatter."""
    g = torch.Generator().manual_seed(0)
    X = torch.randn(16, 6, generator=g)
    Y = torch.randn(16, 2, generator=g)
    a = run_distributed(_bucketed_job, 2, ((X, Y), 4, 128))
    b = run_distributed(_plain_job, 2, ((X, Y), 4))
    assert torch.allclose(a[0], a[1], atol=1e-6)
    assert torch.allclose(a[0], b[0], atol=1e-5)


def _bcast_worker(rank, world, port, q):
    import os

    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bigdl_amd.nn as nn
    from bigdl_amd.parallel.broadcast import ModelBroadcast

    torch.manual_seed(rank)
    m = nn.Sequential().add(nn.Linear(4, 3)).add(nn.BatchNormalization(3))
    with torch.no_grad():
        m.modules[1].runningMean.fill_(float(rank))
    ModelBroadcast().broadcast(m)
    # plain numpy payloads: a tensor would travel as a shared-memory handle that vanishes when this worker exits
    q.put((rank, m.modules[0].weight.detach().clone().numpy(), m.modules[1].runningMean.clone().numpy()))
    dist.destroy_process_group()


def test_model_broadcast_gloo():
    import multiprocessing as mp
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_bcast_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (torch.from_numpy(w), torch.from_numpy(rm))) for r, w, rm in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(60)
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[1][1], torch.zeros(3))


def _compress_modes(rank, world):
    import torch

    from bigdl_amd.parallel.allreduce_parameter import AllReduceParameter

    out = {}
    for mode in ("fp16", "bf16"):
        comm = AllReduceParameter(256, compress=mode)
        g = torch.full((comm.padded,), 1.0 + 2 ** -8 + 2 ** -10)
        work, chunk = comm.reduce_scatter_range(g, 0, comm.padded, average=False)
        if work is not None:
            work.wait()
        out[mode] = chunk.clone()
    return out


def test_fp16_compression_is_reference_truncation():
    """bigdl.compress=fp16 reproduces the reference FP16CompressedTensor (S/parameters/FP16CompressedTensor.scala:
    271-279: the upper 16 bits of each fp32): 1 + 2^-8 + 2^-10 truncates to 1.0 on both ranks (sum 2.0), while the
    bf16 mode rounds to nearest even (1 + 2^-7 each)."""
    from bigdl_amd.utils.testing import run_distributed

    res = run_distributed(_compress_modes, 2)
    for r in res:
        assert torch.all(r["fp16"] == 2.0), r["fp16"][:4]
        assert torch.all(r["bf16"] == 2.0 * (1.0 + 2 ** -7)), r["bf16"][:4]
    x = torch.randn(1000) * 100
    from bigdl_amd.ops.nnk import f32_to_bf16_rtz

    t = f32_to_bf16_rtz(x)
    assert torch.equal(t.float().view(torch.int32), x.view(torch.int32) & -65536)   # bits & 0xffff0000
