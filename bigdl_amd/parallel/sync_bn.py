"""Cross-replica (synchronized) BatchNorm.

Reference: S/utils/ParameterSynchronizer.scala:25-106 — thread replicas publish per-channel mean / std and
their gradient counterparts through a CyclicBarrier exchange (S/nn/SpatialBatchNormalization.scala:1116-1151,
1258-1329), enabled by ``setParallism`` (S/nn/BatchNormalization.scala:72-76).

MI355X mapping: one process per GPU; the BN kernels produce packed fp32 [sum, sumsq] (forward) and
[sum dy, sum dy*(x-mean)] (backward) buffers of 2C floats; ``sync_fn`` all-reduces that buffer (RCCL over xGMI
on GPU, gloo on CPU) and returns the global element count, so normalisation uses statistics of the global
batch. One collective of 2C floats per BN layer per direction.
"""
import torch
import torch.distributed as dist


def make_sync_fn(group=None):
    def sync(buf, count):
        if not (dist.is_available() and dist.is_initialized()):
            return count
        ws = dist.get_world_size(group)
        if ws == 1:
            return count
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
        return count * ws

    return sync


def enable_sync_bn(model, group=None):
    """Turn every BatchNormalization in ``model`` into a synchronized BN over ``group``."""
    from ..nn.normalization import BatchNormalization

    fn = make_sync_fn(group)
    n = 0
    for m in model.flattened_layers():
        if isinstance(m, BatchNormalization):
            m.sync_fn = fn
            n += 1
    return n
