"""Gradient processors applied to the sharded gradient between reduce-scatter and the optimizer step.

Reference: S/parameters/ParameterOperations.scala:33-133 — ``ParameterProcessor`` with two hooks:
``collectGlobalData`` (driver-coordinated reduction over every partition, e.g. the global L2 norm) and
``processParameters`` (applied to each partition's gradient shard). ConstantClippingProcessor clamps
element-wise; L2NormClippingProcessor rescales by ``min(1, threshold / ||g||)``.

Here a "partition" is a rank's ZeRO-1 gradient shard and the driver reduction is one scalar all-reduce over
RCCL, so the global norm costs one 4-byte collective instead of a Spark job.
"""
import torch


def _native():
    from ..ops import native

    return native.get()


class ParameterProcessor:
    """Subclasses must be independent of each other (they run in registration order)."""

    def collectGlobalData(self, g_shard, comm, state):
        """Cross-rank reduction; results go into ``state``."""

    def processParameters(self, g_shard, state):
        raise NotImplementedError

    def __call__(self, g_shard, comm=None):
        state = {}
        self.collectGlobalData(g_shard, comm, state)
        self.processParameters(g_shard, state)
        return g_shard


class ConstantClippingProcessor(ParameterProcessor):
    def __init__(self, min, max):
        if min > max:
            raise ValueError(f"min value {min} can not be larger than max {max}")
        self.min, self.max = float(min), float(max)

    def processParameters(self, g_shard, state):
        g_shard.clamp_(self.min, self.max)


class L2NormClippingProcessor(ParameterProcessor):
    def __init__(self, l2NormThreshold):
        if l2NormThreshold <= 0:
            raise ValueError("l2NormThreshold must be positive")
        self.threshold = float(l2NormThreshold)

    def collectGlobalData(self, g_shard, comm, state):
        sq = torch.zeros(1, device=g_shard.device)
        if g_shard.is_cuda:
            _native().sumsq(g_shard, sq)
        else:
            sq += (g_shard.float() * g_shard.float()).sum()
        if comm is not None:
            comm.all_reduce_scalar(sq)
        state["l2Norm"] = sq.sqrt()

    def processParameters(self, g_shard, state):
        # stays on the device: no host sync for the norm
        scale = torch.clamp(self.threshold / (state["l2Norm"] + 1e-6), max=1.0)
        if g_shard.is_cuda:
            _native().scale_f32(g_shard, scale, 1.0)
        else:
            g_shard.mul_(scale)


__all__ = ["ParameterProcessor", "ConstantClippingProcessor", "L2NormClippingProcessor"]
