"""Gradient processors applied to the reduced gradient shard between reduce-scatter and the optimizer step.

Reference: S/parameters/ParameterOperations.scala:33-133 — ``ParameterProcessor`` with two hooks:
``collectGlobalData`` (driver-coordinated reduction over every partition, e.g. the global L2 norm) and
``processParameters`` (applied to each partition's gradient shard). ConstantClippingProcessor clamps
element-wise; L2NormClippingProcessor rescales by ``min(1, threshold / ||g||)``; LarsProcessor
(S/optim/LarsSGD.scala:288-340) reduces per-layer ||w||² and ||g||² across partitions and hands every
LarsSGD its layer's trust scale.

Here a "partition" is the set of flat ranges this rank owns (one ZeRO-1 shard, or one chunk per bucket) and
the driver reduction is one small all-reduce over RCCL: a 4-byte norm for clipping, 2 x L floats for LARS —
no host synchronisation, the scales stay on the device.
"""
import torch

from .. import ops


def _native():
    from ..ops import native

    return native.get()


def _owned_grads(step):
    """Gradient views of every range this rank updates (the plan pieces)."""
    return [step.g[p.lo:p.hi] for p in step.plan]


def _sumsq_into(t, out):
    if t.is_cuda and t.dtype == torch.float32 and t.is_contiguous():
        _native().sumsq(t, out)
    else:
        out += (t.float() * t.float()).sum()


class ParameterProcessor:
    """Subclasses must be independent of each other (they run in registration order)."""

    def collectGlobalData(self, step, state):
        """Cross-rank reduction; results go into ``state``."""

    def processParameters(self, step, state):
        raise NotImplementedError

    def __call__(self, step, comm=None):
        if isinstance(step, torch.Tensor):       # legacy form: (g_shard, comm)
            step = _ShardView(step, comm)
        state = {}
        self.collectGlobalData(step, state)
        self.processParameters(step, state)
        return step


class _ShardView:
    """Adapter: a bare gradient shard + comm presented like a TrainStep with one piece."""

    class _P:
        def __init__(self, n):
            self.lo, self.hi = 0, n

    def __init__(self, g, comm):
        self.g, self.comm = g, comm
        self.plan = [self._P(g.numel())]
        self.device = g.device


class ConstantClippingProcessor(ParameterProcessor):
    def __init__(self, min, max):
        if min > max:
            raise ValueError(f"min value {min} can not be larger than max {max}")
        self.min, self.max = float(min), float(max)

    def processParameters(self, step, state):
        for g in _owned_grads(step):
            g.clamp_(self.min, self.max)


class L2NormClippingProcessor(ParameterProcessor):
    def __init__(self, l2NormThreshold):
        if l2NormThreshold <= 0:
            raise ValueError("l2NormThreshold must be positive")
        self.threshold = float(l2NormThreshold)

    def collectGlobalData(self, step, state):
        sq = ops.zeros(1, device=step.device)
        for g in _owned_grads(step):
            _sumsq_into(g, sq)
        if step.comm is not None:
            step.comm.all_reduce_scalar(sq)
        state["l2Norm"] = sq.sqrt()

    def processParameters(self, step, state):
        # stays on the device: no host sync for the norm
        scale = torch.clamp(self.threshold / (state["l2Norm"] + 1e-6), max=1.0)
        for g in _owned_grads(step):
            if g.is_cuda:
                _native().scale_f32(g, scale, 1.0)
            else:
                g.mul_(scale)


class LarsProcessor(ParameterProcessor):
    """Layer-wise trust ratios for every LarsSGD split: scale = (||g|| + wd·||w||) / ||w|| over the WHOLE layer,
    although each rank only owns part of it (reference LarsProcessor.collectGlobalData)."""

    def __init__(self, weightDecay):
        self.weightDecay = float(weightDecay)

    def collectGlobalData(self, step, state):
        from ..optim.methods import LarsSGD

        names = [s[0] for s in step.splits if isinstance(s[3], LarsSGD)]
        idx = {n: i for i, n in enumerate(names)}
        acc = ops.zeros(2 * len(names), device=step.device)
        for p in step.plan:
            i = idx.get(p.name)
            if i is None:
                continue
            _sumsq_into(step.w[p.lo:p.hi], acc[2 * i:2 * i + 1])
            _sumsq_into(step.g[p.lo:p.hi], acc[2 * i + 1:2 * i + 2])
        step.comm.all_reduce_scalar(acc)
        nw = acc[0::2].sqrt()
        ng = acc[1::2].sqrt()
        scale = (ng + self.weightDecay * nw) / nw
        # reference getGradientScale guards: inf -> 1e4, ~0 -> 1e-4, nan -> 1
        scale = torch.where(torch.isinf(scale), torch.full_like(scale, 1e4), scale)
        scale = torch.where(scale.abs() < 1e-4, torch.full_like(scale, 1e-4), scale)
        scale = torch.where(torch.isnan(scale), torch.ones_like(scale), scale)
        state["larsScale"] = {n: scale[i] for n, i in idx.items()}

    def processParameters(self, step, state):
        sc = state["larsScale"]
        for p in step.plan:
            if p.name in sc:
                p.method.setGradientScale(sc[p.name])


__all__ = ["ParameterProcessor", "ConstantClippingProcessor", "L2NormClippingProcessor", "LarsProcessor"]
