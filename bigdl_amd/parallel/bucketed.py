"""Bucketed, backward-overlapped gradient synchronisation (the ParallelOptimizer strategy).

Reference: S/optim/ParallelOptimizer.scala:42-791 + S/utils/DistriParameterSynchronizer.scala:66-475 — the
flat parameter vector is cut into ``bigdl.parallelOptimizer.parameterBlocks`` blocks walking the layers in
reverse execution order; as soon as a layer's backward finishes (AbstractModule.scala:282-297 hook) the blocks
it completes are put / fetched / aggregated asynchronously on a communication thread pool while the
remaining layers keep computing, and each block is updated by its own optim method.

MI355X mapping (one process per GPU, RCCL over xGMI):
  * buckets are contiguous ranges of the padded flat fp32 gradient buffer whose sizes are multiples of
    64 x world, so every bucket reduce-scatters into equal per-rank chunks (ZeRO-1 per bucket);
  * the training step runs the model's backward unit by unit (top-level layers, recursing into plain
    Sequential containers; fused residual blocks are one unit) and launches ``reduce_scatter_tensor(AVG,
    async_op=True)`` for every bucket that the finished units complete — RCCL runs it on its own stream
    while the next units' HIP kernels run on the compute stream;
  * after backward each rank updates its chunk of every bucket with a per-bucket clone of the optim method
    (fused HIP optimizer kernel, fp32 master -> bf16 shadow), then all-gathers the bf16 chunks bucket by
    bucket (async, all issued before the first wait).
Buckets default to ~8M elements (32 MB fp32): large enough to run the xGMI links near their per-link rate,
small enough that the last bucket's reduce-scatter hides behind a few layers of backward.
"""
import copy

import torch
import torch.distributed as dist


def backward_units(model):
    """Leaf units of the backward schedule, in forward order: top-level children, recursing into plain
    Sequential containers (a Sequential with a fused residual plan is a single unit)."""
    from ..nn.containers import Sequential

    units = []

    def rec(m):
        if type(m) is Sequential and m._residual_plan is None and m.modules:
            for c in m.modules:
                rec(c)
        else:
            units.append(m)

    rec(model)
    return units


def _nparams(m):
    p = m.parameters()
    return sum(t.numel() for t in p[0]) if p else 0


class BucketedGradSync:
    def __init__(self, model, w, g, w16, optim, world, rank, group=None, bucket_elems=8 << 20, total=None):
        self.model, self.w, self.g, self.w16 = model, w, g, w16
        self.world, self.rank, self.group = world, rank, group
        unit = 64 * world
        padded = w.numel()
        assert padded % unit == 0
        bucket_elems = max(unit, (bucket_elems // unit) * unit)
        self.bounds = []
        b0 = 0
        while b0 < padded:
            b1 = min(padded, b0 + bucket_elems)
            self.bounds.append((b0, b1))
            b0 = b1
        self.units = backward_units(model)
        offs, off = [], 0
        for u in self.units:
            offs.append(off)
            off += _nparams(u)
        self.unit_off = offs
        total = off if total is None else total
        # the first unit index that touches each bucket: the bucket is complete once that unit's backward ran
        self.first_unit = []
        for (b0, b1) in self.bounds:
            fu = len(self.units) - 1
            for i, (o, u) in enumerate(zip(offs, self.units)):
                n = _nparams(u)
                if n and o < b1 and o + n > b0:
                    fu = i
                    break
            if b0 >= total:       # pure padding bucket: ready immediately
                fu = len(self.units)
            self.first_unit.append(fu)
        self.chunks = [(b1 - b0) // world for (b0, b1) in self.bounds]
        self.g_chunk = [torch.empty(c, dtype=g.dtype, device=g.device) for c in self.chunks]
        self.w_chunk = [w[b0 + rank * c: b0 + (rank + 1) * c] for (b0, _), c in zip(self.bounds, self.chunks)]
        self.optims = []
        for i, ((b0, _), c) in enumerate(zip(self.bounds, self.chunks)):
            om = optim if i == 0 else copy.deepcopy(optim)
            if getattr(optim, "_wd_segments", None) is not None:
                om._wd_segments = optim._wd_segments
                om._seg_base = b0 + rank * c
            if w16 is not None:
                om.attach_shadow(w16[b0 + rank * c: b0 + (rank + 1) * c])
            self.optims.append(om)
        self.works = {}

    # ---------------------------------------------------------------------------------------- backward
    def _launch(self, b):
        b0, b1 = self.bounds[b]
        self.works[b] = dist.reduce_scatter_tensor(self.g_chunk[b], self.g[b0:b1], op=dist.ReduceOp.AVG,
                                                   group=self.group, async_op=True)

    def unit_done(self, ui):
        for b in range(len(self.bounds) - 1, -1, -1):
            if b not in self.works and self.first_unit[b] >= ui:
                self._launch(b)

    def backward(self, input, gradOutput):
        """Run the model's backward unit by unit, firing bucket reduce-scatters as they complete."""
        self.works = {}
        for b in range(len(self.bounds)):
            if self.first_unit[b] >= len(self.units):
                self._launch(b)
        g = gradOutput
        outs = [u.output for u in self.units]
        for i in range(len(self.units) - 1, -1, -1):
            inp = outs[i - 1] if i > 0 else input
            g = self.units[i].backward(inp, g)
            self.unit_done(i)
        return g

    # ---------------------------------------------------------------------------------------- update
    def update(self, loss):
        for b in range(len(self.bounds)):
            if b not in self.works:
                self._launch(b)
        lead = self.optims[0].state
        for om in self.optims[1:]:                         # keep the clones' schedules in lock-step
            for k in ("neval", "epoch"):
                if k in lead.keys():
                    om.state[k] = lead[k]
        for b in range(len(self.bounds) - 1, -1, -1):     # buckets completed first were launched first
            self.works[b].wait()
            gc = self.g_chunk[b]
            self.optims[b].optimize(lambda _: (loss, gc), self.w_chunk[b])
        gathers = []
        target = self.w16 if self.w16 is not None else self.w
        for (b0, b1), c in zip(self.bounds, self.chunks):
            mine = target[b0 + self.rank * c: b0 + (self.rank + 1) * c].clone()
            gathers.append(dist.all_gather_into_tensor(target[b0:b1], mine, group=self.group, async_op=True))
        for h in gathers:
            h.wait()
