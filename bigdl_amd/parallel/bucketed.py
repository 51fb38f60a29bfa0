"""Bucketed, backward-overlapped gradient synchronisation (the ParallelOptimizer strategy).

Reference: S/optim/ParallelOptimizer.scala:42-791 + S/utils/DistriParameterSynchronizer.scala:66-475 — the
flat parameter vector is cut into ``bigdl.parallelOptimizer.parameterBlocks`` blocks walking the layers in
reverse execution order; as soon as a layer's backward finishes (AbstractModule.scala:282-297 hook) the blocks
it completes are put / fetched / aggregated asynchronously on a communication thread pool while the
remaining layers keep computing; each layer is updated by its own optim method (expandOptimMethods,
ParallelOptimizer.scala:642-670) and the synchronised weights are fetched in priority order (first-executed
layer first, defaultPrioritize :675-683) before the layer's next forward (AbstractModule.scala:1184-1199).

MI355X mapping (one process per GPU, RCCL over xGMI):
  * buckets are contiguous ranges of the padded flat fp32 gradient buffer whose sizes are multiples of
    64 x world, so every bucket reduce-scatters into equal per-rank chunks (ZeRO-1 per bucket);
  * the training step runs the model's backward unit by unit (top-level layers, recursing into plain
    Sequential containers; fused residual blocks are one unit) and launches an in-place
    ``reduce_scatter_tensor(async_op=True)`` for every bucket the finished units complete — RCCL runs it on its
    own stream while the next units' HIP kernels run on the compute stream (fp32, or bf16-compressed);
  * after backward each rank updates its chunk of every bucket (fused HIP optimizer kernel, fp32 master ->
    bf16 shadow) bucket by bucket as the reduce-scatters land;
  * the all-gather of the updated chunks is deferred: the next step issues every bucket's all-gather in
    priority order before its forward and waits for a bucket only right before the first unit that reads it,
    so weight distribution overlaps the forward pass. ``gather_all`` finishes it at any sync point.
Buckets default to ~8M elements (32 MB fp32): large enough to run the xGMI links near their per-link rate,
small enough that the last bucket's reduce-scatter hides behind a few layers of backward.
"""
import torch


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
    def __init__(self, step, bucket_elems=8 << 20, priorities=None):
        self.step = step
        self.model, self.w, self.g, self.w16 = step.model, step.w, step.g, step.w16
        self.comm = step.comm
        world, rank = self.comm.world, self.comm.rank
        self.world, self.rank = world, rank
        unit = 64 * world
        padded = self.w.numel()
        assert padded % unit == 0
        bucket_elems = max(unit, (bucket_elems // unit) * unit)
        self.bounds = []
        b0 = 0
        while b0 < padded:
            b1 = min(padded, b0 + bucket_elems)
            self.bounds.append((b0, b1))
            b0 = b1
        self.units = backward_units(self.model)
        offs, off = [], 0
        for u in self.units:
            offs.append(off)
            off += _nparams(u)
        self.unit_off = offs
        total = step.total
        nb, nu = len(self.bounds), len(self.units)
        # the first unit index that touches each bucket: the bucket's gradient is complete once that unit's
        # backward ran (units run backward last-to-first); the same unit is the first forward reader
        self.first_unit = []
        self.last_unit = []
        for (b0, b1) in self.bounds:
            fu, lu = nu - 1, 0
            touched = [i for i, (o, u) in enumerate(zip(offs, self.units))
                       if _nparams(u) and o < b1 and o + _nparams(u) > b0]
            if touched:
                fu, lu = touched[0], touched[-1]
            if b0 >= total:       # pure padding bucket: ready immediately
                fu, lu = nu, nu
            self.first_unit.append(fu)
            self.last_unit.append(lu)
        # buckets a unit must wait for before its forward
        self.unit_needs = [[b for b in range(nb) if self.first_unit[b] <= i <= self.last_unit[b]]
                           for i in range(nu)]
        self.chunks = [(b1 - b0) // world for (b0, b1) in self.bounds]
        self.order = self._priority_order(priorities)
        self.works = {}
        self.ag_works = {}

    def _priority_order(self, priorities):
        """Bucket all-gather issue order: highest priority first; default = forward execution order
        (reference defaultPrioritize: priority = len - execution index)."""
        nb = len(self.bounds)
        if not priorities:
            return list(range(nb))
        pr = []
        for b in range(nb):
            best = float("-inf")
            for i in range(min(self.first_unit[b], len(self.units) - 1), min(self.last_unit[b], len(self.units) - 1) + 1):
                best = max(best, priorities.get(self.units[i].getName(), len(self.units) - i))
            pr.append(best)
        return sorted(range(nb), key=lambda b: (-pr[b], b))

    def owned_ranges(self):
        return [(b0 + self.rank * c, b0 + (self.rank + 1) * c) for (b0, _), c in zip(self.bounds, self.chunks)]

    # ---------------------------------------------------------------------------------------- forward
    def start_gather(self):
        self.ag_works = {}
        for b in self.order:
            b0, b1 = self.bounds[b]
            self.ag_works[b] = self.comm.all_gather_range(self.w, self.w16, b0, b1, async_op=True)

    def _wait_ag(self, buckets):
        for b in buckets:
            h = self.ag_works.pop(b, None)
            if h is not None:
                h.wait()

    def gather_all(self):
        if not self.ag_works:
            self.start_gather()
        self._wait_ag(list(self.ag_works))

    def forward(self, x):
        """Forward unit by unit, waiting for each bucket's weight all-gather only before its first reader."""
        if self.step._pending_gather:
            self.start_gather()
            self.step._pending_gather = False
        out = x
        for i, u in enumerate(self.units):
            if self.ag_works:
                self._wait_ag(self.unit_needs[i])
            out = u.forward(out)
        self._wait_ag(list(self.ag_works))
        self.model.output = out
        return out

    # ---------------------------------------------------------------------------------------- backward
    def _launch(self, b):
        b0, b1 = self.bounds[b]
        self.works[b] = self.comm.reduce_scatter_range(self.g, b0, b1, async_op=True)[0]

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
        self.model.gradInput = g
        return g

    # ---------------------------------------------------------------------------------------- update
    def update(self, loss):
        for b in range(len(self.bounds)):
            if b not in self.works:
                self._launch(b)
        step = self.step
        if step.processors:
            # processors (clipping, LARS) need the whole reduced gradient first
            for b in range(len(self.bounds)):
                h = self.works.pop(b)
                if h is not None:
                    h.wait()
            step.apply_processors()
            step.optimize_pieces(loss)
            return
        step._lockstep()
        for b in range(len(self.bounds) - 1, -1, -1):     # buckets completed first were launched first
            h = self.works.pop(b)
            if h is not None:
                h.wait()
            b0, b1 = self.bounds[b]
            pieces = [p for p in step.plan if b0 <= p.lo and p.hi <= b1]
            for p in pieces:
                gs = self.g[p.lo:p.hi]
                p.method.optimize(lambda _x, _g=gs: (loss, _g), self.w[p.lo:p.hi])
