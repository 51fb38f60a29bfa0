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
  * model-agnostic per-module hooks, as in the reference: every module of the tree (Sequential, Graph, any
    container, fused residual blocks) carries this synchroniser in ``_sync``; ``AbstractModule`` calls
    ``before_forward`` / ``after_backward`` around every forward / backward (also for subclasses that override
    them, see ``abstractnn._sync_wrap``). When a module's backward returns, the parameters of every leaf under it
    are final (unless a leaf is still owed a backward from a second use in the same step); a bucket whose
    leaves are all final launches its in-place ``reduce_scatter_tensor(async_op=True)`` right there, so RCCL
    runs it on its own stream while the remaining layers' HIP kernels run on the compute stream;
  * after backward each rank updates its chunk of every bucket (fused HIP optimizer kernel, fp32 master ->
    bf16 shadow) bucket by bucket as the reduce-scatters land;
  * the all-gather of the updated chunks is deferred: the next step issues every bucket's all-gather in
    priority order before its forward and waits for a bucket only right before the first module that reads it
    (a leaf with parameters, or a fused container that runs its children's kernels itself), so weight
    distribution overlaps the forward pass. ``gather_all`` finishes it at any sync point.
Buckets default to ~8M elements (32 MB fp32): large enough to run the xGMI links near their per-link rate,
small enough that the last bucket's reduce-scatter hides behind a few layers of backward. Every rank executes
the same module sequence, so every rank launches the buckets in the same order (an RCCL requirement).
"""
import torch

from ..ops import side_stream as _side


def _own_ranges(m, base, es):
    """[lo, hi) element ranges of ``m``'s OWN parameters inside the flat buffer starting at ``base``."""
    out = []
    for wname, _ in getattr(m, "_params", ()):
        t = getattr(m, wname, None)
        if isinstance(t, torch.Tensor) and t.numel():
            lo = (t.data_ptr() - base) // es
            out.append((int(lo), int(lo) + t.numel()))
    return out


def _bypasses_children(m):
    """Containers whose forward runs (some of) their children's kernels without calling the children's forward:
    the fused ResNet block (nn/fusion.py residual plan) reads the last BN's weights inside its own forward."""
    return getattr(m, "_residual_plan", None) is not None


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
        self.chunks = [(b1 - b0) // world for (b0, b1) in self.bounds]
        self._index_modules(step.total)
        self.order = self._priority_order(priorities)
        self.works = {}
        self.ag_works = {}
        self._fwd = {}
        self._done = set()
        self._rem = list(self._rem0)
        self.launch_log = []          # bucket ids in launch order, for tests / diagnostics
        self.install()

    # ---------------------------------------------------------------------------------------- module index
    def _index_modules(self, total):
        base, es = self.w.data_ptr(), self.w.element_size()
        mods, seen = [], set()

        def rec(m):
            if id(m) in seen:
                return
            seen.add(id(m))
            mods.append(m)
            for c in m.modules_list() or []:
                rec(c)

        rec(self.model)
        self.modules = mods
        # leaves = modules owning parameters, in flat-buffer order (= module order of the parameter vector)
        leaves = [(r, m) for m in mods for r in [_own_ranges(m, base, es)] if r]
        leaves.sort(key=lambda t: t[0][0][0])
        self.leaves = [m for _, m in leaves]
        self.leaf_index = {id(m): i for i, m in enumerate(self.leaves)}
        nb = len(self.bounds)
        self.leaf_buckets = []
        for rngs, _ in leaves:
            bs = sorted({b for (lo, hi) in rngs for b, (b0, b1) in enumerate(self.bounds) if lo < b1 and hi > b0})
            self.leaf_buckets.append(bs)
        self._rem0 = [0] * nb
        for bs in self.leaf_buckets:
            for b in bs:
                self._rem0[b] += 1
        # every module -> the leaves under it (itself included)
        self.sub_leaves = {}

        def leaves_of(m, memo):
            k = id(m)
            if k in memo:
                return memo[k]
            memo[k] = []           # cycle guard (shared sub-trees)
            out = []
            if k in self.leaf_index:
                out.append(self.leaf_index[k])
            for c in m.modules_list() or []:
                out.extend(leaves_of(c, memo))
            memo[k] = sorted(set(out))
            return memo[k]

        memo = {}
        for m in mods:
            self.sub_leaves[id(m)] = leaves_of(m, memo)
        # buckets a module must have gathered before its forward reads weights
        self.fwd_buckets = {}
        for m in mods:
            if id(m) in self.leaf_index:
                self.fwd_buckets[id(m)] = self.leaf_buckets[self.leaf_index[id(m)]]
            elif _bypasses_children(m):
                self.fwd_buckets[id(m)] = sorted({b for li in self.sub_leaves[id(m)] for b in self.leaf_buckets[li]})
        self._pad_buckets = [b for b in range(nb) if self._rem0[b] == 0]

    def install(self):
        for m in self.modules:
            m._sync = self

    def uninstall(self):
        for m in self.modules:
            if getattr(m, "_sync", None) is self:
                m._sync = None

    def _priority_order(self, priorities):
        """Bucket all-gather issue order: highest priority first; default = forward execution order
        (reference defaultPrioritize: priority = number of layers - execution index)."""
        nb = len(self.bounds)
        if not priorities:
            return list(range(nb))
        nl = len(self.leaves)
        pr = [float("-inf")] * nb
        for li, (m, bs) in enumerate(zip(self.leaves, self.leaf_buckets)):
            p = priorities.get(m.getName(), nl - li)
            for b in bs:
                pr[b] = max(pr[b], p)
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
                with self.step.phase.span("ag"):     # the compute stream's stall on this all-gather (phase_timer)
                    h.wait()

    def gather_all(self):
        if not self.ag_works:
            self.start_gather()
        self._wait_ag(list(self.ag_works))

    def begin_step(self):
        """Called once per training step before the forward: issue the deferred all-gathers, reset the
        per-step backward bookkeeping."""
        if self.step._pending_gather:
            self.start_gather()
            self.step._pending_gather = False
        self.works = {}
        self._fwd = {}
        self._done = set()
        self._rem = list(self._rem0)
        self.launch_log = []

    def before_forward(self, m):
        k = id(m)
        self._fwd[k] = self._fwd.get(k, 0) + 1
        if self.ag_works:
            bs = self.fwd_buckets.get(k)
            if bs:
                self._wait_ag(bs)

    def end_forward(self):
        self._wait_ag(list(self.ag_works))

    # ---------------------------------------------------------------------------------------- backward
    def _launch(self, b):
        if b in self.works:
            return
        b0, b1 = self.bounds[b]
        self.launch_log.append(b)
        from . import graph_segments

        side = _side.pending_stream()
        if side is None or graph_segments.active() is not None or not getattr(self.comm, "_inplace", False):
            _side.join()     # weight gradients issued on the side stream (ops/side_stream.py) land first
            self.works[b] = self.comm.reduce_scatter_range(self.g, b0, b1, async_op=True)[0]
            return
        # launch from the side stream after it waited for the compute stream (BN parameter gradients are written
        # there): the collective follows every weight gradient of the bucket, and the compute stream never stalls
        # for the side stream mid-backward; update() waits for the collective on the compute stream
        side.wait_stream(torch.cuda.current_stream(side.device))
        with torch.cuda.stream(side):
            self.works[b] = self.comm.reduce_scatter_range(self.g, b0, b1, async_op=True)[0]

    def after_backward(self, m):
        if self.step.defer_sync:   # straggler drop: every rank reduces after the finished vote (TrainStep)
            return
        k = id(m)
        n = self._fwd.get(k, 0)
        if n > 1:                  # used again earlier in the forward: its gradient is not final yet
            self._fwd[k] = n - 1
            return
        self._fwd[k] = 0
        ready = []
        for li in self.sub_leaves.get(k, ()):
            if li in self._done:
                continue
            leaf = self.leaves[li]
            if self._fwd.get(id(leaf), 0) > 0 and leaf is not m:
                continue           # the leaf still owes a backward of its own (shared elsewhere)
            self._done.add(li)
            for b in self.leaf_buckets[li]:
                self._rem[b] -= 1
                if self._rem[b] == 0:
                    ready.append(b)
        # buckets completed by the same backward launch last-first: launch order is the reverse of the flat-buffer
        # (= forward execution) order, identical on every rank
        for b in sorted(ready, reverse=True):
            self._launch(b)

    def begin_backward(self):
        if self.step.defer_sync:
            return
        for b in self._pad_buckets:          # pure padding buckets: nothing to wait for
            self._launch(b)

    def end_backward(self):
        for b in range(len(self.bounds) - 1, -1, -1):
            if b not in self.works:
                self._launch(b)

    # ---------------------------------------------------------------------------------------- update
    def update(self, loss):
        self.end_backward()
        step = self.step
        if step.processors:
            # processors (clipping, LARS) need the whole reduced gradient first
            for b in list(self.launch_log):
                h = self.works.pop(b)
                if h is not None:
                    with step.phase.span("rs"):
                        h.wait()
            step.apply_processors()
            step.optimize_pieces(loss)
            return
        step._lockstep()
        for b in list(self.launch_log):                   # in launch order: the earliest collectives land first
            h = self.works.pop(b)
            if h is not None:
                with step.phase.span("rs"):               # the compute stream's stall on this reduce-scatter
                    h.wait()
            b0, b1 = self.bounds[b]
            pieces = [p for p in step.plan if b0 <= p.lo and p.hi <= b1]
            for p in pieces:
                gs = self.g[p.lo:p.hi]
                p.method.optimize(lambda _x, _g=gs: (loss, _g), self.w[p.lo:p.hi])
