"""One synchronous data-parallel training iteration on one device rank.

This is the per-rank core that the reference spreads over DistriOptimizer's two Spark jobs per iteration
(S/optim/DistriOptimizer.scala:204-396): getWeights → forward/backward → putGradients → aggregate shard →
parameter processors → optimize shard (per sub-module OptimMethod, :370-389) → sendWeightPartition.
On MI355X it is:

  zero grads (one memset of the flat fp32 gradient buffer)
  forward / criterion / backward through the BigDL module protocol (HIP kernels, bf16 NHWC activations)
  reduce-scatter of the flat gradients over RCCL (ZeRO-1 shard per rank)                      [N > 1]
  parameter processors on the shard (clipping, LARS layer norms: one small all-reduce each)
  fused optimizer kernel per (owned range ∩ sub-module split), writing the bf16 compute shard
  all-gather of the updated weights over RCCL (exact fp32 master on every rank, or bf16)      [N > 1]

With ``overlap`` (ParallelOptimizer) the flat buffer is cut into buckets: each bucket's reduce-scatter is
launched as soon as backward has produced it, and the all-gather of the updated weights is deferred to the
start of the NEXT step where each bucket is waited for only right before the first layer that reads it
(reference: update deferred to the next forward, S/nn/abstractnn/AbstractModule.scala:1184-1199; layers
synchronised in priority order, S/optim/ParallelOptimizer.scala:675-683). ``flush()`` completes a pending
all-gather (before a checkpoint, validation or the end of training).

Layer regularizers (L1/L2) are folded into the optimizer kernel as per-segment decay (identical maths:
the reference adds lambda*w inside accGradParameters before the gradient average, which equals adding it
after the average). Nothing in ``step`` synchronises with the host, so the whole step — including the RCCL
collectives — can be captured into a HIP graph once buffers are warm (``optim/graphed.py``).
"""
import copy

import os

import torch

from .. import ops
from ..ops import native

# BIGDL_NATIVE_FILL bit mask (default 7): 1 gradient zeroing, 2 BN statistics arena, 4 strided-dgrad phase fill as
# runtime memsets / native kernels instead of aten fills (A/B and bisection switch)
_NATIVE_FILL = int(os.environ.get("BIGDL_NATIVE_FILL", "7"))

from ..optim.regularizer import L1L2Regularizer
from ..parallel.allreduce_parameter import AllReduceParameter


def fold_regularizers(model, total, device):
    """Collect L2 regularizer coefficients per parameter segment of the flat buffer; disable them in the
    modules. Returns (seg_off int64, seg_wd fp32) device tensors or None when nothing is regularized."""
    offs, vals = [], []
    off = 0
    folded_any = False
    for m in model.flattened_layers():
        if m.modules_list():
            continue
        for w, g in m._params:
            t = getattr(m, w, None)
            if t is None:
                continue
            reg = m.bRegularizer if w == "bias" else m.wRegularizer
            lam = 0.0
            if reg is not None:
                if not isinstance(reg, L1L2Regularizer) or reg.l1 != 0.0:
                    return None  # unsupported for folding: keep module-level regularization
                lam = reg.l2 * (m.scaleB if w == "bias" else m.scaleW)
            offs.append(off)
            vals.append(lam)
            off += t.numel()
            folded_any = folded_any or lam != 0.0
    if not folded_any:
        return None
    for m in model.flattened_layers():
        if m.wRegularizer is not None or m.bRegularizer is not None:
            m._reg_folded = True
    # merge consecutive equal segments
    mo, mv = [], []
    for o, v in zip(offs, vals):
        if mv and mv[-1] == v:
            continue
        mo.append(o)
        mv.append(v)
    return (torch.tensor(mo, dtype=torch.int64, device=device), torch.tensor(mv, dtype=torch.float32, device=device))


# --------------------------------------------------------------------------------------------- splits
def find_module(model, name):
    for m in model.flattened_layers():
        if m.getName() == name:
            return m
    return None


def _param_range(model, sub, fw):
    """[lo, hi) of ``sub``'s parameters inside the flat weight buffer ``fw`` (they are contiguous)."""
    p = sub.parameters()
    if not p:
        return None
    base = fw.data_ptr()
    es = fw.element_size()
    lo = min((w.data_ptr() - base) // es for w in p[0])
    hi = max((w.data_ptr() - base) // es + w.numel() for w in p[0])
    return int(lo), int(hi)


def parameter_splits(model, methods, fw, total, expand=False):
    """Map each OptimMethod to the flat range of the sub-module it is registered for.

    Reference DistriOptimizer.scala:816-853: one method for the whole model, or one per named sub-module whose
    ranges must tile the whole parameter vector. With ``expand`` (ParallelOptimizer.expandOptimMethods,
    ParallelOptimizer.scala:642-670) every leaf layer without an explicit method inherits its nearest
    ancestor's (consecutive leaves inheriting the same method share one split — element-wise methods make that
    identical to per-layer clones).
    Returns a list of (name, lo, hi, method) sorted by lo.
    """
    if len(methods) == 1 and not expand:
        name, m = next(iter(methods.items()))
        if name != model.getName() and find_module(model, name) is None:
            raise ValueError(f"{name} doesn't have corresponding sub-module in {model.getName()}")
        sub = model if name == model.getName() else find_module(model, name)
        rng = (0, total) if sub is model else _param_range(model, sub, fw)
        if rng != (0, total):
            raise ValueError(f"DistriOptimizer: All subModules should have an OptimMethod ({name} covers "
                             f"{rng} of {total})")
        return [(name, 0, total, m)]
    if expand:
        out = []

        def walk(mod, inherited):
            meth = methods.get(mod.getName(), inherited)
            kids = mod.modules_list()
            if not kids:
                rng = _param_range(model, mod, fw)
                if rng is not None:
                    if meth is None:
                        raise ValueError(f"{mod.getName()}'s parent optim method should not be null")
                    out.append((mod.getName(), rng[0], rng[1], meth))
                return
            for k in kids:
                walk(k, meth)

        walk(model, methods.get(model.getName()))
        out.sort(key=lambda t: t[1])
        # LarsSGD is not element-wise (one trust ratio per split): every leaf keeps its own split, as the
        # reference's per-layer clones do
        from .methods import LarsSGD

        merged = []
        for s in out:
            if merged and merged[-1][3] is s[3] and merged[-1][2] == s[1] and not isinstance(s[3], LarsSGD):
                merged[-1] = (merged[-1][0], merged[-1][1], s[2], s[3])
            else:
                merged.append(s)
        out = merged
    else:
        out = []
        for name, m in methods.items():
            sub = model if name == model.getName() else find_module(model, name)
            if sub is None:
                raise ValueError(f"Optimizer couldn't find {name} in {model.getName()}")
            rng = _param_range(model, sub, fw)
            if rng is None:
                continue
            out.append((name, rng[0], rng[1], m))
        out.sort(key=lambda t: t[1])
    pos = 0
    for name, lo, hi, _ in out:
        if lo != pos:
            raise ValueError(f"DistriOptimizer: All subModules should have an OptimMethod (gap at {pos}, "
                             f"next split {name} starts at {lo})")
        pos = hi
    if pos != total:
        raise ValueError(f"DistriOptimizer: All subModules should have an OptimMethod (covered {pos} of {total})")
    return out


class UpdatePiece:
    """One optimizer call per step: ``method`` on flat range [lo, hi) owned by this rank."""

    __slots__ = ("name", "lo", "hi", "method", "split_lo", "split_hi", "primary")

    def __init__(self, name, lo, hi, method, split_lo, split_hi, primary):
        self.name, self.lo, self.hi, self.method = name, lo, hi, method
        self.split_lo, self.split_hi, self.primary = split_lo, split_hi, primary

    def __repr__(self):
        return f"UpdatePiece({self.name}, [{self.lo},{self.hi}), {type(self.method).__name__})"


def build_update_plan(owned, splits, w16, seg):
    """Intersect this rank's owned ranges with the method splits. The first piece of every split uses the
    registered method object itself; further pieces use clones (per-piece optimizer state, like the reference's
    per-partition OptimMethod copies)."""
    plan = []
    seen, used = set(), set()
    for (a, b) in owned:
        for name, lo, hi, m in splits:
            x, y = max(a, lo), min(b, hi)
            if y <= x:
                continue
            primary = name not in seen
            seen.add(name)
            meth = m if id(m) not in used else _clone_method(m)
            used.add(id(meth))
            if seg is not None:
                meth._wd_segments = seg
                meth._seg_base = x
            if w16 is not None:
                meth.attach_shadow(w16[x:y])
            plan.append(UpdatePiece(name, x, y, meth, lo, hi, primary))
    return plan


def _clone_method(m):
    sh = m._shadow16
    m._shadow16 = None
    try:
        c = copy.deepcopy(m)
    finally:
        m._shadow16 = sh
    return c


# --------------------------------------------------------------------------------------------- TrainStep
def wait_event(ev, poll_s=100e-6):
    """Host wait for a device event by polling (``hipEventQuery`` + short sleeps) instead of the blocking
    ``hipEventSynchronize``: a blocking wait parks on a completion interrupt, and on this stack a missed one was
    measured to stall the host for 3.3 s in an otherwise 26 ms/step loop (``bench.py`` trace: one enqueue gap of
    3316 ms, the device idle behind it)."""
    import time

    while not ev.query():
        time.sleep(poll_s)


class TrainStep:
    def __init__(self, model, criterion, optim_method, device=None, comm=None, compress="auto", fuse=True,
                 overlap=None, bucket_elems=8 << 20, processors=None, expand_methods=False, priorities=None):
        from ..utils.engine import Engine

        self.device = torch.device(device) if device is not None else Engine.device()
        if self.device.type == "cuda":
            from ..ops import side_stream

            side_stream.priority_compute_stream(self.device)     # data-gradient chain ahead of the side stream
        self.model = model
        self.criterion = criterion
        self.methods = dict(optim_method) if isinstance(optim_method, dict) else {model.getName(): optim_method}
        self.optim = next(iter(self.methods.values()))
        model.to(self.device)
        criterion.to(self.device)
        if fuse and self.device.type == "cuda":
            from ..nn.fusion import fuse_for_training

            fuse_for_training(model)
        ws, _ = model.parameters() or ([], [])
        total = sum(w.numel() for w in ws)
        self.total = total
        self.comm = comm if comm is not None else AllReduceParameter(total, compress=compress)
        self.w, self.g = model.getParameters()
        if self.w.numel() != self.comm.padded:
            # re-flatten into a padded buffer so every rank's shard has the same size
            pw = torch.zeros(self.comm.padded, device=self.device)
            pg = torch.zeros(self.comm.padded, device=self.device)
            pw[:total].copy_(self.w[:total])
            model._flat = None
            self.w, self.g = _reflatten(model, pw, pg)
        self.comm.init(self.w, [t for t in (model.getExtraParameter() or [])])
        self.w16 = None
        if self.device.type == "cuda":
            self.w16 = torch.empty(self.comm.padded, dtype=torch.bfloat16, device=self.device)
            self.w16.copy_(self.w)
            model.attach_bf16_shadow(self.w16)
        self.seg = fold_regularizers(model, total, self.device) if self.device.type == "cuda" else None
        self.w_shard = self.comm.shard_of(self.w)
        self.g_shard = self.comm.shard_of(self.g)
        self.splits = parameter_splits(model, self.methods, self.w, total, expand=expand_methods)
        self.processors = list(processors or [])
        from ..optim.methods import LarsSGD

        lars = [s for s in self.splits if isinstance(s[3], LarsSGD)]
        if lars:
            from ..parallel.processors import LarsProcessor

            self.processors.append(LarsProcessor(lars[0][3].weightDecay))
        self.loss = None
        # ParallelOptimizer-style bucketed reduce-scatter overlapped with backward (parallel/bucketed.py)
        if overlap is None:
            overlap = self.comm.active
        self.bucketed = None
        if overlap and self.comm.active:
            from ..parallel.bucketed import BucketedGradSync

            self.bucketed = BucketedGradSync(self, bucket_elems, priorities)
            owned = self.bucketed.owned_ranges()
        else:
            owned = [(self.comm.start, self.comm.end)]
        self.plan = build_update_plan(owned, self.splits, self.w16, self.seg)
        self._pending_gather = False
        from .phase_timer import PhaseTimer

        # device-timed phases (compute / exposed reduce-scatter / exposed all-gather / update), optim/phase_timer.py
        self.phase = PhaseTimer(enabled=self.device.type == "cuda"
                                and os.environ.get("BIGDL_PHASE_TIMING", "1") != "0")

    # ------------------------------------------------------------------ pieces
    def zero_grad(self):
        if self.g.is_cuda and _NATIVE_FILL & 1:
            native.get().fill_bytes(self.g, 0)       # one runtime memset, no aten fill kernel
        else:
            self.g.zero_()

    def forward_backward(self, x, y):
        m, c = self.model, self.criterion
        m.training()
        self.phase.begin_step()
        bk = self.bucketed
        if bk is not None:
            bk.begin_step()
        out = m.forward(x)
        if bk is not None:
            bk.end_forward()
        loss = c.forward(out, y)
        gout = c.backward(out, y)
        convs = self._dgrad_convs()
        if convs:
            from ..ops import conv as cv

            cv.prepare_dgrad_weights(convs)       # every conv weight transposed for its dgrad in one launch
        try:
            if bk is not None:
                bk.begin_backward()
            m.backward(x, gout)
        finally:
            if convs:
                cv.end_dgrad_weights()
        self.phase.mark("bwd")
        return loss

    def forward_backward_step(self, x, y):
        """forward_backward inside this step's BN-statistics arena (what ``step`` runs before the update)."""
        arena = None
        if self.device.type == "cuda":
            from ..ops.bn import ARENA as arena

            arena.begin(self.device)
        try:
            return self.forward_backward(x, y)
        finally:
            if arena is not None:
                arena.end()

    def _dgrad_convs(self):
        """Convolutions whose backward runs the native data-gradient GEMM (GPU engine, one group)."""
        if getattr(self, "_dgrad_conv_list", None) is None:
            from ..nn.conv import SpatialConvolution

            dev = getattr(self, "device", None)
            ok = dev is not None and torch.device(dev).type == "cuda"
            self._dgrad_conv_list = [q for q in self.model.flattened_layers()
                                     if ok and isinstance(q, SpatialConvolution) and getattr(q, "nGroup", 1) == 1
                                     and hasattr(q, "_dgrad_gpu") and hasattr(q, "_w16_padded")]
        return self._dgrad_conv_list

    def _lockstep(self):
        """Keep every method clone's iteration/epoch counters equal to its primary's."""
        prim = {p.name: p.method for p in self.plan if p.primary}
        for p in self.plan:
            if not p.primary:
                lead = prim[p.name].state
                for k in ("neval", "epoch", "Loss", "score"):
                    if k in lead.keys():
                        p.method.state[k] = lead[k]

    def apply_processors(self):
        for proc in self.processors:
            proc(self)

    def optimize_pieces(self, loss, pieces=None, g=None):
        self._lockstep()
        g = self.g if g is None else g
        for p in (self.plan if pieces is None else pieces):
            gs = g[p.lo:p.hi]
            p.method.optimize(lambda _x, _g=gs: (loss, _g), self.w[p.lo:p.hi])

    def sync_and_update(self, loss, finished=None):
        """Reduce gradients, run processors and the sharded update, publish the weights.

        ``finished`` (straggler drop, DistriOptimizer.scala:421-449): this rank's 0/1 contribution weight; the
        gradient is averaged over the ranks that finished and the update is skipped when fewer than
        ``min_finished`` did. Returns False when the update was skipped."""
        if finished is not None:
            ok = self._sync_and_update_weighted(loss, finished)
            self.phase.end_step()
            return ok
        if self.bucketed is not None:
            self.bucketed.update(loss)
            self._pending_gather = True
            self.phase.end_step()
            return True
        with self.phase.span("rs", self.comm.active):
            self.comm.reduce_scatter_gradients(self.g, out=self.g_shard)
        self.apply_processors()
        self.optimize_pieces(loss)
        with self.phase.span("ag", self.comm.active):
            self.comm.all_gather_weights(self.w, self.w16)
        self.phase.end_step()
        return True

    min_finished = 0.0
    # straggler drop: no collective may start inside backward (a late rank skips it), so the bucketed hooks only
    # record and ``_sync_and_update_weighted`` reduces once every rank has voted
    defer_sync = False

    def _sync_and_update_weighted(self, loss, finished):
        """A dropped rank (``finished`` 0) on a GPU may still have kernels of its abandoned iteration queued on the
        compute stream (a slow device, see nn/abstractnn.py DevicePacer). Its part of the exchange — the vote, a
        zero gradient contribution, the update of the shard it owns and the weight all-gather — runs on a stream that
        does not wait for the compute stream, so the finished ranks are not held in the collectives by its backlog;
        the compute stream waits for that stream before the next iteration. The zero contribution comes from a
        separate buffer: the abandoned kernels may still be writing the gradient buffer."""
        self.flush()
        late = not finished and self.device.type == "cuda"
        if not late:
            return self._weighted_exchange(loss, finished, self.g)
        if getattr(self, "_late_stream", None) is None:
            from ..ops import side_stream

            self._late_stream = side_stream.peer_stream(self.device)
            with torch.cuda.stream(self._late_stream):     # zeroed on the stream that reads it (the compute stream
                self._late_g = ops.zero_(torch.empty_like(self.g))   # may be backlogged: a fill there races the use)
        cur = torch.cuda.current_stream(self.device)
        s = self._late_stream
        with torch.cuda.stream(s):
            try:
                return self._weighted_exchange(loss, 0.0, self._late_g)
            finally:
                ops.zero_(self._late_g)         # the reduced chunks landed in it
                cur.wait_stream(s)

    def _weighted_exchange(self, loss, finished, g):
        cnt = torch.tensor([float(finished)], device=self.device)
        self.comm.all_reduce_scalar(cnt)
        n = float(cnt.item())
        if not finished and g is self.g:
            ops.zero_(self.g)
        if self.bucketed is not None:
            # the update plan is per bucket (this rank owns one chunk of every bucket, not [start, end)):
            # reduce each bucket into its owned chunk and average those chunks over the finished ranks
            chunks = []
            for (b0, b1) in self.bucketed.bounds:
                work, chunk = self.comm.reduce_scatter_range(g, b0, b1, average=False)
                if work is not None:
                    work.wait()
                chunks.append(chunk)
            if n <= 0 or n < self.min_finished:
                return False
            for c in chunks:
                c.mul_(1.0 / n)
        else:
            shard = self.comm.shard_of(g)
            self.comm.reduce_scatter_gradients(g, out=shard, average=False)
            if n <= 0 or n < self.min_finished:
                return False
            shard.mul_(1.0 / n)
        if g is not self.g:
            self._processors_on(g)
        else:
            self.apply_processors()
        self.optimize_pieces(loss, g=g)
        if self.bucketed is not None:
            self.bucketed.gather_all()
        else:
            self.comm.all_gather_weights(self.w, self.w16)
        return True

    def _processors_on(self, g):
        """Run the parameter processors (clipping, LARS) on another gradient buffer than ``self.g``."""
        if not self.processors:
            return
        keep = self.g
        self.g = g
        try:
            self.apply_processors()
        finally:
            self.g = keep

    def flush(self):
        """Complete a deferred (bucketed) weight all-gather: afterwards every rank holds the current weights."""
        if self._pending_gather:
            self.bucketed.gather_all()
            self._pending_gather = False

    def gather_model(self):
        """Reference DistriOptimizer.getModel: exact fp32 weights everywhere and rank 0's extra state (BN
        running statistics) on every rank. Collective: every rank must call it."""
        self.flush()
        self.comm.gather_master(self.w)
        if self.comm.active:
            for t in self.model.getExtraParameter() or []:
                self.comm.broadcast(t, 0)
        return self.model

    def step(self, x, y):
        arena = None
        if self.device.type == "cuda":
            from ..ops.bn import ARENA as arena

            arena.begin(self.device)
        try:
            self.zero_grad()
            loss = self.forward_backward(x, y)
            self.sync_and_update(loss)
        finally:
            if arena is not None:
                arena.end()
        self.loss = loss
        self.throttle()
        return loss

    MAX_INFLIGHT = int(os.environ.get("BIGDL_MAX_INFLIGHT", "2"))

    def throttle(self):
        """Bound how many enqueued iterations the host runs ahead of the device (``MAX_INFLIGHT``). Blocks that a
        side-stream kernel still reads (``record_stream``, ops/side_stream.py) are reusable only once that kernel
        ran; a host far ahead keeps allocating fresh blocks for every queued iteration until the caching allocator
        hits the device limit and falls back to synchronising frees (measured: 27 -> 100-150 ms/step on an
        unthrottled 20-step loop). Not inside a HIP-graph capture."""
        if self.device.type != "cuda" or torch.cuda.is_current_stream_capturing():
            return
        q = self.__dict__.setdefault("_inflight", [])
        ev = torch.cuda.Event()
        ev.record()
        q.append(ev)
        while len(q) > self.MAX_INFLIGHT:
            wait_event(q.pop(0))
        # the device finished at least that iteration: a persistent-kernel timeout in it is visible now
        from ..ops import native

        native.check_persistent()
        self.phase_done = self.phase.collect()     # phases of the iterations that completed (no synchronisation)

    # ------------------------------------------------------------------ optimizer state (checkpoints)
    def _method_layout(self):
        """{registered method name: (method, [(split name, split lo, split hi, offset in the method's state)])}.

        A registered OptimMethod may cover several splits (``expand``: one split per run of leaves inheriting it);
        its checkpointed per-element state is the concatenation of those splits in flat-buffer order, so the saved
        layout depends only on the model and the registration, not on the rank count or the bucket layout."""
        out = {}
        for mname, meth in self.methods.items():
            segs, off = [], 0
            for sname, lo, hi, m in self.splits:
                if m is meth:
                    segs.append((sname, lo, hi, off))
                    off += hi - lo
            out[mname] = (meth, segs, off)
        return out

    def gather_optim_state(self):
        """Full-size optimizer state per registered method, identical on every rank (collective).

        Every per-element state tensor of a piece (same length as the piece) is placed at its offset inside a
        zero tensor as long as everything the method covers, and the disjoint pieces of all ranks are summed with
        one all-reduce. Scalars and schedules come from the method object. Returns {method name: OptimMethod}."""
        out = {}
        for mname, (meth, segs, size) in self._method_layout().items():
            full = _clone_method(meth)
            full._shadow16 = None
            seg_of = {s[0]: s for s in segs}
            keys = {}
            for p in self.plan:
                sg = seg_of.get(p.name)
                if sg is None:
                    continue
                base = sg[3] + (p.lo - sg[1])
                for k, v in p.method.state.items():
                    if torch.is_tensor(v) and v.dim() == 1 and v.numel() == p.hi - p.lo:
                        if k not in keys:
                            keys[k] = torch.zeros(size, dtype=v.dtype, device=v.device)
                        keys[k][base:base + (p.hi - p.lo)].copy_(v)
            for k in list(full.state.keys()):
                if torch.is_tensor(full.state[k]) and full.state[k].dim() == 1:
                    del full.state[k]
            # ranks may own no piece of a method: agree on the key set first
            names = sorted(_all_keys(self.comm, mname, list(keys)))
            for k in names:
                t = keys.get(k)
                if t is None:
                    t = torch.zeros(size, dtype=torch.float32, device=self.device)
                self.comm.all_reduce_scalar(t)
                full.state[k] = t
            out[mname] = full
        return out

    def load_optim_state(self, methods):
        """Inverse of ``gather_optim_state``: slice each method's full-size state into this rank's pieces (on
        this rank's device); scalar state (counters, schedules) is copied to every piece."""
        layout = self._method_layout()
        for mname, src in methods.items():
            if mname not in layout:
                continue
            _, segs, size = layout[mname]
            seg_of = {s[0]: s for s in segs}
            for p in self.plan:
                sg = seg_of.get(p.name)
                if sg is None:
                    continue
                base = sg[3] + (p.lo - sg[1])
                for k, v in src.state.items():
                    if torch.is_tensor(v) and v.dim() == 1:
                        if v.numel() != size:
                            raise ValueError(f"optimizer state {mname}.{k}: {v.numel()} elements, the model "
                                             f"needs {size}")
                        p.method.state[k] = v[base:base + (p.hi - p.lo)].to(device=self.device).clone()
                    elif not torch.is_tensor(v):
                        p.method.state[k] = v


def _all_keys(comm, name, keys):
    if comm.world == 1:
        return set(keys)
    import torch.distributed as dist

    got = [None] * comm.world
    dist.all_gather_object(got, keys, group=comm.group)
    s = set()
    for g in got:
        s.update(g)
    return s


def _reflatten(model, fw, fg):
    """Rebind every parameter of ``model`` into the given (padded) flat buffers, keeping values."""
    ws, gs = model.parameters()
    views = []
    off = 0
    from ..nn.abstractnn import _dense_strides

    for w, g in zip(ws, gs):
        n = w.numel()
        st = _dense_strides(w)
        vw = fw[off:off + n].as_strided(w.shape, st)
        vg = fg[off:off + n].as_strided(w.shape, st)
        vw.copy_(w.detach())
        vg.copy_(g.detach())
        views.append((vw, vg, off, n, st))
        off += n
    model._rebind_params(views)
    model._flat = (fw, fg)
    model._flat_views = views
    model._flat_total = off
    return fw, fg
