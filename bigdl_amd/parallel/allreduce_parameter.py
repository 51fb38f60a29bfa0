"""Sharded synchronous parameter exchange over RCCL/xGMI (ZeRO-1).

Reference: S/parameters/AllReduceParameter.scala:80-329 — the reference splits the flat parameter vector
into ``partitionNum`` shards (:103-104, :138-142); every iteration each executor ``putGradients`` (:287-309),
``aggregateGradientPartition`` sums its shard (:236-278), the optimizer updates only that shard
(S/optim/DistriOptimizer.scala:370-389) and ``sendWeightPartition`` / ``getWeights`` publish and gather the
updated weights (:315-328, :201-228). Traffic goes through the Spark BlockManager with bf16-truncated
("FP16CompressedTensor") payloads; ``DistriOptimizer.getModel`` (:658-697) collects the exact fp32 shards
(``weightPartition``) before a checkpoint or the return of ``optimize()``.

MI355X mapping (one process per GPU, torch.distributed backend "nccl" == RCCL over xGMI):
  putGradients + aggregateGradientPartition  ->  ONE reduce_scatter_tensor, in place (the shard is a view of
                                                 the flat gradient at this rank's offset): fp32, or bf16 when
                                                 compression is on (native bf16 instead of truncation)
  optimMethod.optimize on the shard          ->  the fused HIP optimizer kernel on this rank's shard; it also
                                                 writes the shard of the bf16 compute copy
  sendWeightPartition + getWeights           ->  ONE in-place all_gather_into_tensor:
        compress=None : of the fp32 master shards, then one cast of the whole buffer into the bf16 compute copy
                        (every rank holds exact fp32 weights after every step, so any layer may read them)
        compress=bf16 : of the bf16 compute shards (half the bytes), then the non-owned fp32 ranges are
                        rebuilt from them — exactly the reference's decompress-into-local-weights semantics;
                        ``gather_master`` gathers the exact fp32 shards (reference getModel) on demand
The flat buffers are padded so every rank's shard has the same size (a multiple of 64 elements).
"""
import torch
import torch.distributed as dist

from .graph_segments import issue as _issue


def dist_ready():
    return dist.is_available() and dist.is_initialized()


def _native():
    from ..ops import native

    return native.get()


class AllReduceParameter:
    def __init__(self, total, world_size=None, rank=None, compress="auto", group=None, align=64):
        self.world = world_size if world_size is not None else (dist.get_world_size(group) if dist_ready() else 1)
        self.rank = rank if rank is not None else (dist.get_rank(group) if dist_ready() else 0)
        self.group = group
        self.total = total
        unit = align * self.world
        self.padded = -(-total // unit) * unit
        self.shard = self.padded // self.world
        self.start = self.rank * self.shard
        self.end = self.start + self.shard
        if compress == "auto":
            # the reference's wire format: 16-bit gradients and weights whenever anything goes over the wire
            # (S/parameters/AllReduceParameter.scala:171-172,297-302,321); fp32 is the opt-in ("none" / "fp32")
            compress = "bf16" if self.world > 1 else None
        if compress in ("none", "fp32"):
            compress = None
        if compress not in (None, "bf16", "fp16", "fp16-truncate", "bf16-rtz"):
            raise ValueError(f"unsupported gradient compression {compress!r} (None, 'bf16' or 'fp16')")
        # "fp16" (the reference's bigdl.compress value) is its FP16CompressedTensor: the upper 16 bits of each fp32,
        # i.e. bf16 by truncation (S/parameters/FP16CompressedTensor.scala:271-279) — kept bit-exact here as a
        # parity mode; "bf16" rounds to nearest even (half the error, the default for new jobs)
        self.rtz = compress in ("fp16", "fp16-truncate", "bf16-rtz")
        self.compress = "bf16" if compress is not None else None
        self._g16 = None
        # run the collectives even on one rank (BIGDL_FORCE_COLLECTIVES=1): exercises the RCCL path and its HIP
        # graph capture on a single GPU
        import os

        self.active = self.world > 1 or os.environ.get("BIGDL_FORCE_COLLECTIVES", "0") == "1" and dist_ready()
        # RCCL collectives exchange tensors in place; gloo wants distinct buffers
        self._inplace = dist_ready() and dist.get_backend(group) == "nccl"

    @property
    def wire_format(self):
        """What the gradient / weight exchange puts on the wire (for logs and the bench JSON)."""
        if not self.active:
            return "none (no exchange)"
        if self.compress is None:
            return "fp32"
        return "bf16-rtz (reference FP16CompressedTensor)" if self.rtz else "bf16"

    @property
    def localPartitionRange(self):
        """(start, length) of this rank's shard in the flat vector (reference :117)."""
        return self.start, self.shard

    # -- C8: broadcast of the initial weights from rank 0 (reference ModelBroadcast)
    def init(self, flat_w, extra=None):
        if self.active:
            dist.broadcast(flat_w, 0, group=self.group)
            for t in extra or []:
                dist.broadcast(t, 0, group=self.group)
        return self

    def shard_of(self, flat):
        return flat[self.start:self.end]

    # ------------------------------------------------------------------------- collectives on a range
    def _rs(self, out_shard, full, op, async_op=False):
        if self._inplace:
            w = _issue(lambda: dist.reduce_scatter_tensor(out_shard, full, op=op, group=self.group, async_op=True))
            if not async_op:
                _wait(w)
            return w
        tmp = torch.empty_like(out_shard)
        w = dist.reduce_scatter_tensor(tmp, full, op=op, group=self.group)
        out_shard.copy_(tmp)
        return _Done() if async_op else w

    def _ag(self, full, my_shard, async_op=False):
        if self._inplace:
            w = _issue(lambda: dist.all_gather_into_tensor(full, my_shard, group=self.group, async_op=True))
            if not async_op:
                _wait(w)
            return w
        w = dist.all_gather_into_tensor(full, my_shard.clone(), group=self.group)
        return _Done() if async_op else w

    # -- C2/C3: reduce-scatter of gradients (averaged over ranks unless ``scale`` is given: sum then scale)
    def reduce_scatter_range(self, g, lo, hi, async_op=False, average=True):
        """Reduce-scatter ``g[lo:hi]`` (a multiple of ``world`` long) into this rank's chunk of it, in place.
        Returns (work or None, chunk view)."""
        n = (hi - lo) // self.world
        chunk = g[lo + self.rank * n: lo + (self.rank + 1) * n]
        if not self.active:
            return None, chunk
        op = dist.ReduceOp.AVG if average and self._avg_ok() else dist.ReduceOp.SUM
        if self.compress == "bf16":
            g16 = self._bf16_buf(g)
            (_cast_f32_bf16_rtz if self.rtz else _cast_f32_bf16)(g[lo:hi], g16[lo:hi])
            c16 = g16[lo + self.rank * n: lo + (self.rank + 1) * n]
            work = self._rs(c16, g16[lo:hi], op, async_op=async_op)
            return _Post(work, lambda: (_cast_bf16_f32(c16, chunk), self._fix_avg(chunk, op, average))), chunk
        work = self._rs(chunk, g[lo:hi], op, async_op=async_op)
        if op == dist.ReduceOp.SUM and average:
            return _Post(work, lambda: chunk.mul_(1.0 / self.world)), chunk
        return work, chunk

    def _avg_ok(self):
        return self._inplace          # gloo has no AVG reduction

    def _fix_avg(self, chunk, op, average):
        if average and op == dist.ReduceOp.SUM:
            chunk.mul_(1.0 / self.world)

    def _bf16_buf(self, like):
        if self._g16 is None or self._g16.numel() != like.numel() or self._g16.device != like.device:
            self._g16 = torch.empty(like.numel(), dtype=torch.bfloat16, device=like.device)
        return self._g16

    def reduce_scatter_gradients(self, flat_g, out=None, average=True):
        work, chunk = self.reduce_scatter_range(flat_g, 0, self.padded, average=average)
        _wait(work)
        if out is not None and out.data_ptr() != chunk.data_ptr():
            out.copy_(chunk)
            return out
        return chunk

    # -- C4/C5: all-gather of the updated weights
    def all_gather_range(self, w, w16, lo, hi, async_op=False):
        """Publish this rank's updated chunk of ``[lo, hi)`` to every rank (see module docstring for the two
        compression modes). Returns a work handle whose ``wait()`` also finishes the local bf16/fp32
        conversion of the range."""
        if not self.active:
            return None
        n = (hi - lo) // self.world
        a, b = lo + self.rank * n, lo + (self.rank + 1) * n
        if self.compress == "bf16" and w16 is not None:
            work = self._ag(w16[lo:hi], w16[a:b], async_op=async_op)

            def post():
                if a > lo:
                    _cast_bf16_f32(w16[lo:a], w[lo:a])
                if hi > b:
                    _cast_bf16_f32(w16[b:hi], w[b:hi])
            return _Post(work, post)
        work = self._ag(w[lo:hi], w[a:b], async_op=async_op)
        if w16 is None:
            return work
        return _Post(work, lambda: _cast_f32_bf16(w[lo:hi], w16[lo:hi]))

    def all_gather_weights(self, w, w16=None):
        _wait(self.all_gather_range(w, w16, 0, self.padded))
        return w

    def gather_master(self, w):
        """Exact fp32 weights on every rank (reference DistriOptimizer.getModel :658-697). With uncompressed
        exchange they already are; with bf16 exchange the fp32 master shards are all-gathered."""
        if self.active and self.compress == "bf16":
            _wait(self._ag(w, w[self.start:self.end]))
        return w

    # -- C7: global scalar reductions (gradient norm clipping, loss averaging, LARS norms, finished counts)
    def all_reduce_scalar(self, t, op="sum"):
        if self.active:
            rop = dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX
            _wait(_issue(lambda: dist.all_reduce(t, op=rop, group=self.group, async_op=True)))
        return t

    def broadcast(self, t, src=0):
        if self.active:
            _wait(_issue(lambda: dist.broadcast(t, src, group=self.group, async_op=True)))
        return t


class _Done:
    def wait(self):
        return True


class _Post:
    """A collective handle plus a local step to run once it completed (cast / scale)."""

    def __init__(self, work, post):
        self.work, self.post = work, post
        self._done = False

    def wait(self):
        if not self._done:
            _wait(self.work)
            self.post()
            self._done = True
        return True


def _wait(work):
    if work is not None:
        work.wait()


def _cast_f32_bf16(src, dst):
    if src.is_cuda:
        _native().cast_f32_bf16(src, dst)
    else:
        dst.copy_(src)


def _cast_f32_bf16_rtz(src, dst):
    """bf16 by truncation (drop the low 16 mantissa bits), the reference FP16CompressedTensor encoding."""
    from ..ops.nnk import f32_to_bf16_rtz

    f32_to_bf16_rtz(src, out=dst)


def _cast_bf16_f32(src, dst):
    if src.is_cuda:
        _native().cast_bf16_f32(src, dst)
    else:
        dst.copy_(src)
