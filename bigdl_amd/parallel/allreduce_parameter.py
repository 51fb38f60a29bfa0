"""Sharded synchronous parameter exchange over RCCL/xGMI (ZeRO-1).

Reference: S/parameters/AllReduceParameter.scala:80-329 — the reference splits the flat parameter vector
into ``partitionNum`` shards (:103-104, :138-142); every iteration each executor ``putGradients`` (:287-309),
``aggregateGradientPartition`` sums its shard (:236-278), the optimizer updates only that shard
(S/optim/DistriOptimizer.scala:370-389) and ``sendWeightPartition`` / ``getWeights`` publish and gather the
updated weights (:315-328, :201-228). Traffic goes through the Spark BlockManager with bf16-truncated
("FP16CompressedTensor") payloads.

MI355X mapping (one process per GPU, torch.distributed backend "nccl" == RCCL over xGMI):
  putGradients + aggregateGradientPartition  ->  ONE reduce_scatter_tensor (fp32, or bf16 when compression
                                                 is on — native bf16 instead of truncation), op=AVG
  optimMethod.optimize on the shard          ->  the fused HIP optimizer kernel on this rank's shard
  sendWeightPartition + getWeights           ->  ONE all_gather_into_tensor of the bf16 compute weights
The flat buffers are padded so every rank's shard has the same size (a multiple of 64 elements).
"""
import torch
import torch.distributed as dist


def dist_ready():
    return dist.is_available() and dist.is_initialized()


class AllReduceParameter:
    def __init__(self, total, world_size=None, rank=None, compress=None, group=None, align=64):
        self.world = world_size if world_size is not None else (dist.get_world_size(group) if dist_ready() else 1)
        self.rank = rank if rank is not None else (dist.get_rank(group) if dist_ready() else 0)
        self.group = group
        self.total = total
        unit = align * self.world
        self.padded = -(-total // unit) * unit
        self.shard = self.padded // self.world
        self.start = self.rank * self.shard
        self.end = self.start + self.shard
        self.compress = compress  # None / "bf16"
        self._g16 = None
        self._s16 = None

    # -- C8: broadcast of the initial weights from rank 0 (reference ModelBroadcast)
    def init(self, flat_w, extra=None):
        if self.world > 1:
            dist.broadcast(flat_w, 0, group=self.group)
            for t in extra or []:
                dist.broadcast(t, 0, group=self.group)
        return self

    def shard_of(self, flat):
        return flat[self.start:self.end]

    # -- C2/C3: reduce-scatter of gradients, averaged over ranks
    def reduce_scatter_gradients(self, flat_g, out=None):
        shard = self.shard_of(flat_g) if out is None else out
        if self.world == 1:
            return shard
        if self.compress == "bf16":
            if self._g16 is None:
                self._g16 = torch.empty(self.padded, dtype=torch.bfloat16, device=flat_g.device)
                self._s16 = torch.empty(self.shard, dtype=torch.bfloat16, device=flat_g.device)
            from .. import ops

            ops.native.get().cast_f32_bf16(flat_g, self._g16)
            dist.reduce_scatter_tensor(self._s16, self._g16, op=dist.ReduceOp.AVG, group=self.group)
            ops.native.get().cast_bf16_f32(self._s16, shard)
            return shard
        tmp = torch.empty_like(shard) if out is None else shard
        dist.reduce_scatter_tensor(tmp, flat_g, op=dist.ReduceOp.AVG, group=self.group)
        if out is None:
            shard.copy_(tmp)
        return shard

    # -- C4/C5: all-gather of the updated (bf16 compute or fp32 master) weights
    def all_gather_weights(self, flat):
        if self.world == 1:
            return flat
        dist.all_gather_into_tensor(flat, flat[self.start:self.end].clone(), group=self.group)
        return flat

    # -- C7: global scalar reductions (gradient norm clipping, loss averaging)
    def all_reduce_scalar(self, t, op="sum"):
        if self.world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX, group=self.group)
        return t
