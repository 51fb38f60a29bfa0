"""Data pipeline core (reference S/dataset/: Sample.scala:138-586, MiniBatch.scala:34-764,
Transformer.scala:86-391 (``->`` chaining, SampleToMiniBatch :309), DataSet.scala:53-669).

* ``Sample``: features + labels (tensors or lists of tensors).
* ``MiniBatch``: stacked input/target with ``slice(offset, length)`` (1-based offset like the reference).
* ``Transformer``: iterator -> iterator; chain with ``a >> b`` (reference ``a -> b``) or ``a.then(b)``.
* ``DataSet``: ``array`` (local), ``rdd``-style ``distributed`` (each rank of the torch.distributed job owns
  a disjoint shard, the analogue of the reference's one-partition-per-node coalesce at DataSet.scala:362-371),
  ``data(train)`` yields an infinite shuffled stream for training and a finite pass for evaluation.
"""
import math
import threading
import queue

import torch

from ..utils.table import Table


class Sample:
    def __init__(self, features, labels=None):
        self.features = list(features) if isinstance(features, (list, tuple)) else [features]
        if labels is None:
            self.labels = []
        else:
            self.labels = list(labels) if isinstance(labels, (list, tuple)) else [labels]
        self.features = [_as_tensor(f) for f in self.features]
        self.labels = [_as_tensor(l) for l in self.labels]

    def feature(self, i=0):
        return self.features[i]

    def label(self, i=0):
        return self.labels[i] if self.labels else None

    def numFeature(self):
        return len(self.features)

    def numLabel(self):
        return len(self.labels)

    def getFeatureSize(self):
        return [tuple(f.shape) for f in self.features]

    def getLabelSize(self):
        return [tuple(l.shape) for l in self.labels]

    def __repr__(self):
        return f"Sample(features={self.getFeatureSize()}, labels={self.getLabelSize()})"


def _as_tensor(t):
    """torch tensor of a feature / label: bigdl_amd Tensor / SparseTensor wrappers unwrap to their torch tensor
    (sparse COO stays sparse)."""
    if getattr(t, "_is_bigdl_tensor", False):
        return t._t
    return t if isinstance(t, torch.Tensor) else torch.as_tensor(t)


ArraySample = Sample
TensorSample = Sample


class PaddingParam:
    """Pad variable-length features to the longest in a batch (reference MiniBatch PaddingParam)."""

    def __init__(self, paddingTensor=None, paddingStrategy="default", fixedLength=None):
        self.paddingTensor = paddingTensor
        self.fixedLength = fixedLength
        self.value = 0.0 if paddingTensor is None else float(torch.as_tensor(paddingTensor).reshape(-1)[0])


class MiniBatch:
    def __init__(self, input, target=None):
        self.input = input
        self.target = target

    def getInput(self):
        return self.input

    def getTarget(self):
        return self.target

    def size(self):
        x = self.input
        if isinstance(x, Table):
            x = x[1]
        return x.shape[0]

    def slice(self, offset, length):
        """1-based offset, as in the reference (MiniBatch.scala:49)."""
        def sl(t):
            if t is None:
                return None
            if isinstance(t, Table):
                o = Table()
                for k, v in t.items():
                    o[k] = sl(v)
                return o
            return t.narrow(0, offset - 1, length)

        return MiniBatch(sl(self.input), sl(self.target))

    def to(self, device, non_blocking=False):
        def mv(t):
            if t is None:
                return None
            if isinstance(t, Table):
                return t.to(device)
            return t.to(device, non_blocking=non_blocking)

        return MiniBatch(mv(self.input), mv(self.target))

    def __repr__(self):
        return f"MiniBatch(size={self.size()})"


def _stack(ts, pad=None):
    shapes = {tuple(t.shape) for t in ts}
    if len(shapes) == 1:
        return torch.stack(ts)
    # variable length along dim 0: pad to the max (or fixed) length
    L = max(t.shape[0] for t in ts)
    if pad is not None and pad.fixedLength:
        L = max(L, pad.fixedLength)
    val = pad.value if pad is not None else 0.0
    out = torch.full((len(ts), L) + tuple(ts[0].shape[1:]), val, dtype=ts[0].dtype)
    for i, t in enumerate(ts):
        out[i, : t.shape[0]] = t
    return out


def _batch_sparse(ts):
    """Concatenate per-sample sparse COO tensors along a new leading batch dimension: sample i's indices get
    batch index i (1-D [D] features, or [1, D] rows, batch to [B, D]; reference SparseTensorUtils.concat used by
    SparseMiniBatch.set, S/dataset/MiniBatch.scala:588-660)."""
    idx, val = [], []
    shape = None
    for i, t in enumerate(ts):
        t = t.coalesce()
        ind = t.indices()
        if t.dim() == 2 and t.shape[0] == 1:            # [1, D] row -> [D]
            ind = ind[1:]
            tshape = tuple(t.shape[1:])
        else:
            tshape = tuple(t.shape)
        if shape is None:
            shape = tshape
        elif len(tshape) != len(shape):
            raise ValueError(f"SparseMiniBatch: sample {i} has rank {len(tshape)}, expected {len(shape)}")
        shape = tuple(max(a, b) for a, b in zip(shape, tshape))
        idx.append(torch.cat([torch.full((1, ind.shape[1]), i, dtype=torch.int64), ind], 0))
        val.append(t.values())
    return torch.sparse_coo_tensor(torch.cat(idx, 1), torch.cat(val), (len(ts),) + shape).coalesce()


def _batch_feature(ts, pad=None):
    return _batch_sparse(ts) if ts[0].is_sparse else _stack(ts, pad)


class SparseMiniBatch(MiniBatch):
    """MiniBatch whose inputs may be sparse COO tensors (reference SparseMiniBatch, S/dataset/MiniBatch.scala:588):
    each sparse feature of the samples is concatenated into one [batch, ...] sparse tensor, dense features and
    labels are stacked as usual; ``SampleToMiniBatch`` produces it whenever a sample feature is sparse (wide &
    deep: SparseLinear / SparseJoinTable inputs)."""

    def size(self):
        x = self.input
        if isinstance(x, Table):
            x = x[1]
        return x.shape[0]

    def slice(self, offset, length):
        def sl(t):
            if t is None:
                return None
            if isinstance(t, Table):
                o = Table()
                for k, v in t.items():
                    o[k] = sl(v)
                return o
            if t.is_sparse:
                return t.index_select(0, torch.arange(offset - 1, offset - 1 + length)).coalesce()
            return t.narrow(0, offset - 1, length)

        return SparseMiniBatch(sl(self.input), sl(self.target))

    def to(self, device, non_blocking=False):
        mb = super().to(device, non_blocking)
        return SparseMiniBatch(mb.input, mb.target)


def samples_to_minibatch(samples, featurePadding=None, labelPadding=None):
    if any(f.is_sparse for f in samples[0].features):
        nf, nl = samples[0].numFeature(), samples[0].numLabel()
        feats = [_batch_feature([s.features[i] for s in samples], featurePadding) for i in range(nf)]
        inp = feats[0] if nf == 1 else Table(*feats)
        labs = [_batch_feature([s.labels[i] for s in samples], labelPadding) for i in range(nl)]
        tgt = None if nl == 0 else (labs[0] if nl == 1 else Table(*labs))
        return SparseMiniBatch(inp, tgt)
    nf = samples[0].numFeature()
    nl = samples[0].numLabel()
    if nf == 1:
        inp = _stack([s.features[0] for s in samples], featurePadding)
    else:
        inp = Table(*[_stack([s.features[i] for s in samples], featurePadding) for i in range(nf)])
    if nl == 0:
        tgt = None
    elif nl == 1:
        tgt = _stack([s.labels[0] for s in samples], labelPadding)
    else:
        tgt = Table(*[_stack([s.labels[i] for s in samples], labelPadding) for i in range(nl)])
    return MiniBatch(inp, tgt)


class Transformer:
    """iterator -> iterator. ``a >> b`` chains (reference ``->``)."""

    def apply(self, it):
        raise NotImplementedError

    def __call__(self, it):
        return self.apply(it)

    def __rshift__(self, other):
        return ChainedTransformer(self, other)

    def then(self, other):
        return self >> other

    def cloneTransformer(self):
        import copy

        return copy.deepcopy(self)


class ChainedTransformer(Transformer):
    def __init__(self, first, last):
        self.first, self.last = first, last

    def apply(self, it):
        return self.last.apply(self.first.apply(it))


class FnTransformer(Transformer):
    """Per-element map."""

    def __init__(self, fn):
        self.fn = fn

    def apply(self, it):
        for x in it:
            yield self.fn(x)


class Identity(Transformer):
    def apply(self, it):
        return it


class SampleToMiniBatch(Transformer):
    """Group samples into MiniBatches of ``batchSize`` (per rank: total batch / partitionNum)."""

    def __init__(self, batchSize, featurePaddingParam=None, labelPaddingParam=None, partitionNum=None,
                 dropRemainder=False):
        self.batchSize = batchSize
        self.featurePadding, self.labelPadding = featurePaddingParam, labelPaddingParam
        self.partitionNum = partitionNum
        self.dropRemainder = dropRemainder

    def _per_rank(self):
        from ..utils.engine import Engine

        n = self.partitionNum or Engine.world_size()
        assert self.batchSize % n == 0, f"batch size {self.batchSize} must be a multiple of {n} ranks"
        return self.batchSize // n

    def apply(self, it):
        bs = self._per_rank()
        buf = []
        for s in it:
            buf.append(s)
            if len(buf) == bs:
                yield samples_to_minibatch(buf, self.featurePadding, self.labelPadding)
                buf = []
        if buf and not self.dropRemainder:
            yield samples_to_minibatch(buf, self.featurePadding, self.labelPadding)


SampleToBatch = SampleToMiniBatch


class Prefetch(Transformer):
    """Background-thread prefetch of ``depth`` elements (overlaps host data prep with device compute)."""

    def __init__(self, depth=2):
        self.depth = depth

    def apply(self, it):
        q = queue.Queue(self.depth)
        sentinel = object()

        def worker():
            try:
                for x in it:
                    q.put(x)
            finally:
                q.put(sentinel)

        t = threading.Thread(target=worker, daemon=True)
        t.start()
        while True:
            x = q.get()
            if x is sentinel:
                return
            yield x


# ---------------------------------------------------------------------------------------------- DataSet
class AbstractDataSet:
    def data(self, train):
        raise NotImplementedError

    def size(self):
        raise NotImplementedError

    def shuffle(self):
        pass

    def transform(self, transformer):
        return TransformedDataSet(self, transformer)

    def __rshift__(self, transformer):
        return self.transform(transformer)

    def toLocal(self):
        return self

    def toDistributed(self):
        return self

    def isDistributed(self):
        return False


class LocalDataSet(AbstractDataSet):
    """A dataset iterated in this process (reference LocalDataSet, DataSet.scala:134-153): ``data`` yields the
    elements, ``toLocal`` is the identity, it is never distributed."""

    def toLocal(self):
        return self

    def isDistributed(self):
        return False


class LocalArrayDataSet(LocalDataSet):
    """In-memory dataset; training iteration is an infinite stream reshuffled every epoch starting at a
    random offset (reference DataSet.scala:247-324)."""

    def __init__(self, buffer, shuffle=True, seed=None):
        self.buffer = list(buffer)
        self._do_shuffle = shuffle
        self._perm = list(range(len(self.buffer)))
        self._gen = torch.Generator().manual_seed(seed if seed is not None else 42)

    def size(self):
        return len(self.buffer)

    def shuffle(self):
        if self._do_shuffle and len(self.buffer) > 1:
            self._perm = torch.randperm(len(self.buffer), generator=self._gen).tolist()

    def data(self, train):
        n = len(self.buffer)
        if not train:
            for i in range(n):
                yield self.buffer[i]
            return
        while True:
            self.shuffle()
            for i in self._perm:
                yield self.buffer[i]


class DistributedDataSet(LocalArrayDataSet):
    """Rank-sharded dataset: rank r owns elements r, r+world, ... of the global collection."""

    def __init__(self, buffer, shuffle=True, seed=None, rank=None, world=None):
        from ..utils.engine import Engine

        self.rank = Engine.rank() if rank is None else rank
        self.world = Engine.world_size() if world is None else world
        allb = list(buffer)
        self.global_size = len(allb)
        super().__init__(allb[self.rank::self.world], shuffle, None if seed is None else seed + self.rank)

    def size(self):
        return self.global_size

    def isDistributed(self):
        return True

    def originRDD(self):
        return self.buffer


class CachedDistriDataSet(DistributedDataSet):
    """Rank-local partition held in memory with an index permutation (reference CachedDistriDataSet,
    DataSet.scala:247-321).

    ``data(True)`` is an endless stream over this rank's elements in index order starting at a random offset
    (``RNG.uniform(0, n - (groupSize - 1))``); ``data(False)`` walks them once in order. ``shuffle`` draws a new
    permutation unless ``isInOrder`` (sequence data whose consecutive ``groupSize`` records form one batch).
    ``cache`` / ``unpersist`` toggle ``isCached``; ``originRDD`` is the partition buffer."""

    def __init__(self, buffer, isInOrder=False, groupSize=1, rank=None, world=None):
        super().__init__(buffer, shuffle=False, rank=rank, world=world)
        self.isInOrder, self.groupSize = bool(isInOrder), int(groupSize)
        self.indexes = list(range(len(self.buffer)))
        self.isCached = False

    def data(self, train):
        from ..utils.random_generator import RNG

        n = len(self.buffer)
        if not train:
            for i in range(n):
                yield self.buffer[self.indexes[i]]
            return
        if n == 0:
            return
        group = self.groupSize if self.isInOrder else 1
        span = max(1, n - (group - 1))
        i = int(RNG.uniform(0, span))
        while True:
            yield self.buffer[self.indexes[i % n]]
            i += 1

    def shuffle(self):
        if not self.isInOrder:
            perm = torch.randperm(len(self.buffer), generator=self._gen).tolist()
            self.indexes = perm

    def cache(self):
        self.isCached = True

    def unpersist(self):
        self.isCached = False


class TransformedDataSet(AbstractDataSet):
    def __init__(self, base, transformer):
        self.base = base
        self.transformer = transformer

    def size(self):
        return self.base.size()

    def shuffle(self):
        self.base.shuffle()

    def data(self, train):
        return self.transformer.apply(self.base.data(train))

    def isDistributed(self):
        return self.base.isDistributed()

    def transform(self, transformer):
        return TransformedDataSet(self, transformer)


class DataSet:
    @staticmethod
    def array(data, shuffle=True):
        return LocalArrayDataSet(data, shuffle)

    @staticmethod
    def rdd(data, shuffle=True):
        """Distributed dataset over the ranks of the job (Spark RDD analogue)."""
        return DistributedDataSet(data, shuffle)

    distributed = rdd

    @staticmethod
    def imageFrame(frame):
        from .vision import ImageFrameDataSet

        return ImageFrameDataSet(frame)

    @staticmethod
    def SeqFileFolder():
        from .seqfile import SeqFileFolder
        return SeqFileFolder

    @staticmethod
    def ImageFolder():
        from .seqfile import ImageFolder
        return ImageFolder

    @staticmethod
    def from_tensors(x, y=None, shuffle=True, distributed=False):
        samples = [Sample(x[i], None if y is None else y[i]) for i in range(x.shape[0])]
        return DataSet.rdd(samples, shuffle) if distributed else DataSet.array(samples, shuffle)


def batches_per_epoch(size, batch):
    return int(math.ceil(size / float(batch)))


class ArrayTensorMiniBatch(MiniBatch):
    """Dense mini-batch built from per-sample tensors (reference ArrayTensorMiniBatch, MiniBatch.scala:92): stacks
    ``inputData`` / ``targetData`` (lists of equally shaped tensors, or of tensor lists for multi-input samples)
    into batch tensors (a Table for several inputs)."""

    def __init__(self, inputData, targetData=None):
        def stack(col):
            if col is None or len(col) == 0:
                return None
            if isinstance(col[0], (list, tuple)):
                return Table(*[torch.stack([c[j] for c in col]) for j in range(len(col[0]))])
            return torch.stack(list(col))

        super().__init__(stack(inputData), stack(targetData))
