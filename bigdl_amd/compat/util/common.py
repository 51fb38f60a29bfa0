"""``bigdl.util.common`` for bigdl_amd (reference P/util/common.py:46-735).

The reference reaches a JVM through py4j and distributes work as Spark RDDs. Here the engine is in-process
and distributed over ``torch.distributed`` ranks, so:
  * ``SparkContext`` / ``RDD`` are a small local stand-in (``parallelize``, ``map``, ``zip``, ``collect``, ...)
    so reference scripts that build ``RDD[Sample]`` run unchanged; an RDD handed to an Optimizer becomes a
    rank-sharded ``DataSet.rdd`` (each rank of the job owns every world-th record);
  * ``init_engine`` initialises the engine (and the process group when launched under torch.distributed.run);
  * ``Sample`` / ``JTensor`` keep numpy features and labels, converted to engine tensors on use.
"""
import os
import random
import tempfile

import numpy as np
import torch

from .._convert import to_numpy


class JTensor:
    """A dense (or COO sparse) ndarray carrier (reference JTensor: storage, shape, indices)."""

    def __init__(self, storage, shape, bigdl_type="float", indices=None):
        self.storage = np.asarray(storage, dtype=np.float32).reshape(-1)
        self.shape = np.asarray(shape, dtype=np.int32)
        self.indices = None if indices is None else np.asarray(indices, dtype=np.int32)
        self.bigdl_type = bigdl_type

    @classmethod
    def from_ndarray(cls, a_ndarray, bigdl_type="float"):
        if a_ndarray is None:
            return None
        a = np.asarray(a_ndarray)
        return cls(a.astype(np.float32).reshape(-1), a.shape, bigdl_type)

    @classmethod
    def sparse(cls, a_ndarray, i_ndarray, shape, bigdl_type="float"):
        return cls(np.asarray(a_ndarray), shape, bigdl_type, indices=np.asarray(i_ndarray))

    def to_ndarray(self):
        if self.indices is None:
            return self.storage.reshape(tuple(int(s) for s in self.shape))
        dense = np.zeros(tuple(int(s) for s in self.shape), dtype=np.float32)
        idx = self.indices.reshape(len(self.shape), -1)
        dense[tuple(idx)] = self.storage
        return dense

    def to_torch(self):
        if self.indices is None:
            return torch.from_numpy(self.to_ndarray().copy())
        from ...tensor.tensor import SparseTensor

        return SparseTensor(torch.from_numpy(self.indices.reshape(len(self.shape), -1).astype(np.int64)),
                            torch.from_numpy(self.storage.copy()), [int(s) for s in self.shape])

    def __repr__(self):
        return f"JTensor: storage: {self.storage}, shape: {self.shape}" + \
            (f", indices: {self.indices}" if self.indices is not None else "")


class Sample:
    """A record of feature tensor(s) and label tensor(s) (reference Sample.from_ndarray :309)."""

    def __init__(self, features, labels, bigdl_type="float"):
        self.feature = features[0]
        self.features = features
        self.label = labels[0]
        self.labels = labels
        self.bigdl_type = bigdl_type

    @classmethod
    def from_ndarray(cls, features, labels, bigdl_type="float"):
        feats = [JTensor.from_ndarray(f) for f in (features if isinstance(features, list) else [features])]
        if isinstance(labels, list):
            labs = [JTensor.from_ndarray(l) for l in labels]
        else:
            labs = [JTensor.from_ndarray(np.asarray(labels, dtype=np.float32))]
        return cls(feats, labs, bigdl_type)

    @classmethod
    def from_jtensor(cls, features, labels, bigdl_type="float"):
        feats = features if isinstance(features, list) else [features]
        labs = labels if isinstance(labels, list) else [labels]
        return cls(feats, labs, bigdl_type)

    def to_engine(self):
        from ...dataset.core import Sample as ESample

        f = [j.to_torch() for j in self.features]
        l = [j.to_torch() for j in self.labels]
        return ESample(f[0] if len(f) == 1 else f, l[0] if len(l) == 1 else l)

    def __repr__(self):
        return f"Sample: features: {self.features}, labels: {self.labels}"


class EvaluatedResult:
    def __init__(self, result, total_num, method):
        self.result, self.total_num, self.method = result, total_num, method

    def __repr__(self):
        return f"Evaluated result: {self.result}, total_num: {self.total_num}, method: {self.method}"

    __str__ = __repr__


class RDD:
    """Local, eagerly materialised stand-in for a Spark RDD (the transformations reference scripts use)."""

    def __init__(self, items, num_slices=None):
        self._items = list(items)
        self.num_slices = num_slices or 1

    def map(self, f):
        return RDD([f(x) for x in self._items], self.num_slices)

    def flatMap(self, f):
        return RDD([y for x in self._items for y in f(x)], self.num_slices)

    def filter(self, f):
        return RDD([x for x in self._items if f(x)], self.num_slices)

    def zip(self, other):
        return RDD(list(zip(self._items, other._items)), self.num_slices)

    def zipWithIndex(self):
        return RDD([(x, i) for i, x in enumerate(self._items)], self.num_slices)

    def mapPartitions(self, f):
        return RDD(list(f(iter(self._items))), self.num_slices)

    def collect(self):
        return list(self._items)

    def count(self):
        return len(self._items)

    def take(self, n):
        return self._items[:n]

    def first(self):
        return self._items[0]

    def cache(self):
        return self

    persist = cache

    def unpersist(self):
        return self

    def repartition(self, n):
        return RDD(self._items, n)

    coalesce = repartition

    def getNumPartitions(self):
        return self.num_slices

    def union(self, other):
        return RDD(self._items + other._items, self.num_slices)

    def sample(self, withReplacement, fraction, seed=None):
        rnd = random.Random(seed)
        return RDD([x for x in self._items if rnd.random() < fraction], self.num_slices)

    def randomSplit(self, weights, seed=None):
        rnd = random.Random(seed)
        tot = float(sum(weights))
        cuts = np.cumsum([w / tot for w in weights])
        outs = [[] for _ in weights]
        for x in self._items:
            r = rnd.random()
            outs[int(np.searchsorted(cuts, r, side="right")) if r < cuts[-1] else len(weights) - 1].append(x)
        return [RDD(o, self.num_slices) for o in outs]

    def __iter__(self):
        return iter(self._items)

    def __len__(self):
        return len(self._items)


class SparkConf(dict):
    def set(self, k, v):
        self[k] = v
        return self

    def setAppName(self, name):
        return self.set("spark.app.name", name)

    def setMaster(self, master):
        return self.set("spark.master", master)

    def setAll(self, pairs):
        for k, v in pairs:
            self[k] = v
        return self

    def get(self, k, default=None):
        return dict.get(self, k, default)


class SparkContext:
    """Local SparkContext stand-in: ``parallelize`` builds an RDD; ``stop`` shuts the engine down."""

    _active = None

    def __init__(self, master=None, appName=None, conf=None, **kw):
        self.master = master or (conf.get("spark.master") if conf else None) or "local[1]"
        self.appName = appName
        self.conf = conf or SparkConf()
        SparkContext._active = self

    @classmethod
    def getOrCreate(cls, conf=None):
        return cls._active or cls(conf=conf)

    def parallelize(self, c, numSlices=None):
        return RDD(list(c), numSlices)

    def textFile(self, path, minPartitions=None):
        with open(path) as f:
            return RDD([l.rstrip("\n") for l in f], minPartitions)

    def broadcast(self, value):
        class _B:
            def __init__(self, v):
                self.value = v

        return _B(value)

    def stop(self):
        SparkContext._active = None

    @property
    def defaultParallelism(self):
        from ...utils.engine import Engine

        return Engine.world_size()


def init_engine(bigdl_type="float"):
    """Reference init_engine (:420): initialise the engine; under torch.distributed.run (WORLD_SIZE > 1) also
    the process group, one rank per GPU."""
    from ...utils.engine import Engine

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if not Engine.isInitialized():
        Engine.init(master=f"local[{world}]", dist=world > 1)
    return Engine


def init_executor_gateway(sc, bigdl_type="float"):
    return None


def get_node_and_core_number(bigdl_type="float"):
    from ...utils.engine import Engine

    return Engine.nodeNumber(), Engine.coreNumber()


def redire_spark_logs(bigdl_type="float", log_path=None):
    import logging

    log_path = log_path or os.path.join(os.getcwd(), "bigdl.log")
    h = logging.FileHandler(log_path)
    logging.getLogger("bigdl_amd").addHandler(h)


def show_bigdl_info_logs(bigdl_type="float"):
    import logging

    logging.getLogger("bigdl_amd").setLevel(logging.INFO)


def get_bigdl_conf():
    return {"spark.shuffle.reduceLocality.enabled": "false", "spark.shuffle.blockTransferService": "nio",
            "spark.scheduler.minRegisteredResourcesRatio": "1.0", "spark.speculation": "false"}


def create_spark_conf():
    return SparkConf().setAll(get_bigdl_conf().items())


def get_spark_context(conf=None):
    return SparkContext.getOrCreate(conf or create_spark_conf())


def get_spark_sql_context(sc):
    return None


def to_list(a):
    if isinstance(a, list):
        return a
    return [a]


def to_sample_rdd(x, y, numSlices=None):
    """ndarrays (features, labels) -> RDD[Sample] (reference :481)."""
    return RDD([Sample.from_ndarray(np.asarray(f), np.asarray(l)) for f, l in zip(x, y)], numSlices)


def create_tmp_path():
    return tempfile.mkdtemp(prefix="bigdl")


def text_from_path(path):
    with open(path) as f:
        return f.read()


def get_local_file(a_path):
    return a_path


def is_distributed(path):
    return "://" in path


def get_activation_by_name(activation_name, activation_id=None):
    from ..nn import layer as L

    names = {"tanh": L.Tanh, "sigmoid": L.Sigmoid, "hard_sigmoid": L.HardSigmoid, "relu": L.ReLU,
             "softmax": L.SoftMax, "softplus": L.SoftPlus, "softsign": L.SoftSign, "linear": L.Identity}
    if activation_name not in names:
        raise Exception(f"Unsupported activation type: {activation_name}")
    act = names[activation_name]()
    if activation_id:
        act.set_name(activation_id)
    return act


class RNG:
    def __init__(self, bigdl_type="float"):
        self.bigdl_type = bigdl_type

    def set_seed(self, seed):
        from ...utils.random_generator import RNG as E

        E.setSeed(seed)

    def uniform(self, a, b, size):
        from ...utils.random_generator import RNG as E

        return to_numpy(E.uniform(a, b, tuple(size)) if hasattr(E, "uniform") else
                        torch.empty(tuple(size)).uniform_(a, b))


def samples_to_engine(data):
    """RDD / list of compat Samples (or (features, label) ndarray pairs) -> engine Samples."""
    out = []
    for s in data:
        if isinstance(s, Sample):
            out.append(s.to_engine())
        elif isinstance(s, tuple) and len(s) == 2:
            f = [np.asarray(a) for a in s[0]] if isinstance(s[0], list) else np.asarray(s[0])
            out.append(Sample.from_ndarray(f, np.asarray(s[1])).to_engine())
        else:
            out.append(s)
    return out


def to_engine_dataset(data, shuffle=True):
    """An RDD of Samples -> rank-sharded engine DataSet (reference: RDD partitions per executor)."""
    from ...dataset.core import AbstractDataSet, DataSet

    if isinstance(data, AbstractDataSet):
        return data
    return DataSet.rdd(samples_to_engine(data), shuffle=shuffle)


__all__ = ["JTensor", "Sample", "EvaluatedResult", "RDD", "SparkConf", "SparkContext", "init_engine",
           "init_executor_gateway", "get_node_and_core_number", "redire_spark_logs", "show_bigdl_info_logs",
           "get_bigdl_conf", "create_spark_conf", "get_spark_context", "get_spark_sql_context", "to_list",
           "to_sample_rdd", "create_tmp_path", "text_from_path", "get_local_file", "is_distributed",
           "get_activation_by_name", "RNG", "np"]
