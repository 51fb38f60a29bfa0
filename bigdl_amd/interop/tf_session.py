"""TensorFlow sessions: training / prediction of imported graphs fed by their own TF input pipelines, and
TensorFlow-variable checkpoints.

Reference: S/utils/tf/Session.scala:54-182 (BigDLSessionImpl: ``train(endPoints, optMethod, endWhen, isDataBatch,
batchSize, sc, loss)`` over graphs whose input is a queue / reader op — inputOp = ReaderReadV2, QueueDequeueV2,
QueueDequeueManyV2, Placeholder — with the input sub-graph (filename queues, TFRecord / fixed-length readers,
enqueue ops) evaluated to produce the data set; ``predict``; ``saveParameters``), TensorflowLoader.checkpoints /
loadBinFiles / saveBinFile (TensorflowLoader.scala:88-172: a session whose variables come from a name -> tensor
file) and S/nn/Module.scala:108 (``Module.tensorflowCheckpoints``).

Design. The graph is cut at the data boundary: the queue dequeue op that feeds the model. Everything upstream —
filename queues, TFRecordReaderV2 / FixedLengthRecordReaderV2, ParseSingleExample / ParseExample, DecodeRaw,
Cast / Reshape / arithmetic — is the host-side input pipeline and is evaluated per record by a small NodeDef
interpreter (``_HostPipeline``), producing Samples (one feature per dequeued component). Everything downstream,
from the dequeued tensors to the loss, is converted by the regular TensorFlow loader into an nn.Graph that runs
on the device engine. Gradients come from that graph's backward (the engine differentiates the imported forward
graph), so TensorFlow's generated gradient / Apply* update sub-graph is not executed; the OptimMethod updates the
parameters. Variables (VariableV2 + Assign initialisers) take their values from the session's ``context`` when
present (a checkpoint bin file), and ``saveParameters`` writes the trained values back under the variable names.
"""
import os
import struct

import numpy as np
import torch

from .. import nn
from ..nn.tf_ops import MULTI_OUTPUT, OPS, run_op
from ..utils.table import Table
from .tensorflow import _split_ref, attrs_of, load_tf, read_graph

DEQUEUE = ("QueueDequeueV2", "QueueDequeueManyV2", "QueueDequeueUpToV2")
ENQUEUE = ("QueueEnqueueV2", "QueueEnqueueManyV2")
READERS = ("TFRecordReaderV2", "FixedLengthRecordReaderV2")
_NP = {"DT_FLOAT": np.float32, "DT_DOUBLE": np.float64, "DT_INT32": np.int32, "DT_INT64": np.int64,
       "DT_UINT8": np.uint8, "DT_INT8": np.int8, "DT_INT16": np.int16, "DT_UINT16": np.uint16}


# ---------------------------------------------------------------------------------------------- record files
def tfrecord_iterator(path):
    """Records of a TFRecord file (length, masked CRC32C of the length, data, masked CRC32C of the data)."""
    from ..visualization.tensorboard import read_records

    return read_records(path)


def write_tfrecords(path, records):
    from ..visualization.tensorboard import masked_crc32c

    with open(path, "wb") as f:
        for rec in records:
            ln = struct.pack("<Q", len(rec))
            f.write(ln + struct.pack("<I", masked_crc32c(ln)) + rec + struct.pack("<I", masked_crc32c(rec)))


def fixed_length_records(path, header_bytes, record_bytes, footer_bytes=0, hop_bytes=0):
    """Reference FixedLengthRecordReader.scala: skip the header, then records of record_bytes every hop_bytes
    (record_bytes when 0) up to the footer."""
    with open(path, "rb") as f:
        data = f.read()
    end = len(data) - footer_bytes
    step = hop_bytes or record_bytes
    pos = header_bytes
    while pos + record_bytes <= end:
        yield data[pos:pos + record_bytes]
        pos += step


# ---------------------------------------------------------------------------------------------- host pipeline
def _bytes(v):
    if isinstance(v, (bytes, bytearray)):
        return bytes(v)
    if isinstance(v, list) and len(v) == 1:
        return _bytes(v[0])
    if isinstance(v, str):
        return v.encode()
    raise TypeError(f"expected a string scalar, got {type(v)}")


class _HostPipeline:
    """Evaluates input-pipeline NodeDefs on the host (string / record tensors, parsing, decoding)."""

    def __init__(self, nodes):
        self.nodes = {n["name"][0]: n for n in nodes}
        self.consumers = {}
        for n in nodes:
            for r in n.get("input", []):
                ref = _split_ref(r)
                if ref is not None:
                    self.consumers.setdefault(ref[0], []).append(n["name"][0])

    def op(self, name):
        return self.nodes[name]["op"][0]

    def ins(self, name):
        return [r for r in (_split_ref(x) for x in self.nodes[name].get("input", [])) if r is not None]

    def eval(self, ref, feeds, memo):
        name, port = ref
        if (name, port) in feeds:
            return feeds[(name, port)]
        key = (name, port)
        if key in memo:
            return memo[key]
        if name in memo and isinstance(memo[name], list):
            return memo[name][port]
        op, at = self.op(name), attrs_of(self.nodes[name])
        xs = lambda: [self.eval(r, feeds, memo) for r in self.ins(name)]  # noqa: E731
        if op == "Const":
            v = at.get("value")
        elif op in ("Identity", "StopGradient", "Snapshot"):
            v = xs()[0]
        elif op in ("ParseSingleExample", "ParseExample"):
            v = self._parse(op, at, xs())
            memo[name] = v
            return v[port]
        elif op == "DecodeRaw":
            buf = xs()[0]
            dt = _NP.get(at.get("out_type", "DT_UINT8"), np.uint8)
            dt = np.dtype(dt).newbyteorder("<" if at.get("little_endian", True) else ">")
            bufs = buf if isinstance(buf, list) and len(buf) > 1 else [_bytes(buf)]
            arrs = [np.frombuffer(b, dtype=dt).astype(dt.newbyteorder("=")) for b in bufs]
            v = torch.from_numpy(np.stack(arrs) if len(arrs) > 1 else arrs[0].copy())
        elif op in OPS:
            r = run_op(op, xs(), at)
            if op in MULTI_OUTPUT or isinstance(r, (list, tuple)):
                memo[name] = list(r)
                return memo[name][port]
            v = r
        else:
            raise NotImplementedError(f"input pipeline op {op} ({name}) is not supported on the host")
        memo[key] = v
        return v

    @staticmethod
    def _parse(op, at, xs):
        from ..nn.tf import _KIND_DTYPE, _parse_example_proto

        dense_keys = at.get("dense_keys") or []
        shapes = at.get("dense_shapes") or [[] for _ in dense_keys]
        n_sparse = int(at.get("num_sparse", at.get("Nsparse", 0)) or 0)
        if n_sparse:
            raise NotImplementedError("sparse features are not supported (the reference parses dense only)")
        if op == "ParseSingleExample":
            serialized, defaults = [_bytes(xs[0])], xs[1:1 + len(dense_keys)]
        else:   # ParseExample: serialized[batch], names, sparse_keys..., dense_keys..., dense_defaults...
            serialized = [_bytes(s) for s in xs[0]] if isinstance(xs[0], list) else [_bytes(xs[0])]
            defaults = xs[2 + 2 * len(dense_keys) - len(dense_keys):][:len(dense_keys)]
        parsed = [_parse_example_proto(s) for s in serialized]
        outs = []
        for i, k in enumerate(dense_keys):
            rows = []
            for p in parsed:
                if k in p:
                    kind, vals = p[k]
                    rows.append(torch.tensor(vals, dtype=_KIND_DTYPE.get(kind, torch.float32)) if kind != "bytes"
                                else vals)
                else:
                    rows.append(torch.as_tensor(defaults[i]))
            shape = list(shapes[i]) if i < len(shapes) and shapes[i] is not None else []
            t = [r.reshape(shape) if isinstance(r, torch.Tensor) else r for r in rows]
            outs.append(t[0] if op == "ParseSingleExample" else
                        (torch.stack(t) if isinstance(t[0], torch.Tensor) else t))
        return outs

    # -- queues and readers
    def enqueues_of(self, queue):
        return [n for n in self.consumers.get(queue, []) if self.op(n) in ENQUEUE and self.ins(n)[0][0] == queue]

    def queue_elements(self, queue, memo=None):
        """Every element enqueued into ``queue`` (its enqueue ops evaluated over all their input records), as
        lists of components."""
        out = []
        for e in self.enqueues_of(queue):
            comps = self.ins(e)[1:]
            reader = self._upstream_reader(e)
            many = self.op(e) == "QueueEnqueueManyV2"
            if reader is None:
                vals = [self.eval(c, {}, {}) for c in comps]
                out.extend(_unbatch(vals) if many else [vals])
                continue
            for key, value in self.read(reader):
                feeds = {(reader, 0): [key], (reader, 1): [value]}
                vals = [self.eval(c, feeds, {}) for c in comps]
                out.extend(_unbatch(vals) if many else [vals])
        return out

    def _upstream_reader(self, name, seen=None):
        seen = seen if seen is not None else set()
        if name in seen:
            return None
        seen.add(name)
        if self.op(name) == "ReaderReadV2":
            return name
        for r in self.ins(name):
            got = self._upstream_reader(r[0], seen)
            if got is not None:
                return got
        return None

    def read(self, read_node):
        """(key, value) records of a ReaderReadV2: the files come from its filename queue."""
        reader, queue = self.ins(read_node)[0][0], self.ins(read_node)[1][0]
        files = []
        for comps in self.queue_elements(queue):
            f = comps[0]
            files.extend([_bytes(x).decode() for x in f] if isinstance(f, list) and len(f) > 1 else
                         [_bytes(f).decode()])
        rop, at = self.op(reader), attrs_of(self.nodes[reader])
        for path in files:
            if rop == "TFRecordReaderV2":
                it = tfrecord_iterator(path)
            elif rop == "FixedLengthRecordReaderV2":
                it = fixed_length_records(path, int(at.get("header_bytes", 0)), int(at["record_bytes"]),
                                          int(at.get("footer_bytes", 0)), int(at.get("hop_bytes", 0)))
            else:
                raise NotImplementedError(f"reader {rop}")
            for i, rec in enumerate(it):
                yield f"{path}:{i}".encode(), rec


def _unbatch(vals):
    n = len(vals[0]) if isinstance(vals[0], list) else vals[0].shape[0]
    return [[v[i] for v in vals] for i in range(n)]


# ---------------------------------------------------------------------------------------------- session
class _LossOutput(nn.AbstractCriterion):
    """The model's output IS the loss (reference BigDLSessionImpl.FakeCriterion): loss = mean(output), gradient 1."""

    def updateOutput(self, input, target):
        self.output = input.float().mean()
        return self.output

    def updateGradInput(self, input, target):
        self.gradInput = torch.full_like(input, 1.0 / max(input.numel(), 1))
        return self.gradInput


class BigDLSession:
    """Session over a TensorFlow GraphDef (file path or parsed node list) with an optional variable context
    (name -> tensor, e.g. from a checkpoint bin file)."""

    def __init__(self, graph, inputs=None, context=None):
        self.nodes = read_graph(graph) if isinstance(graph, str) else list(graph)
        self.graph_file = graph if isinstance(graph, str) else None
        self.inputs = list(inputs or [])
        self.context = dict(context or {})
        self.host = _HostPipeline(self.nodes)
        self._model = None
        self._bindings = []

    # -- model construction
    def _input_node(self, endpoints):
        found, stack, seen = [], [e.split(":")[0] for e in endpoints], set()
        while stack:
            n = stack.pop()
            if n in seen or n not in self.host.nodes:
                continue
            seen.add(n)
            if self.host.op(n) in DEQUEUE + ("Placeholder",):
                found.append(n)
                continue
            stack.extend(r[0] for r in self.host.ins(n))
        if len(found) != 1:
            raise ValueError(f"expected exactly one input (queue dequeue / placeholder) op, found {sorted(found)}")
        return found[0]

    def _build(self, inp, outputs):
        from .tensorflow import _Loader

        loader = _Loader(self.nodes, [inp], outputs)
        loader.context = self.context
        model = loader.build()
        self._bindings = loader.var_bindings
        return model

    def _samples(self, inp, is_batch):
        op = self.host.op(inp)
        if op not in DEQUEUE:
            raise ValueError(f"{inp} ({op}) is not a queue dequeue: feed placeholders through a DataSet")
        from ..dataset.core import Sample

        elems = self.host.queue_elements(self.host.ins(inp)[0][0])
        if is_batch:                # each enqueued element is already a batch: split it into samples
            elems = [e for el in elems for e in _unbatch(el)]
        return [Sample([torch.as_tensor(c).float() if torch.as_tensor(c).is_floating_point() else torch.as_tensor(c)
                        for c in comps], torch.zeros(1)) for comps in elems]

    # -- API
    def train(self, outputs, dataset=None, optMethod=None, criterion=None, endWhen=None, batchSize=None,
              isDataBatch=False, loss=None):
        """``dataset`` given: placeholder-fed training with ``criterion`` (reference train(outputs, dataSet, ...)).
        Otherwise queue-fed: ``loss`` (or the single endpoint) is a scalar loss node computed from the dequeued
        input; the data set is produced by the graph's own input pipeline."""
        from ..dataset.core import DataSet
        from ..optim import Optimizer, Trigger

        if dataset is not None:
            inp = self.inputs[0] if self.inputs else self._input_node(outputs)
            model = self._build(inp, outputs)
            opt = Optimizer(model=model, dataset=dataset, criterion=criterion, batchSize=batchSize)
        else:
            target = loss or outputs[0]
            inp = self._input_node([target])
            model = self._build(inp, [target])
            data = self._samples(inp, isDataBatch)
            opt = Optimizer(model=model, dataset=DataSet.array(data), criterion=_LossOutput(),
                            batchSize=batchSize or 32)
        opt.setOptimMethod(optMethod).setEndWhen(endWhen or Trigger.maxEpoch(1))
        self._model = opt.optimize()
        return self._model

    def predict(self, endPoints, isDataBatch=False, batchSize=32):
        """Run ``endPoints`` over the graph's own input pipeline (queue-fed) and return the stacked outputs."""
        inp = self._input_node(endPoints)
        model = self._model if self._model is not None else self._build(inp, endPoints)
        model.evaluate()
        data = self._samples(inp, isDataBatch)
        outs = []
        with torch.no_grad():
            for i in range(0, len(data), batchSize):
                chunk = data[i:i + batchSize]
                x = Table()
                for k in range(chunk[0].numFeature()):
                    x[k + 1] = torch.stack([s.feature(k) for s in chunk])
                outs.append(model.forward(x[1] if chunk[0].numFeature() == 1 else x))
        return torch.cat([o.float().reshape(o.shape[0], -1) if o.dim() else o.reshape(1, 1) for o in outs])

    def variables(self):
        """Current value of every variable bound to a model parameter (TF layout), name -> tensor."""
        out = {}
        for name, mod, attr, layout in self._bindings:
            t = getattr(mod, attr).detach().float().cpu()
            out[name] = {"t": lambda x: x.t(), "hwio": lambda x: x.permute(2, 3, 1, 0)}.get(layout, lambda x: x)(t)
        return out

    def saveParameters(self, binFile):
        """Write the variables (trained values) as a name -> tensor file (reference saveBinFile)."""
        save_bin(binFile, {**self.context, **self.variables()})
        return self


def save_bin(path, tensors):
    from safetensors.torch import save_file

    save_file({k: v.contiguous().float() for k, v in tensors.items()}, path)


def load_bin(path):
    from safetensors.torch import load_file

    return dict(load_file(path))


def checkpoints(graphFile, binFile, byteOrder=None):
    """Reference TensorflowLoader.checkpoints / Module.tensorflowCheckpoints: a session over ``graphFile`` whose
    variables take the values stored in ``binFile``."""
    return BigDLSession(graphFile, context=load_bin(binFile))


__all__ = ["BigDLSession", "checkpoints", "save_bin", "load_bin", "tfrecord_iterator", "write_tfrecords",
           "fixed_length_records"]
