"""Batch inference and the thread-safe prediction service.

Reference: S/optim/Predictor.scala:35-257 (distributed predict / predictClass / predictImage: batches are
spread over the ranks and gathered back in order),
LocalPredictor.scala:33-197, PredictionService.scala:56-354 (pool of model clones, ``predict(Activity)``
:79 and ``predict(bytes)`` :128 with (de)serialized activities).

On MI355X the "pool of clones" is a pool of replicas that share one copy of the weights, each with its own
HIP stream, so concurrent requests overlap on the device. ``predict(bytes)`` uses a small self-describing tensor wire format
(JSON header + raw little-endian payload) instead of the reference's protobuf Activity message.
"""
import torch

from ..dataset.core import AbstractDataSet, DataSet, MiniBatch, Sample, SampleToMiniBatch, samples_to_minibatch
from ..utils.table import Table


def _dist_world():
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist, dist.get_world_size(), dist.get_rank()
    return None, 1, 0


def _gather_ordered(dist, world, rank, mine, dev):
    """All-gather every rank's ``[(batch index, output)]`` and return the outputs of ALL batches in batch order
    (the reference's ordered ``mapPartitions(...).collect()``). Tensor outputs go through one padded tensor
    all-gather (RCCL on the GPU engine); Tables / other activities through ``all_gather_object``."""
    tensors = all(isinstance(o, torch.Tensor) for _, o in mine)
    flag = torch.tensor([1.0 if tensors else 0.0], device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if flag.item() < 1.0:
        got = [None] * world
        dist.all_gather_object(got, [(i, o.to("cpu") if hasattr(o, "to") else o) for i, o in mine])
        allb = sorted((b for g in got for b in g), key=lambda t: t[0])
        return [o for _, o in allb]
    # shapes / batch indices of every rank, then one all-gather of the concatenated (padded) payloads
    meta = [(i, tuple(o.shape), str(o.dtype).split(".")[-1]) for i, o in mine]
    metas = [None] * world
    dist.all_gather_object(metas, meta)
    dtype = next((getattr(torch, m[0][2]) for m in metas if m), torch.float32)
    flat = torch.cat([o.reshape(-1).to(dtype) for _, o in mine]) if mine else torch.empty(0, dtype=dtype)
    sizes = [sum(int(torch.Size(sh).numel()) for _, sh, _ in m) for m in metas]
    cap = max(sizes) if sizes else 0
    buf = torch.zeros(cap, dtype=dtype, device=dev)
    buf[:flat.numel()].copy_(flat.to(dev))
    out = torch.empty(world * cap, dtype=dtype, device=dev)
    dist.all_gather_into_tensor(out, buf)
    out = out.cpu()
    allb = []
    for r, m in enumerate(metas):
        off = r * cap
        for i, sh, _ in m:
            n = int(torch.Size(sh).numel())
            allb.append((i, out[off:off + n].reshape(sh)))
            off += n
    allb.sort(key=lambda t: t[0])
    return [o for _, o in allb]


class Predictor:
    """Batch inference (reference S/optim/Predictor.scala:152-180 + LocalPredictor.scala).

    Distributed (``torch.distributed`` initialised with more than one rank): the model is already replicated
    (every rank holds the broadcast weights), batch ``b`` of the input is predicted by rank ``b % world`` — the
    analogue of one Spark partition per executor — and the per-rank outputs are gathered back in input order on
    every rank. ``gather=False`` returns only this rank's outputs (``(batch index, output)`` pairs)."""

    def __init__(self, model, batchSize=-1, batchPerPartition=4):
        self.model = model
        self.batchSize = batchSize if batchSize and batchSize > 0 else 32 * batchPerPartition

    def _batches(self, data):
        if isinstance(data, torch.Tensor):
            for i in range(0, data.shape[0], self.batchSize):
                yield data[i:i + self.batchSize]
            return
        if isinstance(data, AbstractDataSet):
            it = data.data(train=False)
        else:
            it = iter(data)
        buf = []
        for s in it:
            if isinstance(s, MiniBatch):
                yield s.getInput()
                continue
            buf.append(s if isinstance(s, Sample) else Sample(s))
            if len(buf) == self.batchSize:
                yield samples_to_minibatch(buf).getInput()
                buf = []
        if buf:
            yield samples_to_minibatch(buf).getInput()

    def predict(self, data, gather=True):
        dist, world, rank = _dist_world()
        # a rank-sharded dataset (DataSet.rdd: rank r owns global elements r, r+world, ...) is already split:
        # predict the whole local shard and re-interleave the rows after the gather
        sharded = dist is not None and isinstance(data, AbstractDataSet) and data.isDistributed()
        was = self.model.isTraining()
        self.model.evaluate()
        dev = self.model.device
        mine = []
        with torch.no_grad():
            for b, x in enumerate(self._batches(data)):
                if not sharded and b % world != rank:
                    continue
                x = x.to(dev)
                y = self.model.forward(x)
                mine.append((b, y.float() if isinstance(y, torch.Tensor) else y))
        if was:
            self.model.training()
        if not gather:
            return [(b, y.cpu() if isinstance(y, torch.Tensor) else y) for b, y in mine]
        if dist is None:
            outs = [y.cpu() if isinstance(y, torch.Tensor) else y for _, y in mine]
        else:
            cdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
            if sharded:
                local = torch.cat([y for _, y in mine], 0) if mine else torch.empty(0)
                parts = _gather_ordered(dist, world, rank, [(rank, local)], cdev)
                n = sum(p.shape[0] for p in parts)
                out = torch.empty((n,) + tuple(parts[0].shape[1:]), dtype=parts[0].dtype)
                for r, p in enumerate(parts):
                    out[r::world][:p.shape[0]] = p
                return out
            outs = _gather_ordered(dist, world, rank, mine, cdev)
        if outs and isinstance(outs[0], torch.Tensor):
            return torch.cat(outs, 0)
        return outs

    def predictClass(self, data):
        out = self.predict(data)
        return out.argmax(dim=-1) + 1   # 1-based classes

    def predictImage(self, imageFrame, outputLayer=None, shareBuffer=False, batchPerPartition=4,
                     predictKey="predict"):
        feats = imageFrame.array()
        x = torch.stack([f.toTensor() for f in feats])
        out = self.predict(x)
        for f, o in zip(feats, out):
            f[predictKey] = o
        return imageFrame


LocalPredictor = Predictor


# ------------------------------------------------------------------------------------- wire format
# The reference's bytes protocol (S/optim/PredictionService.scala:178-280): an activity is one protobuf ``AttrValue``
# of bigdl.proto (utils/bigdl_proto.py schema) —
#   Tensor              -> AttrValue{dataType: TENSOR, tensorValue: BigDLTensor with its TensorStorage inline}
#   Table(key, Tensor)  -> AttrValue{dataType: ARRAY_VALUE, arrayValue{datatype: TENSOR, tensor: [isKeyPrimitive (BOOL
#                          scalar), keys..., values...]}}, a primitive key as a scalar tensor of its type
# and a failure comes back as a STRING scalar tensor ("Exception caught during [stage]! ..."), which decodes to a str.
def _bigdl_tensor(x):
    """BigDLTensor dict (storage included) of a torch tensor, or of a str / Python scalar key (a scalar tensor)."""
    from ..utils import bigdl_proto as bp

    if isinstance(x, str):
        return {"datatype": ["STRING"], "size": [], "stride": [], "offset": [1], "dimension": [0], "nElements": [1],
                "isScalar": [True], "storage": [{"datatype": ["STRING"], "string_data": [x], "id": [1]}], "id": [1],
                "tensorType": ["DENSE"]}
    if isinstance(x, bool):
        x = torch.tensor(x)
    elif isinstance(x, int):
        x = torch.tensor(x, dtype=torch.int32 if -(1 << 31) <= x < (1 << 31) else torch.int64)
    elif isinstance(x, float):
        x = torch.tensor(x, dtype=torch.float32)
    if not isinstance(x, torch.Tensor):
        raise TypeError(f"PredictionService: unsupported activity element {type(x).__name__}")
    x = x.detach().cpu()
    if x.dtype in (torch.uint8, torch.int8):
        x = x.to(torch.int32)
    ctx = bp._SerCtx()
    tid = _one_id(bp._tensor_attr(x, ctx))
    return ctx.storages[tid]


def _one_id(d):
    return d["id"][0]


def serialize_activity(a):
    """Activity (Tensor, Table of tensors keyed by primitives or tensors, or an error message str) -> bytes of a
    bigdl.proto ``AttrValue`` (PredictionService.serializeActivity)."""
    from ..utils import bigdl_proto as bp

    if isinstance(a, Table):
        items = list(a.items())
        if not items:
            raise ValueError("PredictionService: cannot serialize an empty Table")
        prim = not isinstance(items[0][0], torch.Tensor)
        tensors = [_bigdl_tensor(torch.tensor(prim))] + [_bigdl_tensor(k) for k, _ in items] + \
                  [_bigdl_tensor(v) for _, v in items]
        attr = {"dataType": ["ARRAY_VALUE"],
                "arrayValue": [{"size": [len(tensors)], "datatype": ["TENSOR"], "tensor": tensors}]}
    elif isinstance(a, (torch.Tensor, str)):
        attr = {"dataType": ["TENSOR"], "tensorValue": [_bigdl_tensor(a)]}
    else:
        raise TypeError(f"PredictionService: unsupported activity type {type(a).__name__}")
    return bp.SCHEMA.encode("AttrValue", attr)


def _tensor_of(d):
    from ..utils import bigdl_proto as bp

    st = bp._one(d, "storage", {})
    if bp._one(d, "datatype") == "STRING" or bp._one(st, "datatype") == "STRING":
        vals = st.get("string_data", [])
        return vals[0] if len(vals) == 1 else list(vals)
    return bp._tensor_from(d, bp._LoadCtx({}))


def deserialize_activity(b):
    """bytes of a bigdl.proto ``AttrValue`` -> Tensor / Table (PredictionService.deSerializeActivity); a STRING tensor
    (the error Activity) decodes to its str."""
    from ..utils import bigdl_proto as bp

    attr = bp.SCHEMA.decode("AttrValue", bytes(b))
    dt = bp._one(attr, "dataType")
    if dt == "ARRAY_VALUE":
        ts = [_tensor_of(t) for t in bp._one(attr, "arrayValue", {}).get("tensor", [])]
        n = (len(ts) - 1) // 2
        prim = bool(ts[0].item()) if isinstance(ts[0], torch.Tensor) else bool(ts[0])
        keys = [(k.item() if isinstance(k, torch.Tensor) else k) if prim else k for k in ts[1:n + 1]]
        out = Table()
        for k, v in zip(keys, ts[n + 1:]):
            out[k] = v
        return out
    if dt == "TENSOR" or "tensorValue" in attr:
        return _tensor_of(bp._one(attr, "tensorValue", {}))
    raise ValueError(f"PredictionService: unsupported AttrValue dataType {dt}")


def _error_activity(stage, e):
    """The reference's errorTensor: a STRING scalar naming the stage and the exception."""
    import traceback

    return f"Exception caught during [{stage}]! \n{e}\n" + "".join(traceback.format_tb(e.__traceback__)[-3:])


def _share_weights(src, dst):
    """Point the parameters and buffers of the clone ``dst`` at the tensors of ``src`` (replicas differ only in
    their activation buffers)."""
    for a, b in zip(src.flattened_layers(), dst.flattened_layers()):
        for w, _ in getattr(a, "_params", ()):
            t = getattr(a, w, None)
            if t is not None:
                setattr(b, w, t)
        for name in getattr(a, "_buffers", ()):
            t = getattr(a, name, None)
            if t is not None:
                setattr(b, name, t)


class PredictionService:
    """Thread-safe serving (reference PredictionService.scala:56-354): a pool of ``numThreads`` model replicas
    sharing one copy of the weights; on the GPU each replica owns a HIP stream, so concurrent requests run
    concurrently on the device instead of queueing behind one lock."""

    def __init__(self, model, numThreads=1):
        import queue

        self.model = model.evaluate()
        self.numThreads = max(1, int(numThreads))
        dev = getattr(self.model, "device", torch.device("cpu"))
        self._pool = queue.Queue()
        for i in range(self.numThreads):
            m = self.model
            if i > 0:
                m = self.model.cloneModule()
                _share_weights(self.model, m)
                m.evaluate()
            stream = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
            self._pool.put((m, stream))

    def predict(self, request):
        """Activity in, Activity out; or bigdl.proto ``AttrValue`` bytes in, bytes out (the reference's protocol,
        PredictionService.scala:113-160). Failures come back as the reference's error Activity (a STRING scalar)
        instead of raising."""
        if isinstance(request, (bytes, bytearray, memoryview)):
            try:
                act = deserialize_activity(bytes(request))
            except Exception as e:
                return serialize_activity(_error_activity("DeSerialize Input", e))
            out = self._run(act)
            try:
                return serialize_activity(out)
            except Exception as e:
                return serialize_activity(_error_activity("Serialize Output", e))
        return self._run(request)

    def _run(self, act):
        import contextlib

        model, stream = self._pool.get()
        try:
            dev = getattr(model, "device", torch.device("cpu"))
            ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
            try:
                with ctx, torch.no_grad():
                    act = act.to(dev) if hasattr(act, "to") else act
                    out = model.forward(act)
            except Exception as e:      # the reference returns its error Activity (PredictionService.scala:84-87)
                return _error_activity("running forward", e)
            try:
                return out.float().cpu() if isinstance(out, torch.Tensor) else out.to("cpu")
            except Exception as e:
                return _error_activity("Clone Result", e)
        finally:
            self._pool.put((model, stream))
