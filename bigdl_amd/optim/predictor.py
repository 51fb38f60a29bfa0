"""Batch inference and the thread-safe prediction service.

Reference: S/optim/Predictor.scala:35-257 (distributed predict / predictClass / predictImage: batches are
spread over the ranks and gathered back in order),
LocalPredictor.scala:33-197, PredictionService.scala:56-354 (pool of model clones, ``predict(Activity)``
:79 and ``predict(bytes)`` :128 with (de)serialized activities).

On MI355X the "pool of clones" is a pool of replicas that share one copy of the weights, each with its own
HIP stream, so concurrent requests overlap on the device. ``predict(bytes)`` uses a small self-describing tensor wire format
(JSON header + raw little-endian payload) instead of the reference's protobuf Activity message.
"""
import io
import json
import struct

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
def serialize_activity(a):
    """Activity (Tensor or Table of tensors) -> bytes."""
    tensors, meta = [], []

    def enc(x):
        if isinstance(x, torch.Tensor):
            t = x.detach().cpu().contiguous()
            meta_t = {"t": "tensor", "dtype": str(t.dtype).split(".")[-1], "shape": list(t.shape), "i": len(tensors)}
            tensors.append(t)
            return meta_t
        if isinstance(x, Table):
            return {"t": "table", "items": [[k, enc(v)] for k, v in x.items()]}
        raise TypeError(type(x))

    header = json.dumps(enc(a)).encode()
    buf = io.BytesIO()
    buf.write(struct.pack("<I", len(header)))
    buf.write(header)
    for t in tensors:
        raw = t.view(torch.uint8).numpy().tobytes() if t.numel() else b""
        buf.write(struct.pack("<Q", len(raw)))
        buf.write(raw)
    return buf.getvalue()


def deserialize_activity(b):
    mv = memoryview(b)
    (hl,) = struct.unpack_from("<I", mv, 0)
    header = json.loads(bytes(mv[4:4 + hl]).decode())
    off = 4 + hl
    blobs = []
    while off < len(b):
        (n,) = struct.unpack_from("<Q", mv, off)
        off += 8
        blobs.append(bytes(mv[off:off + n]))
        off += n

    def dec(m):
        if m["t"] == "tensor":
            dt = getattr(torch, m["dtype"])
            raw = bytearray(blobs[m["i"]])
            t = torch.frombuffer(raw, dtype=torch.uint8) if raw else torch.empty(0, dtype=torch.uint8)
            return t.view(dt).reshape(m["shape"]).clone()
        t = Table()
        for k, v in m["items"]:
            t[k if not (isinstance(k, str) and k.isdigit()) else int(k)] = dec(v)
        return t

    return dec(header)


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
        if isinstance(request, (bytes, bytearray, memoryview)):
            try:
                act = deserialize_activity(bytes(request))
                out = self._run(act)
                return serialize_activity(out)
            except Exception as e:  # reference returns an error Activity instead of throwing
                return serialize_activity(Table(torch.tensor([0.0]), torch.tensor(list(str(e).encode()), dtype=torch.uint8)))
        return self._run(request)

    def _run(self, act):
        import contextlib

        model, stream = self._pool.get()
        try:
            dev = getattr(model, "device", torch.device("cpu"))
            ctx = torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()
            with ctx, torch.no_grad():
                act = act.to(dev) if hasattr(act, "to") else act
                out = model.forward(act)
                out = out.float().cpu() if isinstance(out, torch.Tensor) else out.to("cpu")
            return out
        finally:
            self._pool.put((model, stream))
