"""Batch inference and the thread-safe prediction service.

Reference: S/optim/Predictor.scala:35-257 (distributed predict / predictClass / predictImage),
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


class Predictor:
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

    def predict(self, data):
        was = self.model.isTraining()
        self.model.evaluate()
        dev = self.model.device
        outs = []
        with torch.no_grad():
            for x in self._batches(data):
                x = x.to(dev) if isinstance(x, torch.Tensor) else x.to(dev)
                y = self.model.forward(x)
                outs.append(y.float().cpu() if isinstance(y, torch.Tensor) else y)
        if was:
            self.model.training()
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
