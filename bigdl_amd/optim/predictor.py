"""Batch inference and the thread-safe prediction service.

Reference: S/optim/Predictor.scala:35-257 (distributed predict / predictClass / predictImage),
LocalPredictor.scala:33-197, PredictionService.scala:56-354 (pool of model clones, ``predict(Activity)``
:79 and ``predict(bytes)`` :128 with (de)serialized activities).

On MI355X the "pool of clones" is one resident model per GPU plus a lock-protected request path; requests
are batched on the device stream. ``predict(bytes)`` uses a small self-describing tensor wire format
(JSON header + raw little-endian payload) instead of the reference's protobuf Activity message.
"""
import io
import json
import struct
import threading

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


class PredictionService:
    """Thread-safe serving of one model (reference PredictionService.scala:56-354)."""

    def __init__(self, model, numThreads=1):
        self.model = model.evaluate()
        self._lock = threading.Lock()
        self.numThreads = numThreads

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
        dev = self.model.device
        act = act.to(dev) if hasattr(act, "to") else act
        with self._lock, torch.no_grad():
            out = self.model.forward(act)
            if isinstance(out, torch.Tensor):
                return out.float().cpu()
            return out.to("cpu")
