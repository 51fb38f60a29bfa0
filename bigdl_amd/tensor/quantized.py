"""QuantizedTensor: an int8 tensor quantized symmetrically per row, the weight container of the int8 layers.

Reference: S/tensor/QuantizedTensor.scala:26-305 (size / stride / nElement, per-row max / min / sum, ``set`` sharing
the storage and descriptor, ``copy`` deep-copying them, ``release`` freeing the native buffer, equality and hashing
over sizes and bytes) and S/nn/quantized/Quantization.scala:35-120 (``q = round(x / max(|max|, |min|) * 127)`` with
Java's round-half-up, per row of the 2-D view [size(1), prod(rest)]).

MI355X mapping: the bytes live in a torch int8 tensor that can sit on the device (``to("cuda")``) — the "native
descriptor" of the reference is that device buffer, which the i8-MFMA kernels of csrc/quant.hip read directly; the
per-row threshold ``max(|max|, |min|) / 127`` is the dequantisation scale their epilogue applies.
"""
import torch

QMAX = 127.0


def _round_half_up(x):
    return torch.floor(x + 0.5)


def _rows(t):
    t = torch.as_tensor(t)
    if t.dim() == 0:
        raise ValueError("QuantizedTensor needs at least one dimension")
    return t.reshape(1, -1) if t.dim() == 1 else t.reshape(t.shape[0], -1)


def _contig_strides(size):
    st, acc = [], 1
    for s in reversed(size):
        st.append(acc)
        acc *= s
    return list(reversed(st))


class QuantizedTensor:
    """int8 data + per-row ``maxOfRow`` / ``minOfRow`` / ``sumOfRow`` (fp32). Dimensions are 1-based like the rest of
    the Tensor API. ``params`` carries the layer descriptor parameters (an opaque dict, kept for parity)."""

    def __init__(self, src=None, params=None, size=None):
        self.params = dict(params or {})
        self._data = None
        self.maxOfRow = self.minOfRow = self.sumOfRow = None
        if src is not None:
            t = src.to_torch() if hasattr(src, "to_torch") else torch.as_tensor(src)
            self._size = list(t.shape)
            self._quantize(t)
        else:
            self._size = list(size or [])
        self._stride = _contig_strides(self._size)

    # ---------------------------------------------------------------- construction
    def _quantize(self, t):
        rows = _rows(t).float()
        mx, mn = rows.amax(dim=1), rows.amin(dim=1)
        thr = torch.maximum(mx.abs(), mn.abs())
        inv = torch.where(thr > 0, QMAX / thr, torch.zeros_like(thr))
        q = _round_half_up(rows * inv[:, None]).clamp_(-128, 127).to(torch.int8)
        self._data = q.reshape(t.shape).contiguous()
        self.maxOfRow, self.minOfRow, self.sumOfRow = mx, mn, rows.sum(dim=1)

    @classmethod
    def from_bytes(cls, data, maxOfRow, minOfRow, sumOfRow, size, params=None):
        """Reference QuantizedTensor(src: Array[Byte], max, min, sum, size, params)."""
        data = torch.as_tensor(data, dtype=torch.int8)
        size = list(size)
        n = 1
        for s in size:
            n *= s
        if data.numel() != n:
            raise ValueError(f"size mismatch: {data.numel()} bytes for shape {size}")
        qt = cls(params=params, size=size)
        qt._data = data.reshape(size).contiguous()
        qt.maxOfRow = torch.as_tensor(maxOfRow, dtype=torch.float32)
        qt.minOfRow = torch.as_tensor(minOfRow, dtype=torch.float32)
        qt.sumOfRow = torch.as_tensor(sumOfRow, dtype=torch.float32) if sumOfRow is not None else None
        return qt

    @classmethod
    def from_scaled(cls, q, scale, params=None):
        """View an int8 weight quantized symmetrically with per-row ``scale`` (= threshold / 127) as a
        QuantizedTensor sharing its bytes (what the quantized layers hold)."""
        thr = torch.as_tensor(scale, dtype=torch.float32) * QMAX
        qt = cls(params=params, size=list(q.shape))
        qt._data = q
        qt.maxOfRow, qt.minOfRow = thr, -thr
        qt.sumOfRow = _rows(q).float().sum(dim=1) * (thr / QMAX).to(q.device)
        return qt

    # ---------------------------------------------------------------- Tensor-API surface
    def getTensorType(self):
        return "QuantizedType"

    def dim(self):
        return len(self._size)

    nDimension = property(dim)

    def size(self, dim=None):
        if dim is None:
            return list(self._size)
        if not 1 <= dim <= len(self._size):
            raise ValueError(f"dimension {dim} out of range of {len(self._size)}D tensor")
        return self._size[dim - 1]

    def stride(self, dim=None):
        if dim is None:
            return list(self._stride)
        if not 1 <= dim <= len(self._size):
            raise ValueError(f"dimension {dim} out of range of {len(self._size)}D tensor")
        return self._stride[dim - 1]

    def nElement(self):
        if not self._size:
            return 0
        n = 1
        for s in self._size:
            n *= s
        return n

    def getStorage(self):
        """The int8 bytes (flat), on whatever device they live."""
        return None if self._data is None else self._data.reshape(-1)

    def getNativeStorage(self):
        """The device-resident buffer the int8 kernels read (the reference's native descriptor)."""
        return self._data

    def threshold(self):
        return torch.maximum(self.maxOfRow.abs(), self.minOfRow.abs())

    def scale(self):
        """Per-row dequantisation scale, threshold / 127."""
        return self.threshold() / QMAX

    def dequantize(self):
        rows = _rows(self._data).float()
        thr = self.threshold().to(rows.device)
        return (rows / QMAX * thr[:, None]).reshape(self._size)

    def to(self, device):
        self._data = self._data.to(device) if self._data is not None else None
        for n in ("maxOfRow", "minOfRow", "sumOfRow"):
            v = getattr(self, n)
            if v is not None:
                setattr(self, n, v.to(device))
        return self

    def cuda(self):
        return self.to("cuda")

    def cpu(self):
        return self.to("cpu")

    def release(self):
        """Drop the buffer (reference frees the BigQuant descriptor); sizes stay."""
        self._data = None
        return self

    def set(self, other=None):
        """set(): empty this tensor; set(other): share other's bytes, row statistics, params and shape."""
        if other is None:
            self._data = None
            self.maxOfRow = self.minOfRow = self.sumOfRow = None
            return self
        if not isinstance(other, QuantizedTensor):
            raise TypeError("can't set from other type of tensor")
        self._data, self.params = other._data, other.params
        self.maxOfRow, self.minOfRow, self.sumOfRow = other.maxOfRow, other.minOfRow, other.sumOfRow
        self._size, self._stride = list(other._size), list(other._stride)
        return self

    def copy(self, other):
        """Deep copy of another QuantizedTensor of the same shape (new storage)."""
        if not isinstance(other, QuantizedTensor) or other.size() != self.size():
            raise TypeError("can't copy from other type or shape of tensor")
        self._data = other._data.clone()
        self.params = dict(other.params)
        self.maxOfRow, self.minOfRow = other.maxOfRow.clone(), other.minOfRow.clone()
        self.sumOfRow = other.sumOfRow.clone() if other.sumOfRow is not None else None
        return self

    def __eq__(self, other):
        if not isinstance(other, QuantizedTensor):
            return False
        if other is self:
            return True
        if self._size != other._size:
            return False
        if self._data is None or other._data is None:
            return self._data is None and other._data is None
        return bool(torch.equal(self._data.cpu(), other._data.cpu()))

    def __hash__(self):
        h = 1
        h = h * 37 + self.dim()
        for s in self._size:
            h = h * 37 + s
        if self._data is not None:
            h = h * 37 + hash(self._data.cpu().numpy().tobytes())
        return h & 0xFFFFFFFF

    # ---------------------------------------------------------------- persistence
    def state_dict(self):
        out = {"data": self._data.cpu(), "max": self.maxOfRow.cpu(), "min": self.minOfRow.cpu()}
        if self.sumOfRow is not None:
            out["sum"] = self.sumOfRow.cpu()
        return out

    @classmethod
    def from_state_dict(cls, sd, params=None):
        return cls.from_bytes(sd["data"], sd["max"], sd["min"], sd.get("sum"), list(sd["data"].shape), params)

    def __repr__(self):
        return f"QuantizedTensor(size={self._size}, device={None if self._data is None else self._data.device})"


__all__ = ["QuantizedTensor"]
