"""Shape / indexing / reduction layers (reference S/nn/*.scala: Reshape, View, InferReshape, Squeeze,
Unsqueeze, Transpose, Contiguous, Narrow, Select, Index, Replicate, Tile, ExpandSize, Padding,
SpatialZeroPadding, Cropping2D, Cropping3D, Reverse, MaskedSelect, Sum, Mean, Max, Min, UpSampling1D/2D/3D,
ResizeBilinear, Pack, Masking). All dimension arguments are 1-based, as in the reference; ``nInputDims`` /
batch-mode semantics follow the reference (an extra leading batch dim shifts positive dims by one).
"""
import torch
import torch.nn.functional as F

from .abstractnn import AutogradModule, TensorModule


def _bdim(dim, x, nInputDims):
    """1-based reference dim -> 0-based torch dim, honouring batch mode."""
    if dim < 0:
        return x.dim() + dim
    d = dim - 1
    if nInputDims is not None and nInputDims > 0 and x.dim() > nInputDims:
        d += 1
    return d


class Reshape(TensorModule):
    def __init__(self, size, batchMode=None):
        super().__init__()
        self.size = tuple(size)
        self.batchMode = batchMode
        n = 1
        for s in self.size:
            n *= s
        self.nElement = n

    def _target(self, x):
        if self.batchMode is True or (self.batchMode is None and x.numel() != self.nElement):
            return (x.shape[0],) + self.size
        return self.size

    def updateOutput(self, input):
        return input.reshape(self._target(input))

    def updateGradInput(self, input, gradOutput):
        return gradOutput.reshape(input.shape)


class View(TensorModule):
    def __init__(self, *sizes):
        super().__init__()
        if len(sizes) == 1 and isinstance(sizes[0], (list, tuple)):
            sizes = tuple(sizes[0])
        self.sizes = tuple(sizes)
        self.numInputDims = None

    def setNumInputDims(self, n):
        self.numInputDims = n
        return self

    def updateOutput(self, input):
        if self.numInputDims is not None and input.dim() > self.numInputDims:
            lead = input.shape[: input.dim() - self.numInputDims]
            return input.reshape(tuple(lead) + self.sizes)
        n = 1
        for s in self.sizes:
            n *= s if s > 0 else 1
        if -1 not in self.sizes and input.numel() != n:
            return input.reshape((-1,) + self.sizes)
        return input.reshape(self.sizes)

    def updateGradInput(self, input, gradOutput):
        return gradOutput.reshape(input.shape)


class InferReshape(TensorModule):
    """Reshape where 0 copies the input dim and -1 is inferred."""

    def __init__(self, size, batchMode=False):
        super().__init__()
        self.size = tuple(size)
        self.batchMode = batchMode

    def updateOutput(self, input):
        shape = list(input.shape[1:] if self.batchMode else input.shape)
        tgt = [shape[i] if s == 0 else s for i, s in enumerate(self.size)]
        if self.batchMode:
            tgt = [input.shape[0]] + tgt
        return input.reshape(tgt)

    def updateGradInput(self, input, gradOutput):
        return gradOutput.reshape(input.shape)


class Squeeze(TensorModule):
    def __init__(self, dim=None, numInputDims=None):
        super().__init__()
        self.dim, self.numInputDims = dim, numInputDims

    def updateOutput(self, input):
        if self.dim is None:
            return input.squeeze()
        dims = self.dim if isinstance(self.dim, (list, tuple)) else [self.dim]
        out = input
        for d in sorted((_bdim(d, input, self.numInputDims) for d in dims), reverse=True):
            out = out.squeeze(d)
        return out

    def updateGradInput(self, input, gradOutput):
        return gradOutput.reshape(input.shape)


class Unsqueeze(TensorModule):
    def __init__(self, pos, numInputDims=None):
        super().__init__()
        self.pos, self.numInputDims = pos, numInputDims

    def updateOutput(self, input):
        return input.unsqueeze(_bdim(self.pos, input, self.numInputDims))

    def updateGradInput(self, input, gradOutput):
        return gradOutput.reshape(input.shape)


class Transpose(TensorModule):
    def __init__(self, permutations):
        super().__init__()
        self.permutations = [tuple(p) for p in permutations]

    def updateOutput(self, input):
        out = input
        for a, b in self.permutations:
            out = out.transpose(a - 1, b - 1)
        return out.contiguous()

    def updateGradInput(self, input, gradOutput):
        g = gradOutput
        for a, b in reversed(self.permutations):
            g = g.transpose(a - 1, b - 1)
        return g.contiguous()


class Contiguous(TensorModule):
    def updateOutput(self, input):
        return input.contiguous()

    def updateGradInput(self, input, gradOutput):
        return gradOutput.contiguous()


class Narrow(TensorModule):
    def __init__(self, dimension, offset, length=1):
        super().__init__()
        self.dimension, self.offset, self.length = dimension, offset, length

    def _args(self, x):
        d = _bdim(self.dimension, x, None)
        off = self.offset - 1 if self.offset > 0 else x.shape[d] + self.offset
        ln = self.length if self.length > 0 else x.shape[d] - off + self.length + 1
        return d, off, ln

    def updateOutput(self, input):
        d, off, ln = self._args(input)
        return input.narrow(d, off, ln)

    def updateGradInput(self, input, gradOutput):
        d, off, ln = self._args(input)
        g = torch.zeros_like(input, dtype=gradOutput.dtype)
        g.narrow(d, off, ln).copy_(gradOutput)
        return g


class Select(TensorModule):
    def __init__(self, dimension, index):
        super().__init__()
        self.dimension, self.index = dimension, index

    def _args(self, x):
        d = _bdim(self.dimension, x, None)
        i = self.index - 1 if self.index > 0 else x.shape[d] + self.index
        return d, i

    def updateOutput(self, input):
        d, i = self._args(input)
        return input.select(d, i)

    def updateGradInput(self, input, gradOutput):
        d, i = self._args(input)
        g = torch.zeros_like(input, dtype=gradOutput.dtype)
        g.select(d, i).copy_(gradOutput)
        return g


class Index(AutogradModule):
    """Table(tensor, indices): index_select along 1-based ``dimension`` with 1-based indices."""

    def __init__(self, dimension):
        super().__init__()
        self.dimension = dimension

    def fn(self, x):
        t, idx = x[1], x[2]
        return t.index_select(self.dimension - 1, idx.long().reshape(-1) - 1)


class Replicate(AutogradModule):
    def __init__(self, nFeatures, dim=1, nDim=None):
        super().__init__()
        self.nFeatures, self.dim, self.nDim = nFeatures, dim, nDim

    def fn(self, x):
        d = self.dim - 1
        if self.nDim is not None and x.dim() > self.nDim:
            d += 1
        return x.unsqueeze(d).expand(*x.shape[:d], self.nFeatures, *x.shape[d:]).contiguous()


class Tile(AutogradModule):
    def __init__(self, dim=1, copies=2):
        super().__init__()
        self.dim, self.copies = dim, copies

    def fn(self, x):
        reps = [1] * x.dim()
        reps[self.dim - 1] = self.copies
        return x.repeat(*reps)


class ExpandSize(AutogradModule):
    def __init__(self, targetSizes):
        super().__init__()
        self.targetSizes = tuple(targetSizes)

    def fn(self, x):
        tgt = [x.shape[i] if s == -1 else s for i, s in enumerate(self.targetSizes)]
        return x.expand(*tgt).contiguous()


class Padding(AutogradModule):
    """Pad ``pad`` entries (negative: before, positive: after) along 1-based ``dim`` with ``value``."""

    def __init__(self, dim, pad, nInputDim, value=0.0, nIndex=1):
        super().__init__()
        self.dim, self.pad, self.nInputDim, self.value, self.nIndex = dim, pad, nInputDim, value, nIndex

    def fn(self, x):
        d = _bdim(self.dim, x, self.nInputDim)
        shape = list(x.shape)
        shape[d] = abs(self.pad)
        p = torch.full(shape, float(self.value), dtype=x.dtype, device=x.device)
        if self.pad < 0:
            return torch.cat([p, x], dim=d)
        return torch.cat([x, p], dim=d)


class SpatialZeroPadding(AutogradModule):
    def __init__(self, padLeft, padRight, padTop, padBottom):
        super().__init__()
        self.p = (padLeft, padRight, padTop, padBottom)

    def fn(self, x):
        return F.pad(x, self.p)


class Cropping2D(AutogradModule):
    def __init__(self, heightCrop, widthCrop, dataFormat="NCHW"):
        super().__init__()
        self.h, self.w, self.fmt = tuple(heightCrop), tuple(widthCrop), dataFormat

    def fn(self, x):
        if self.fmt == "NCHW":
            H, W = x.shape[2], x.shape[3]
            return x[:, :, self.h[0]:H - self.h[1], self.w[0]:W - self.w[1]]
        H, W = x.shape[1], x.shape[2]
        return x[:, self.h[0]:H - self.h[1], self.w[0]:W - self.w[1], :]


class Cropping3D(AutogradModule):
    def __init__(self, dim1Crop, dim2Crop, dim3Crop, dataFormat="channel_first"):
        super().__init__()
        self.c = (tuple(dim1Crop), tuple(dim2Crop), tuple(dim3Crop))
        self.fmt = dataFormat

    def fn(self, x):
        off = 2 if self.fmt == "channel_first" else 1
        sl = [slice(None)] * x.dim()
        for i, (a, b) in enumerate(self.c):
            n = x.shape[off + i]
            sl[off + i] = slice(a, n - b)
        return x[tuple(sl)]


class Reverse(AutogradModule):
    def __init__(self, dimension=1, isInplace=False):
        super().__init__()
        self.dimension = dimension

    def fn(self, x):
        return torch.flip(x, [self.dimension - 1])


class MaskedSelect(AutogradModule):
    def fn(self, x):
        return torch.masked_select(x[1], x[2].bool())


class Sum(AutogradModule):
    def __init__(self, dimension=1, nInputDims=-1, sizeAverage=False, squeeze=True):
        super().__init__()
        self.dimension, self.nInputDims, self.sizeAverage, self.squeeze = dimension, nInputDims, sizeAverage, squeeze

    def fn(self, x):
        d = _bdim(self.dimension, x, self.nInputDims)
        y = x.sum(d, keepdim=not self.squeeze)
        if self.sizeAverage:
            y = y / x.shape[d]
        return y


class Mean(Sum):
    def __init__(self, dimension=1, nInputDims=-1, squeeze=True):
        super().__init__(dimension, nInputDims, True, squeeze)


class Max(AutogradModule):
    def __init__(self, dim=1, numInputDims=None):
        super().__init__()
        self.dim, self.numInputDims = dim, numInputDims

    def fn(self, x):
        return x.max(_bdim(self.dim, x, self.numInputDims)).values


class Min(Max):
    def fn(self, x):
        return x.min(_bdim(self.dim, x, self.numInputDims)).values


class UpSampling1D(AutogradModule):
    def __init__(self, length):
        super().__init__()
        self.length = length

    def fn(self, x):
        from ..ops.pool_nd import upsample_nearest

        return upsample_nearest(x, (self.length,), sequence=True)     # GPU: csrc/pool_nd.hip


class UpSampling2D(AutogradModule):
    def __init__(self, size, format="NCHW"):
        super().__init__()
        self.size, self.format = tuple(size), format

    def fn(self, x):
        from ..ops.pool_nd import upsample_nearest

        return upsample_nearest(x, self.size, channels_last=self.format == "NHWC")


class UpSampling3D(AutogradModule):
    def __init__(self, size):
        super().__init__()
        self.size = tuple(size)

    def fn(self, x):
        from ..ops.pool_nd import upsample_nearest

        return upsample_nearest(x, self.size)


class ResizeBilinear(AutogradModule):
    def __init__(self, outputHeight, outputWidth, alignCorners=False, dataFormat="NCHW"):
        super().__init__()
        self.size, self.align, self.fmt = (outputHeight, outputWidth), alignCorners, dataFormat

    def fn(self, x):
        if self.fmt == "NHWC":
            x = x.permute(0, 3, 1, 2)
        from ..ops import nnk

        y = nnk.resize_bilinear(x, self.size[0], self.size[1], self.align)   # TF-legacy sampling, GPU kernel
        if self.fmt == "NHWC":
            y = y.permute(0, 2, 3, 1)
        return y


class Pack(AutogradModule):
    """Stack the tensors of an input table along a new 1-based dimension."""

    def __init__(self, dimension):
        super().__init__()
        self.dimension = dimension

    def fn(self, x):
        ts = x.toSeq() if not isinstance(x, torch.Tensor) else [x]
        return torch.stack(ts, dim=self.dimension - 1)


class Masking(AutogradModule):
    def __init__(self, maskValue=0.0):
        super().__init__()
        self.maskValue = maskValue

    def fn(self, x):
        keep = (x != self.maskValue).any(dim=-1, keepdim=True)
        return x * keep.to(x.dtype)


class Flatten(TensorModule):
    """Flatten all but the batch dim (convenience; keras Flatten)."""

    def updateOutput(self, input):
        return input.reshape(input.shape[0], -1)

    def updateGradInput(self, input, gradOutput):
        return gradOutput.reshape(input.shape)


__all__ = [n for n in list(globals()) if n[0].isupper() and n != "F"]
