"""BigDL Tensor API (1-based, Torch7-style) over torch tensors — reference S/tensor/*."""
from .quantized import QuantizedTensor
from .tensor import (SparseTensor, Storage, Tensor, dense, gaussian1D, ones, randperm, range_, scalar, sparse,
                     to_torch, unique, zeros)

range = range_  # noqa: A001  (reference Tensor.range)

__all__ = ["Tensor", "SparseTensor", "QuantizedTensor", "Storage", "ones", "zeros", "range", "randperm", "scalar", "gaussian1D",
           "unique", "dense", "sparse", "to_torch"]
