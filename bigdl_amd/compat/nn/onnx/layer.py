"""Reference ``bigdl.nn.onnx.layer`` (P/nn/onnx/layer.py): the ONNX-semantics layers with their Python
signatures (snake_case, ndarray operands) over the engine modules."""
import numpy as np
import torch

from ....nn import Gemm as _Gemm
from ....nn import onnx as _onnx
from ....nn import tf as _tf
from ....nn.tf_ops import ops as _ops
from ..layer import Layer


def _t(a):
    return torch.as_tensor(np.asarray(a), dtype=torch.float32)


class Constant(Layer):
    def __init__(self, value, bigdl_type="float"):
        super().__init__(jvalue=_tf.Const(_t(value)))


class Gather(Layer):
    def __init__(self, bigdl_type="float"):
        super().__init__(jvalue=_ops.Gather())


class Gemm(Layer):
    def __init__(self, matrix_b, matrix_c, alpha=1.0, beta=1.0, trans_a=0, trans_b=0, bigdl_type="float"):
        super().__init__(jvalue=_Gemm(alpha, beta, bool(trans_a), bool(trans_b), matrixB=_t(matrix_b),
                                      matrixC=_t(matrix_c)))


class Reshape(Layer):
    def __init__(self, shape=None, bigdl_type="float"):
        super().__init__(jvalue=_onnx.Reshape(shape))


class Shape(Layer):
    def __init__(self, bigdl_type="float"):
        super().__init__(jvalue=_onnx.Shape())


__all__ = ["Constant", "Gather", "Gemm", "Reshape", "Shape"]
