"""ONNX-semantics layers (reference S/nn/onnx/{Gemm,Shape,Reshape}.scala; Gemm lives in nn/linear.py).

They differ from the Torch-style layers of the same name: ``Shape`` returns the input's sizes as a float tensor
and ``Reshape`` never infers a batch dimension and also takes its target shape from a Table(data, shape) input,
as ONNX's Reshape node does."""
import torch

from ..utils.table import Table
from .abstractnn import AbstractModule


class Shape(AbstractModule):
    """Input tensor -> 1-D tensor of its sizes (S/nn/onnx/Shape.scala:28-40). No gradient flows to the input."""

    def updateOutput(self, input):
        self.output = torch.tensor(list(input.shape), dtype=torch.float32, device=input.device)
        return self.output

    def updateGradInput(self, input, gradOutput):
        self.gradInput = torch.zeros_like(input)
        return self.gradInput


class Reshape(AbstractModule):
    """Tensor input reshaped to ``shape``, or Table(data, shape) with the shape read from the second tensor
    (S/nn/onnx/Reshape.scala:30-50). Entries follow ONNX: 0 copies the input size, -1 is inferred."""

    def __init__(self, shape=None):
        super().__init__()
        self.shape = None if shape is None else [int(s) for s in shape]

    def _split(self, input):
        if isinstance(input, Table):
            if input.length() != 2:
                raise ValueError("onnx.Reshape takes Table(data, shape)")
            return input[1], [int(v) for v in input[2].reshape(-1).tolist()]
        if self.shape is None:
            raise ValueError("shape should not be null")
        return input, self.shape

    def updateOutput(self, input):
        data, shape = self._split(input)
        if isinstance(input, Table):
            self.shape = shape
        target = [data.shape[i] if s == 0 else s for i, s in enumerate(shape)]
        self.output = data.reshape(target)
        return self.output

    def updateGradInput(self, input, gradOutput):
        data, shape = self._split(input)
        g = gradOutput.reshape(data.shape)
        self.gradInput = Table(g, torch.zeros(len(shape))) if isinstance(input, Table) else g
        return self.gradInput


__all__ = ["Shape", "Reshape"]
