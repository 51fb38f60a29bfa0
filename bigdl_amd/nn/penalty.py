"""Activity-regularisation layers: identity in the forward pass, a penalty term added to the gradient.

Reference: S/nn/L1Penalty.scala:38-90, ActivityRegularization.scala:30-52, NegativeEntropyPenalty.scala:30-69,
TableOperation.scala:28-101 (broadcasting table ops CMulTableExpand / CSubTableExpand).
The penalty value of the last forward is kept in ``loss`` like the reference.
"""
import torch

from ..utils.table import Table
from .abstractnn import AbstractModule, TensorModule
from .shape_ops import ExpandSize
from .table_ops import CMulTable, CSubTable


class L1Penalty(TensorModule):
    def __init__(self, l1weight, sizeAverage=False, provideOutput=True):
        super().__init__()
        self.l1weight, self.sizeAverage, self.provideOutput = l1weight, sizeAverage, provideOutput
        self.loss = 0.0

    def _m(self, x):
        return self.l1weight / x.numel() if self.sizeAverage else float(self.l1weight)

    def updateOutput(self, input):
        self.loss = self._m(input) * float(input.abs().sum())
        return input

    def updateGradInput(self, input, gradOutput):
        g = torch.sign(input) * self._m(input)
        return g + gradOutput if self.provideOutput else g


class ActivityRegularization(TensorModule):
    def __init__(self, l1, l2):
        super().__init__()
        self.l1, self.l2 = l1, l2
        self.loss = 0.0

    def updateOutput(self, input):
        x = input.float()
        self.loss = float(self.l1 * x.abs().sum() + self.l2 * (x * x).sum())
        return input

    def updateGradInput(self, input, gradOutput):
        return (torch.sign(input) * self.l1 + input * (2 * self.l2) + gradOutput).to(gradOutput.dtype)


class NegativeEntropyPenalty(TensorModule):
    """Penalises low-entropy distributions: loss = beta * sum(p log p)."""

    def __init__(self, beta=0.01):
        super().__init__()
        self.beta = beta
        self.loss = 0.0

    def updateOutput(self, input):
        self.loss = self.beta * float((input * torch.log(input)).sum())
        return input

    def updateGradInput(self, input, gradOutput):
        return (torch.log(input) + 1) * self.beta + gradOutput


class TableOperation(AbstractModule):
    """Apply a two-input table op after broadcasting the smaller input to the larger one's shape (batch dim
    free)."""

    def __init__(self, operationLayer):
        super().__init__()
        self.operationLayer = operationLayer
        self._expand = None
        self._small = 1

    def updateOutput(self, input):
        assert input.length() == 2, f"Only support input two tensors, but get {input.length()}"
        a, b = input[1], input[2]
        self._small = 2 if a.numel() > b.numel() else 1
        small, large = input[self._small], input[3 - self._small]
        size = list(large.shape)
        size[0] = -1
        self._expand = ExpandSize(size)
        ex = self._expand.forward(small)
        return self.operationLayer.updateOutput(Table(large, ex))

    def updateGradInput(self, input, gradOutput):
        small, large = input[self._small], input[3 - self._small]
        g = self.operationLayer.updateGradInput(Table(large, self._expand.output), gradOutput)
        out = Table()
        out[3 - self._small] = g[1]
        out[self._small] = self._expand.backward(small, g[2])
        return out

    def __repr__(self):
        return "TableOperationExpand"


def CMulTableExpand():
    return TableOperation(CMulTable())


def CSubTableExpand():
    return TableOperation(CSubTable())


__all__ = ["L1Penalty", "ActivityRegularization", "NegativeEntropyPenalty", "TableOperation", "CMulTableExpand",
           "CSubTableExpand"]
