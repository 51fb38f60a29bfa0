"""Regularizers applied inside accGradParameters (reference S/optim/Regularizer.scala:30-193)."""
import torch


class Regularizer:
    def accRegularization(self, parameter, gradParameter, scale=1.0):
        raise NotImplementedError

    def isRegularized(self):
        return True


class L1L2Regularizer(Regularizer):
    def __init__(self, l1=0.0, l2=0.0):
        self.l1, self.l2 = float(l1), float(l2)

    def accRegularization(self, parameter, gradParameter, scale=1.0):
        if self.l1 != 0.0:
            gradParameter.add_(torch.sign(parameter), alpha=self.l1 * scale)
        if self.l2 != 0.0:
            gradParameter.add_(parameter, alpha=self.l2 * scale)

    def __repr__(self):
        return f"{type(self).__name__}(l1={self.l1}, l2={self.l2})"


class L1Regularizer(L1L2Regularizer):
    def __init__(self, l1):
        super().__init__(l1, 0.0)


class L2Regularizer(L1L2Regularizer):
    def __init__(self, l2):
        super().__init__(0.0, l2)


__all__ = ["Regularizer", "L1L2Regularizer", "L1Regularizer", "L2Regularizer"]
