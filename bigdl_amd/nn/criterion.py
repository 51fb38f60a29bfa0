"""Criterions (reference: 36 files in S/nn/, e.g. ClassNLLCriterion.scala:69, CrossEntropyCriterion.scala:31,
MSECriterion.scala, TimeDistributedCriterion.scala). Class labels are 1-based, as in the reference.

CrossEntropyCriterion on the GPU engine is the fused log-softmax + NLL kernel (csrc/elementwise.hip):
loss and gradient in one pass over the logits.
"""
import math

import torch
import torch.nn.functional as F

from .. import ops
from ..utils.table import Table
from .abstractnn import AbstractCriterion, AutogradCriterion


def _labels0(target, n=None):
    t = target.reshape(-1).long() - 1
    return t


class CrossEntropyCriterion(AbstractCriterion):
    def __init__(self, weights=None, sizeAverage=True):
        super().__init__(sizeAverage)
        self.weights = torch.as_tensor(weights).float() if weights is not None else None

    def updateOutput(self, input, target):
        x = input if input.dim() > 1 else input.unsqueeze(0)
        if x.is_cuda and self.weights is None:
            loss, dl = ops.softmax_xent_gpu(x, target.reshape(-1).to(x.device), 1.0, self.sizeAverage)
            self._grad = dl
            return loss[0]
        self._grad = None
        w = self.weights.to(x.device) if self.weights is not None else None
        return F.cross_entropy(x.float(), _labels0(target).to(x.device), weight=w,
                               reduction="mean" if self.sizeAverage else "sum")

    def updateGradInput(self, input, target):
        if self._grad is not None:
            g = self._grad
            self._grad = None
            return g.reshape(input.shape)
        x = input.detach().float().requires_grad_(True)
        xx = x if x.dim() > 1 else x.unsqueeze(0)
        with torch.enable_grad():
            w = self.weights.to(x.device) if self.weights is not None else None
            loss = F.cross_entropy(xx, _labels0(target).to(x.device), weight=w,
                                   reduction="mean" if self.sizeAverage else "sum")
        return torch.autograd.grad(loss, x)[0].to(input.dtype)


class ClassNLLCriterion(AutogradCriterion):
    """Negative log-likelihood on log-probabilities (or probabilities when logProbAsInput=False)."""

    def __init__(self, weights=None, sizeAverage=True, logProbAsInput=True, paddingValue=-1):
        super().__init__(sizeAverage)
        self.weights = torch.as_tensor(weights).float() if weights is not None else None
        self.logProbAsInput = logProbAsInput
        self.paddingValue = paddingValue

    def loss(self, input, target):
        x = input if input.dim() > 1 else input.unsqueeze(0)
        if not self.logProbAsInput:
            x = torch.log(x.clamp_min(1e-8))
        t = _labels0(target).to(x.device)
        valid = t != (self.paddingValue - 1)
        tc = t.clamp_min(0)
        w = self.weights.to(x.device)[tc] if self.weights is not None else torch.ones_like(tc, dtype=x.dtype)
        w = w * valid.to(x.dtype)
        l = -(x.gather(1, tc.unsqueeze(1)).squeeze(1) * w).sum()
        if self.sizeAverage:
            l = l / w.sum().clamp_min(1e-12)
        return l


class MSECriterion(AutogradCriterion):
    def loss(self, input, target):
        d = input - target.to(input.device, input.dtype)
        return (d * d).mean() if self.sizeAverage else (d * d).sum()


class AbsCriterion(AutogradCriterion):
    def loss(self, input, target):
        d = (input - target.to(input.device, input.dtype)).abs()
        return d.mean() if self.sizeAverage else d.sum()


class SmoothL1Criterion(AutogradCriterion):
    def loss(self, input, target):
        return F.smooth_l1_loss(input, target.to(input.device, input.dtype),
                                reduction="mean" if self.sizeAverage else "sum")


class SmoothL1CriterionWithWeights(AutogradCriterion):
    def __init__(self, sigma, num=0):
        super().__init__(True)
        self.sigma, self.num = sigma, num

    def loss(self, input, target):
        tgt, inw, outw = target[1], target[2], target[3]
        s2 = self.sigma * self.sigma
        d = (input - tgt.to(input.dtype)) * inw.to(input.dtype)
        ad = d.abs()
        l = torch.where(ad < 1.0 / s2, 0.5 * s2 * d * d, ad - 0.5 / s2) * outw.to(input.dtype)
        return l.sum() / (self.num if self.num > 0 else 1)


class BCECriterion(AutogradCriterion):
    def __init__(self, weights=None, sizeAverage=True):
        super().__init__(sizeAverage)
        self.weights = torch.as_tensor(weights).float() if weights is not None else None

    def loss(self, input, target):
        w = self.weights.to(input.device) if self.weights is not None else None
        x = input.clamp(1e-12, 1 - 1e-12)
        return F.binary_cross_entropy(x, target.to(x.device, x.dtype), weight=w,
                                      reduction="mean" if self.sizeAverage else "sum")


class CategoricalCrossEntropy(AutogradCriterion):
    """Cross entropy between a probability input and a one-hot / probability target (Keras style)."""

    def loss(self, input, target):
        x = input.clamp(1e-7, 1 - 1e-7)
        x = x / x.sum(-1, keepdim=True)
        return -(target.to(x.dtype) * torch.log(x)).sum(-1).mean()


class DistKLDivCriterion(AutogradCriterion):
    def loss(self, input, target):
        t = target.to(input.dtype)
        l = torch.where(t > 0, t * (torch.log(t.clamp_min(1e-30)) - input), torch.zeros_like(t)).sum()
        return l / input.numel() if self.sizeAverage else l


class KullbackLeiblerDivergenceCriterion(AutogradCriterion):
    def loss(self, input, target):
        x = input.clamp(1e-7, 1)
        t = target.to(x.dtype).clamp(1e-7, 1)
        return (t * torch.log(t / x)).sum(-1).mean()


class KLDCriterion(AutogradCriterion):
    """VAE KL term for Table(mean, logVar) against N(0, 1)."""

    def loss(self, input, target):
        mean, logvar = input[1], input[2]
        l = -0.5 * (1 + logvar - mean * mean - torch.exp(logvar)).sum()
        return l / mean.shape[0] if self.sizeAverage else l


class GaussianCriterion(AutogradCriterion):
    """Negative log-likelihood of target under N(mean, exp(logVar))."""

    def loss(self, input, target):
        mean, logvar = input[1], input[2]
        t = target.to(mean.dtype)
        return (0.5 * math.log(2 * math.pi) + 0.5 * logvar + 0.5 * (t - mean) ** 2 / torch.exp(logvar)).sum()


class HingeEmbeddingCriterion(AutogradCriterion):
    def __init__(self, margin=1.0, sizeAverage=True):
        super().__init__(sizeAverage)
        self.margin = margin

    def loss(self, input, target):
        return F.hinge_embedding_loss(input, target.to(input.dtype), self.margin,
                                      reduction="mean" if self.sizeAverage else "sum")


class L1HingeEmbeddingCriterion(AutogradCriterion):
    def __init__(self, margin=1.0):
        super().__init__(True)
        self.margin = margin

    def loss(self, input, target):
        d = (input[1] - input[2]).abs().sum()
        y = float(target.reshape(-1)[0])
        return d if y == 1 else torch.clamp(self.margin - d, min=0)


class MarginCriterion(AutogradCriterion):
    def __init__(self, margin=1.0, sizeAverage=True, squared=False):
        super().__init__(sizeAverage)
        self.margin, self.squared = margin, squared

    def loss(self, input, target):
        l = torch.clamp(self.margin - input * target.to(input.dtype), min=0)
        if self.squared:
            l = l * l
        return l.mean() if self.sizeAverage else l.sum()


class MarginRankingCriterion(AutogradCriterion):
    def __init__(self, margin=1.0, sizeAverage=True):
        super().__init__(sizeAverage)
        self.margin = margin

    def loss(self, input, target):
        y = target[1] if isinstance(target, Table) else target
        return F.margin_ranking_loss(input[1].reshape(-1), input[2].reshape(-1), y.reshape(-1).to(input[1].dtype),
                                     self.margin, reduction="mean" if self.sizeAverage else "sum")


class MultiMarginCriterion(AutogradCriterion):
    def __init__(self, p=1, weights=None, margin=1.0, sizeAverage=True):
        super().__init__(sizeAverage)
        self.p, self.margin = p, margin
        self.weights = torch.as_tensor(weights).float() if weights is not None else None

    def loss(self, input, target):
        x = input if input.dim() > 1 else input.unsqueeze(0)
        w = self.weights.to(x.device) if self.weights is not None else None
        return F.multi_margin_loss(x, _labels0(target).to(x.device), self.p, self.margin, w,
                                   reduction="mean" if self.sizeAverage else "sum")


class MultiLabelMarginCriterion(AutogradCriterion):
    def loss(self, input, target):
        x = input if input.dim() > 1 else input.unsqueeze(0)
        t = target.long() - 1
        t = t if t.dim() > 1 else t.unsqueeze(0)
        return F.multilabel_margin_loss(x, t.to(x.device), reduction="mean" if self.sizeAverage else "sum")


class MultiLabelSoftMarginCriterion(AutogradCriterion):
    def __init__(self, weights=None, sizeAverage=True):
        super().__init__(sizeAverage)
        self.weights = torch.as_tensor(weights).float() if weights is not None else None

    def loss(self, input, target):
        w = self.weights.to(input.device) if self.weights is not None else None
        l = F.multilabel_soft_margin_loss(input, target.to(input.dtype), weight=w, reduction="none")
        return l.mean() if self.sizeAverage else l.sum()


class SoftMarginCriterion(AutogradCriterion):
    def loss(self, input, target):
        return F.soft_margin_loss(input, target.to(input.dtype), reduction="mean" if self.sizeAverage else "sum")


class CosineEmbeddingCriterion(AutogradCriterion):
    def __init__(self, margin=0.0, sizeAverage=True):
        super().__init__(sizeAverage)
        self.margin = margin

    def loss(self, input, target):
        y = target[1] if isinstance(target, Table) else target
        a, b = input[1], input[2]
        a = a if a.dim() > 1 else a.unsqueeze(0)
        b = b if b.dim() > 1 else b.unsqueeze(0)
        return F.cosine_embedding_loss(a, b, y.reshape(-1).to(a.dtype), self.margin,
                                       reduction="mean" if self.sizeAverage else "sum")


class CosineDistanceCriterion(AutogradCriterion):
    def loss(self, input, target):
        c = F.cosine_similarity(input, target.to(input.dtype), dim=-1)
        l = 1 - c
        return l.mean() if self.sizeAverage else l.sum()


class CosineProximityCriterion(AutogradCriterion):
    def loss(self, input, target):
        a = F.normalize(input, dim=-1)
        b = F.normalize(target.to(input.dtype), dim=-1)
        return -(a * b).sum(-1).mean()


class DiceCoefficientCriterion(AutogradCriterion):
    def __init__(self, sizeAverage=True, epsilon=1.0):
        super().__init__(sizeAverage)
        self.epsilon = epsilon

    def loss(self, input, target):
        x = input.reshape(input.shape[0], -1) if input.dim() > 1 else input.unsqueeze(0)
        t = target.reshape(x.shape).to(x.dtype)
        inter = (x * t).sum(1)
        l = 1 - (2 * inter + self.epsilon) / (x.sum(1) + t.sum(1) + self.epsilon)
        return l.mean() if self.sizeAverage else l.sum()


class DotProductCriterion(AutogradCriterion):
    def loss(self, input, target):
        l = (input * target.to(input.dtype)).sum()
        return l / input.shape[0] if self.sizeAverage and input.dim() > 1 else l


class L1Cost(AutogradCriterion):
    def loss(self, input, target):
        return input.abs().sum()


class MeanAbsolutePercentageCriterion(AutogradCriterion):
    def loss(self, input, target):
        t = target.to(input.dtype)
        return 100.0 * ((t - input).abs() / t.abs().clamp_min(1e-7)).mean()


class MeanSquaredLogarithmicCriterion(AutogradCriterion):
    def loss(self, input, target):
        a = torch.log(input.clamp_min(1e-7) + 1)
        b = torch.log(target.to(input.dtype).clamp_min(1e-7) + 1)
        return ((a - b) ** 2).mean()


class PoissonCriterion(AutogradCriterion):
    def loss(self, input, target):
        return (input - target.to(input.dtype) * torch.log(input + 1e-7)).mean()


class PGCriterion(AutogradCriterion):
    """Policy-gradient loss: -sum(reward * log(prob of taken action))."""

    def __init__(self, sizeAverage=False):
        super().__init__(sizeAverage)

    def loss(self, input, target):
        l = -(torch.log(input.clamp_min(1e-12)) * target.to(input.dtype)).sum()
        return l / input.shape[0] if self.sizeAverage else l


class SoftmaxWithCriterion(AutogradCriterion):
    """Caffe SoftmaxWithLoss over NCHW logits with 1-based labels and optional ignore label."""

    def __init__(self, ignoreLabel=None, normalizeMode="VALID"):
        super().__init__(True)
        self.ignoreLabel, self.normalizeMode = ignoreLabel, normalizeMode

    def loss(self, input, target):
        t = target.long().reshape(input.shape[0], *input.shape[2:]) - 1
        ig = -100 if self.ignoreLabel is None else int(self.ignoreLabel) - 1
        red = "mean" if self.normalizeMode in ("VALID", "FULL") else "sum"
        return F.cross_entropy(input.float(), t.to(input.device), ignore_index=ig, reduction=red)


class TimeDistributedCriterion(AbstractCriterion):
    """Applies a criterion to every time step of (batch, time, ...) input (reference :149)."""

    def __init__(self, critrn, sizeAverage=False, dimension=2):
        super().__init__(sizeAverage)
        self.critrn = critrn
        self.dimension = dimension

    def _flat_ok(self, input, target):
        """Criterions whose per-step value is a uniform mean (or sum) over the rows of the step can run once over
        all (batch x time) rows: sum_t mean_b(l) == T * mean_{b,t}(l). Weighted / padded NLL is not uniform."""
        c = self.critrn
        if self.dimension != 2 or input.dim() < 3 or target.dim() < 2 or target.shape[:2] != input.shape[:2]:
            return False
        if isinstance(c, CrossEntropyCriterion):
            return c.weights is None
        if isinstance(c, ClassNLLCriterion):
            return c.weights is None and c.paddingValue == -1
        return isinstance(c, (MSECriterion, AbsCriterion))

    def _flat(self, input, target):
        n = input.shape[0] * input.shape[1]
        x = input.reshape((n,) + tuple(input.shape[2:]))
        y = target.reshape((n,) + tuple(target.shape[2:]))
        return x, y

    def updateOutput(self, input, target):
        d = self.dimension - 1
        T = input.shape[d]
        if self._flat_ok(input, target):       # one launch over B*T rows instead of T small ones
            x, y = self._flat(input, target)
            loss = self.critrn.forward(x, y)
            scale = (T if self.critrn.sizeAverage else 1.0) / (T if self.sizeAverage else 1.0)
            return loss * scale if scale != 1.0 else loss      # (no scalar kernel when the T's cancel)
        loss = 0.0
        for t in range(T):
            loss = loss + self.critrn.forward(input.select(d, t), target.select(d, t) if target.dim() > d else target)
        return loss / T if self.sizeAverage else loss

    def updateGradInput(self, input, target):
        d = self.dimension - 1
        T = input.shape[d]
        if self._flat_ok(input, target):
            x, y = self._flat(input, target)
            if getattr(self.critrn, "_grad", None) is None:
                self.critrn.forward(x, y)
            g = self.critrn.backward(x, y).reshape(input.shape)
            scale = (T if self.critrn.sizeAverage else 1.0) / (T if self.sizeAverage else 1.0)
            return g * scale if scale != 1.0 else g
        gs = []
        for t in range(T):
            xi = input.select(d, t)
            ti = target.select(d, t) if target.dim() > d else target
            self.critrn.forward(xi, ti)
            g = self.critrn.backward(xi, ti)
            gs.append(g / T if self.sizeAverage else g)
        return torch.stack(gs, dim=d)


class TimeDistributedMaskCriterion(TimeDistributedCriterion):
    def __init__(self, critrn, paddingValue=0):
        super().__init__(critrn, True, 2)
        self.paddingValue = paddingValue


class MultiCriterion(AbstractCriterion):
    def __init__(self):
        super().__init__()
        self.criterions, self.weights = [], []

    def add(self, criterion, weight=1.0):
        self.criterions.append(criterion)
        self.weights.append(weight)
        return self

    def updateOutput(self, input, target):
        return sum(w * c.forward(input, target) for c, w in zip(self.criterions, self.weights))

    def updateGradInput(self, input, target):
        g = None
        for c, w in zip(self.criterions, self.weights):
            gi = c.backward(input, target) * w
            g = gi if g is None else g + gi
        return g


class ParallelCriterion(AbstractCriterion):
    def __init__(self, repeatTarget=False):
        super().__init__()
        self.repeatTarget = repeatTarget
        self.criterions, self.weights = [], []

    def add(self, criterion, weight=1.0):
        self.criterions.append(criterion)
        self.weights.append(weight)
        return self

    def updateOutput(self, input, target):
        tot = 0.0
        for i, (c, w) in enumerate(zip(self.criterions, self.weights)):
            t = target if self.repeatTarget else target[i + 1]
            tot = tot + w * c.forward(input[i + 1], t)
        return tot

    def updateGradInput(self, input, target):
        gi = Table()
        for i, (c, w) in enumerate(zip(self.criterions, self.weights)):
            t = target if self.repeatTarget else target[i + 1]
            gi[i + 1] = c.backward(input[i + 1], t) * w
        return gi


class TransformerCriterion(AbstractCriterion):
    """Applies transformers to input/target before an inner criterion."""

    def __init__(self, criterion, inputTransformer=None, targetTransformer=None):
        super().__init__()
        self.criterion, self.it, self.tt = criterion, inputTransformer, targetTransformer

    def updateOutput(self, input, target):
        self._ti = self.it.forward(input) if self.it is not None else input
        self._tt = self.tt.forward(target) if self.tt is not None else target
        return self.criterion.forward(self._ti, self._tt)

    def updateGradInput(self, input, target):
        g = self.criterion.backward(self._ti, self._tt)
        return self.it.backward(input, g) if self.it is not None else g




def _regsplex(n):
    """Vertices of a regular n-simplex (n+1 points in n dims, unit norm), ClassSimplexCriterion.regsplex."""
    a = torch.zeros(n + 1, n, dtype=torch.float64)
    for k in range(1, n + 1):
        if k == 1:
            a[0, 0] = 1.0
        else:
            v = a[k - 1, : k - 1].norm(2)
            a[k - 1, k - 1] = torch.sqrt(1.0 - v * v)
        c = (a[k - 1, k - 1] ** 2 - 1.0 - 1.0 / n) / a[k - 1, k - 1]
        a[k:, k - 1] = c
    return a


class ClassSimplexCriterion(MSECriterion):
    """MSE between the input and the class's vertex of a regular simplex embedding (reference
    S/nn/ClassSimplexCriterion.scala: ``regsplex(nClasses - 1)`` padded to ``nClasses`` columns)."""

    def __init__(self, nClasses):
        super().__init__()
        if nClasses <= 1:
            raise ValueError("ClassSimplexCriterion: nClasses must be > 1")
        self.nClasses = nClasses
        simp = _regsplex(nClasses - 1)
        self.simplex = torch.zeros(simp.shape[0], nClasses, dtype=torch.float64)
        self.simplex[:, : simp.shape[1]] = simp

    def _target(self, input, target):
        t = target.reshape(-1).long() - 1
        tb = self.simplex.to(input.device)[t].to(input.dtype)
        if tb.numel() != input.numel():
            raise ValueError(f"ClassSimplexCriterion: input has {input.numel()} elements, target embedding "
                             f"{tb.numel()}")
        return tb.reshape(input.shape)

    def loss(self, input, target):
        return super().loss(input, self._target(input, target))


__all__ = [n for n in list(globals()) if n[0].isupper() and n not in ("F", "Table")]
