"""Validation methods and results (reference S/optim/ValidationMethod.scala:37-1117 — Top1Accuracy :173,
Top5Accuracy :827, Loss :1078, MAE :1103, TreeNNAccuracy :121, MeanAveragePrecision :230 (+ VOC/COCO
:410-413), HitRatio :882, NDCG :949; S/optim/PrecisionRecallAUC.scala:34).

Results are monoids: ``r1 + r2`` merges partial results from different batches / ranks; ``result()``
returns (value, count). Labels are 1-based. ``to_tensor``/``from_tensor`` let the distributed evaluator
merge results with one RCCL/gloo all-reduce.
"""
import math

import torch


class ValidationResult:
    def result(self):
        raise NotImplementedError

    def __add__(self, other):
        raise NotImplementedError

    def to_tensor(self):
        raise NotImplementedError

    def __repr__(self):
        v, n = self.result()
        return f"{type(self).__name__}({v}, count={n})"


class AccuracyResult(ValidationResult):
    def __init__(self, correct, count):
        self.correct, self.count = int(correct), int(count)

    def result(self):
        return (self.correct / self.count if self.count else 0.0), self.count

    def __add__(self, o):
        return AccuracyResult(self.correct + o.correct, self.count + o.count)

    def to_tensor(self):
        return torch.tensor([self.correct, self.count], dtype=torch.float64)

    @staticmethod
    def from_tensor(t):
        return AccuracyResult(int(t[0]), int(t[1]))

    def __repr__(self):
        v, n = self.result()
        return f"Accuracy(correct: {self.correct}, count: {n}, accuracy: {v})"


class LossResult(ValidationResult):
    def __init__(self, loss, count):
        self.loss, self.count = float(loss), int(count)

    def result(self):
        return (self.loss / self.count if self.count else 0.0), self.count

    def __add__(self, o):
        return LossResult(self.loss + o.loss, self.count + o.count)

    def to_tensor(self):
        return torch.tensor([self.loss, self.count], dtype=torch.float64)

    @staticmethod
    def from_tensor(t):
        return LossResult(float(t[0]), int(t[1]))


class ContiguousResult(LossResult):
    pass


class MAPResult(ValidationResult):
    def __init__(self, scores_per_class, labels_per_class, npos_per_class):
        self.scores = scores_per_class
        self.labels = labels_per_class
        self.npos = npos_per_class

    def __add__(self, o):
        return MAPResult([a + b for a, b in zip(self.scores, o.scores)],
                         [a + b for a, b in zip(self.labels, o.labels)],
                         [a + b for a, b in zip(self.npos, o.npos)])

    def result(self):
        aps = []
        for s, l, n in zip(self.scores, self.labels, self.npos):
            if n == 0:
                continue
            order = sorted(range(len(s)), key=lambda i: -s[i])
            tp = 0
            ap = 0.0
            for rank, i in enumerate(order, 1):
                if l[i]:
                    tp += 1
                    ap += tp / rank
            aps.append(ap / n)
        return (sum(aps) / len(aps) if aps else 0.0), len(aps)


class ValidationMethod:
    def __call__(self, output, target):
        return self.apply(output, target)

    def apply(self, output, target):
        raise NotImplementedError

    def format(self):
        return type(self).__name__

    def __repr__(self):
        return self.format()


def _to2d(output):
    o = output.float()
    return o.unsqueeze(0) if o.dim() == 1 else o


class Top1Accuracy(ValidationMethod):
    def apply(self, output, target):
        o = _to2d(output)
        t = target.reshape(-1).to(o.device)
        if o.shape[1] == 1:  # binary classifier with sigmoid output
            pred = (o.reshape(-1) > 0.5).float()
            correct = int((pred == t.float()).sum())
        else:
            pred = o.argmax(dim=1) + 1
            correct = int((pred.float() == t.float()).sum())
        return AccuracyResult(correct, o.shape[0])

    def format(self):
        return "Top1Accuracy"


class Top5Accuracy(ValidationMethod):
    def apply(self, output, target):
        o = _to2d(output)
        t = target.reshape(-1).to(o.device).long() - 1
        k = min(5, o.shape[1])
        top = o.topk(k, dim=1).indices
        correct = int((top == t.unsqueeze(1)).any(dim=1).sum())
        return AccuracyResult(correct, o.shape[0])

    def format(self):
        return "Top5Accuracy"


class TreeNNAccuracy(ValidationMethod):
    """Accuracy on the root of a tree output (batch, nodes, classes): uses node 1."""

    def apply(self, output, target):
        o = output.float()
        root = o[:, 0, :] if o.dim() == 3 else o
        t = target[:, 0] if target.dim() > 1 else target
        pred = root.argmax(dim=1) + 1
        return AccuracyResult(int((pred.float() == t.float().to(pred.device)).sum()), root.shape[0])


class Loss(ValidationMethod):
    def __init__(self, criterion=None):
        from ..nn.criterion import ClassNLLCriterion

        self.criterion = criterion if criterion is not None else ClassNLLCriterion()

    def apply(self, output, target):
        l = float(self.criterion.forward(output, target))
        n = output.shape[0] if output.dim() > 1 else 1
        return LossResult(l * n, n)

    def format(self):
        return "Loss"


class MAE(ValidationMethod):
    def apply(self, output, target):
        o = output.float()
        t = target.float().to(o.device).reshape(o.shape)
        n = o.shape[0] if o.dim() > 1 else 1
        return LossResult(float((o - t).abs().mean()) * n, n)

    def format(self):
        return "MAE"


class HitRatio(ValidationMethod):
    """Recommendation hit ratio @k: output scores of (1 positive + negNum negatives), positive first."""

    def __init__(self, k=10, negNum=100):
        self.k, self.negNum = k, negNum

    def apply(self, output, target):
        o = output.reshape(-1).float()
        t = target.reshape(-1).float().to(o.device)
        pos = int(torch.nonzero(t == 1)[0]) if (t == 1).any() else 0
        rank = int((o > o[pos]).sum()) + 1
        return AccuracyResult(1 if rank <= self.k else 0, 1)

    def format(self):
        return f"HitRate@{self.k}"


class NDCG(ValidationMethod):
    def __init__(self, k=10, negNum=100):
        self.k, self.negNum = k, negNum

    def apply(self, output, target):
        o = output.reshape(-1).float()
        t = target.reshape(-1).float().to(o.device)
        pos = int(torch.nonzero(t == 1)[0]) if (t == 1).any() else 0
        rank = int((o > o[pos]).sum()) + 1
        v = math.log(2) / math.log(rank + 1) if rank <= self.k else 0.0
        return LossResult(v, 1)

    def format(self):
        return f"NDCG@{self.k}"


class MeanAveragePrecision(ValidationMethod):
    """mAP over classes from per-sample class scores and 1-based labels (classification form)."""

    def __init__(self, k, classes):
        self.k, self.classes = k, classes

    def apply(self, output, target):
        o = _to2d(output).cpu()
        t = target.reshape(-1).long().cpu() - 1
        scores = [o[:, c].tolist() for c in range(self.classes)]
        labels = [(t == c).tolist() for c in range(self.classes)]
        npos = [int((t == c).sum()) for c in range(self.classes)]
        return MAPResult(scores, labels, npos)

    def format(self):
        return f"MAP@{self.k}"


class PrecisionRecallAUC(ValidationMethod):
    """Area under the precision-recall curve for a binary classifier."""

    def apply(self, output, target):
        o = output.reshape(-1).float().cpu()
        t = target.reshape(-1).float().cpu()
        return _PRResult(o.tolist(), t.tolist())

    def format(self):
        return "PrecisionRecallAUC"


class _PRResult(ValidationResult):
    def __init__(self, scores, labels):
        self.scores, self.labels = scores, labels

    def __add__(self, o):
        return _PRResult(self.scores + o.scores, self.labels + o.labels)

    def result(self):
        order = sorted(range(len(self.scores)), key=lambda i: -self.scores[i])
        P = sum(1 for l in self.labels if l > 0.5)
        if P == 0:
            return 0.0, len(self.scores)
        tp = fp = 0
        auc, prev_r = 0.0, 0.0
        for i in order:
            if self.labels[i] > 0.5:
                tp += 1
            else:
                fp += 1
            r = tp / P
            p = tp / (tp + fp)
            auc += (r - prev_r) * p
            prev_r = r
        return auc, len(self.scores)


class EvaluateMethods:
    """Batch accuracy counters (reference S/optim/EvaluateMethods.scala:21): ``(correct, count)`` for a
    [batch, classes] or [classes] score tensor against 1-based labels."""

    @staticmethod
    def _topk_hits(output, target, k):
        if output.dim() == 1:
            if target.numel() != 1:
                raise ValueError("a single-sample output needs a single target")
            output = output.unsqueeze(0)
        elif output.dim() != 2:
            raise ValueError("output must be 1-D or 2-D")
        idx = output.float().topk(min(k, output.shape[1]), 1).indices + 1
        t = target.reshape(-1, 1).to(idx.device).long()
        return int((idx == t).any(1).sum()), output.shape[0]

    @staticmethod
    def calcAccuracy(output, target):
        return EvaluateMethods._topk_hits(output, target, 1)

    @staticmethod
    def calcTop5Accuracy(output, target):
        return EvaluateMethods._topk_hits(output, target, 5)


__all__ = ["ValidationResult", "AccuracyResult", "LossResult", "ContiguousResult", "MAPResult", "ValidationMethod",
           "Top1Accuracy", "Top5Accuracy", "TreeNNAccuracy", "Loss", "MAE", "HitRatio", "NDCG",
           "MeanAveragePrecision", "PrecisionRecallAUC", "EvaluateMethods"]
