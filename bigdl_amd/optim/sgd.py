"""SGD and its learning-rate schedules (reference S/optim/SGD.scala:39-690).

Update rule (SGD.scala:54-120): d = g + wd*x; with momentum: buf = d on the first step, else
buf = mom*buf + (1-dampening)*d; d = d + mom*buf (nesterov) or buf; x += clr * d, where clr = -lr from the
schedule. ``dampening`` defaults to ``momentum`` (reference: Double.MaxValue sentinel).
GPU engine: one fused kernel (csrc/elementwise.hip sgd_kernel) per flat buffer / shard.
"""
import math

import torch

from ..ops import native
from .optim_method import OptimMethod, native_ok

_MAXD = float("inf")


class LearningRateSchedule:
    def __init__(self):
        self.currentRate = 0.0
        self.excludeIterations = 0
        self.excludeEpochs = 0
        self.maxIterations = 0

    def updateHyperParameter(self, optim):
        raise NotImplementedError

    def _nevals(self, optim):
        return optim.state.get("evalCounter", 0)

    def _bump(self, optim):
        optim.state["evalCounter"] = self._nevals(optim) + 1


class Default(LearningRateSchedule):
    def updateHyperParameter(self, optim):
        n = self._nevals(optim)
        self.currentRate = -optim.learningRate / (1 + (n - self.excludeIterations) * optim.learningRateDecay)
        self._bump(optim)


class Regime:
    def __init__(self, startEpoch, endEpoch, config):
        self.startEpoch, self.endEpoch, self.config = startEpoch, endEpoch, config


class EpochSchedule(LearningRateSchedule):
    def __init__(self, regimes):
        super().__init__()
        self.regimes = list(regimes)

    def updateHyperParameter(self, optim):
        epoch = optim.state["epoch"] - self.excludeEpochs
        for r in self.regimes:
            if r.startEpoch <= epoch <= r.endEpoch:
                for k, v in r.config.items():
                    if not hasattr(optim, k):
                        raise ValueError(f"EpochSchedule: {k} is not a member of SGD")
                    setattr(optim, k, v)
        self.currentRate = -optim.learningRate


class Poly(LearningRateSchedule):
    def __init__(self, power, maxIteration):
        super().__init__()
        self.power, self.maxIteration = power, maxIteration

    def updateHyperParameter(self, optim):
        n = self._nevals(optim)
        self.currentRate = 0.0 if n > self.maxIteration else \
            -optim.learningRate * math.pow(1.0 - n / self.maxIteration, self.power)
        self._bump(optim)


class Step(LearningRateSchedule):
    def __init__(self, stepSize, gamma):
        super().__init__()
        self.stepSize, self.gamma = stepSize, gamma

    def updateHyperParameter(self, optim):
        n = self._nevals(optim)
        self.currentRate = -optim.learningRate * self.gamma ** max((n - self.excludeIterations) // self.stepSize, 0)
        self._bump(optim)


class MultiStep(LearningRateSchedule):
    def __init__(self, stepSizes, gamma):
        super().__init__()
        self.stepSizes, self.gamma = list(stepSizes), gamma

    def updateHyperParameter(self, optim):
        n = self._nevals(optim) - self.excludeIterations
        k = sum(1 for s in self.stepSizes if n >= s)
        self.currentRate = -optim.learningRate * self.gamma ** k
        self._bump(optim)


class EpochDecay(LearningRateSchedule):
    def __init__(self, decayType):
        super().__init__()
        self.decayType = decayType

    def updateHyperParameter(self, optim):
        decay = self.decayType(optim.state["epoch"] - self.excludeEpochs)
        self.currentRate = -optim.learningRate * math.pow(0.1, decay)


class EpochStep(LearningRateSchedule):
    def __init__(self, stepSize, gamma):
        super().__init__()
        self.stepSize, self.gamma = stepSize, gamma

    def updateHyperParameter(self, optim):
        e = optim.state["epoch"] - self.excludeEpochs
        self.currentRate = -optim.learningRate * self.gamma ** max(e // self.stepSize, 0)


class NaturalExp(LearningRateSchedule):
    def __init__(self, decay_step, gamma):
        super().__init__()
        self.decay_step, self.gamma = decay_step, gamma

    def updateHyperParameter(self, optim):
        p = (self._nevals(optim) - self.excludeIterations) // self.decay_step
        self.currentRate = -optim.learningRate * math.exp(-self.gamma * p)
        self._bump(optim)


class Exponential(LearningRateSchedule):
    def __init__(self, decayStep, decayRate, stairCase=False):
        super().__init__()
        self.decayStep, self.decayRate, self.stairCase = decayStep, decayRate, stairCase

    def updateHyperParameter(self, optim):
        p = (self._nevals(optim) - self.excludeIterations) / float(self.decayStep)
        if self.stairCase:
            p = math.floor(p)
        self.currentRate = -optim.learningRate * math.pow(self.decayRate, p)
        self._bump(optim)


class Plateau(LearningRateSchedule):
    def __init__(self, monitor, factor=0.1, patience=10, mode="min", epsilon=1e-4, cooldown=0, minLr=0.0):
        super().__init__()
        assert factor < 1 and mode in ("min", "max")
        self.monitor, self.factor, self.patience, self.mode = monitor, factor, patience, mode
        self.epsilon, self.cooldown, self.minLr = epsilon, cooldown, minLr
        self.best = float("inf") if mode == "min" else float("-inf")
        self._cool = 0
        self._wait = 0
        self._cur_epoch = 1

    def _better(self, a, b):
        return a < b - self.epsilon if self.mode == "min" else a > b + self.epsilon

    def updateHyperParameter(self, optim):
        epoch = optim.state["epoch"] - self.excludeEpochs
        if epoch == 1:
            self.currentRate = -optim.learningRate
        if epoch == self._cur_epoch:
            return
        self._cur_epoch = epoch
        cur = optim.state.get(self.monitor)
        if cur is None:
            raise ValueError(f"Learning Rate Plateau Reducing requires {self.monitor} available!")
        cur = float(cur)
        if self._cool > 0:
            self._cool -= 1
            self._wait = 0
        if self._better(cur, self.best):
            self.best = cur
            self._wait = 0
        elif self._cool <= 0:
            if self._wait >= self.patience and abs(self.currentRate) > self.minLr * (1 + 1e-4):
                self.currentRate = -max(abs(self.currentRate) * self.factor, self.minLr)
                self._cool = self.cooldown
                self._wait = 0
            self._wait += 1


class Warmup(LearningRateSchedule):
    def __init__(self, delta):
        super().__init__()
        self.delta = delta

    def updateHyperParameter(self, optim):
        n = self._nevals(optim)
        self.currentRate = -optim.learningRate - self.delta * (n - self.excludeIterations)
        self._bump(optim)


class SequentialSchedule(LearningRateSchedule):
    def __init__(self, iterationPerEpoch):
        super().__init__()
        self.iterationPerEpoch = iterationPerEpoch
        self.schedules = []
        self.cur = 0

    def add(self, schedule, maxIteration):
        schedule.excludeIterations = self.schedules[-1].maxIterations if self.schedules else 0
        schedule.maxIterations = schedule.excludeIterations + maxIteration
        schedule.excludeEpochs = schedule.excludeIterations // self.iterationPerEpoch
        self.schedules.append(schedule)
        return self

    def updateHyperParameter(self, optim):
        n = self._nevals(optim)
        if n > self.schedules[self.cur].maxIterations and self.cur + 1 < len(self.schedules):
            optim.learningRate = -self.currentRate
            self.cur += 1
        self.schedules[self.cur].updateHyperParameter(optim)
        self.currentRate = self.schedules[self.cur].currentRate


class EpochDecayWithWarmUp(LearningRateSchedule):
    def __init__(self, warmUpIteration, warmUpDelta, decayType):
        super().__init__()
        self.warmUpIteration, self.warmUpDelta, self.decayType = warmUpIteration, warmUpDelta, decayType

    def updateHyperParameter(self, optim):
        lr = optim.learningRate
        n = self._nevals(optim)
        if n < self.warmUpIteration:
            clr = -lr - self.warmUpDelta * n
        else:
            maxlr = lr + self.warmUpDelta * self.warmUpIteration
            clr = -maxlr * math.pow(0.1, self.decayType(optim.state["epoch"]))
        self.currentRate = clr
        self._bump(optim)


def segment_decay_vector(seg, n, base, device):
    """Expand (segment starts, decays) into a per-element decay vector (CPU / fallback path)."""
    off = seg[0].to("cpu").tolist()
    val = seg[1].to("cpu").tolist()
    v = torch.zeros(n, device=device)
    for i, (o, d) in enumerate(zip(off, val)):
        end = off[i + 1] if i + 1 < len(off) else base + n
        a, b = max(o - base, 0), min(end - base, n)
        if b > a and d != 0:
            v[a:b] = d
    return v


class SGD(OptimMethod):
    def __init__(self, learningRate=1e-3, learningRateDecay=0.0, weightDecay=0.0, momentum=0.0,
                 dampening=_MAXD, nesterov=False, learningRateSchedule=None, learningRates=None,
                 weightDecays=None):
        super().__init__()
        self.learningRate = learningRate
        self.learningRateDecay = learningRateDecay
        self.weightDecay = weightDecay
        self.momentum = momentum
        self.dampening = dampening
        self.nesterov = nesterov
        self.learningRateSchedule = learningRateSchedule if learningRateSchedule is not None else Default()
        self.learningRates = learningRates
        self.weightDecays = weightDecays

    def updateHyperParameter(self):
        self.learningRateSchedule.updateHyperParameter(self)

    def getLearningRate(self):
        return self.learningRateSchedule.currentRate

    def getHyperParameter(self):
        return f"Current learning rate is {-self.learningRateSchedule.currentRate}. "

    def graph_prologue(self):
        """HIP-graph replay support (optim/graphed.py): advance the schedule on the host and publish the rate
        to the device scalar the captured kernel reads."""
        self.updateHyperParameter()
        self._lr_dev.fill_(-self.learningRateSchedule.currentRate)

    def optimize(self, feval, x):
        graphed = getattr(self, "_lr_dev", None) is not None
        if not graphed:
            self.updateHyperParameter()
        if self.dampening == _MAXD:
            self.dampening = self.momentum
        wd, mom, damp, nest = self.weightDecay, self.momentum, self.dampening, self.nesterov
        assert not nest or (mom > 0 and damp == 0), "Nesterov momentum requires a momentum and zero dampening"
        clr = self.learningRateSchedule.currentRate
        fx, dfdx = feval(x)
        if native_ok(x, dfdx) and self.learningRates is None and self.weightDecays is None:
            buf = self.state.get("dfdx")
            first = buf is None
            if mom != 0 and first:
                buf = torch.empty_like(x)
                self.state["dfdx"] = buf
            seg = getattr(self, "_wd_segments", None)
            native.get().sgd_step(x, dfdx, buf if mom != 0 else None, self._shadow16, float(-clr), float(wd),
                                  float(mom), float(damp), bool(nest), bool(first),
                                  self._lr_dev if graphed else None,
                                  seg[0] if seg else None, seg[1] if seg else None,
                                  int(getattr(self, "_seg_base", 0)))
            return x, [fx]
        seg = getattr(self, "_wd_segments", None)
        if seg is not None:
            dfdx = dfdx + segment_decay_vector(seg, x.numel(), getattr(self, "_seg_base", 0), x.device) * x
        if wd != 0:
            dfdx = dfdx.add(x, alpha=wd)
        elif self.weightDecays is not None:
            dfdx = dfdx + self.weightDecays.to(x.device) * x
        if mom != 0:
            buf = self.state.get("dfdx")
            if buf is None:
                buf = dfdx.clone()
                self.state["dfdx"] = buf
            else:
                buf.mul_(mom).add_(dfdx, alpha=1 - damp)
            dfdx = dfdx.add(buf, alpha=mom) if nest else buf
        if self.learningRates is not None:
            x.add_(self.learningRates.to(x.device) * dfdx, alpha=clr)
        else:
            x.add_(dfdx, alpha=clr)
        if self._shadow16 is not None:
            self._shadow16.copy_(x)
        return x, [fx]


__all__ = ["SGD", "LearningRateSchedule", "Default", "Regime", "EpochSchedule", "Poly", "Step", "MultiStep",
           "EpochDecay", "EpochStep", "NaturalExp", "Exponential", "Plateau", "Warmup", "SequentialSchedule",
           "EpochDecayWithWarmUp"]
