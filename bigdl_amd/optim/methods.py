"""Optimization methods beyond SGD (reference S/optim/: Adam.scala:36, ParallelAdam.scala:38, Adagrad.scala,
Adadelta.scala, Adamax.scala, RMSprop.scala, Ftrl.scala:39, LBFGS.scala:48, LineSearch.scala, LarsSGD.scala:47).

All operate on the flat parameter tensor (or this rank's ZeRO-1 shard). On the GPU, Adam (csrc/elementwise.hip
adam_kernel) and Adagrad / RMSprop / Adadelta / Adamax / Ftrl (csrc/optim.hip) are single fused passes that also
write the bf16 compute copy of the weights; on the CPU they are short sequences of tensor ops over the flat buffer.
"""
import math

import torch

from ..ops import native
from .optim_method import OptimMethod, native_ok
from .sgd import Default, SGD


def _state(om, key, like, fill=0.0):
    t = om.state.get(key)
    if t is None or t.shape != like.shape or t.device != like.device:
        t = torch.full_like(like, fill)
        om.state[key] = t
    return t


def _sync_shadow(om, x):
    if om._shadow16 is not None:
        om._shadow16.copy_(x)


class Adam(OptimMethod):
    def __init__(self, learningRate=1e-3, learningRateDecay=0.0, beta1=0.9, beta2=0.999, Epsilon=1e-8,
                 weightDecay=0.0):
        super().__init__()
        self.learningRate, self.learningRateDecay = learningRate, learningRateDecay
        self.beta1, self.beta2, self.Epsilon, self.weightDecay = beta1, beta2, Epsilon, weightDecay

    def getLearningRate(self):
        t = self.state.get("evalCounter", 0)
        return -self.learningRate / (1 + t * self.learningRateDecay)

    def optimize(self, feval, x):
        fx, g = feval(x)
        t = self.state.get("evalCounter", 0)
        clr = self.learningRate / (1 + t * self.learningRateDecay)
        t += 1
        self.state["evalCounter"] = t
        m = _state(self, "s", x)
        v = _state(self, "r", x)
        bc1 = 1 - self.beta1 ** t
        bc2 = 1 - self.beta2 ** t
        if native_ok(x, g, m, v):
            native.get().adam_step(x, g, m, v, self._shadow16, clr, self.beta1, self.beta2, self.Epsilon,
                                   self.weightDecay, bc1, bc2)
            return x, [fx]
        if self.weightDecay:
            g = g + self.weightDecay * x
        m.mul_(self.beta1).add_(g, alpha=1 - self.beta1)
        v.mul_(self.beta2).addcmul_(g, g, value=1 - self.beta2)
        denom = v.sqrt().add_(self.Epsilon)
        x.addcdiv_(m, denom, value=-clr * math.sqrt(bc2) / bc1)
        _sync_shadow(self, x)
        return x, [fx]


class ParallelAdam(Adam):
    """Reference ParallelAdam splits the update over CPU threads; on the GPU the fused kernel is already
    parallel over the whole buffer, so the maths (and this class) equal Adam."""

    def __init__(self, learningRate=1e-3, learningRateDecay=0.0, beta1=0.9, beta2=0.999, Epsilon=1e-8,
                 parallelNum=None):
        super().__init__(learningRate, learningRateDecay, beta1, beta2, Epsilon)


class Adagrad(OptimMethod):
    def __init__(self, learningRate=1e-3, learningRateDecay=0.0, weightDecay=0.0):
        super().__init__()
        self.learningRate, self.learningRateDecay, self.weightDecay = learningRate, learningRateDecay, weightDecay

    def optimize(self, feval, x):
        fx, g = feval(x)
        n = self.state.get("evalCounter", 0)
        clr = self.learningRate / (1 + n * self.learningRateDecay)
        var = _state(self, "paramVariance", x)
        if native_ok(x, g, var):
            native.get().optim_step(0, x, g, var, None, self._shadow16, clr, self.weightDecay, 0.0, 0.0, 0.0)
            self.state["evalCounter"] = n + 1
            return x, [fx]
        if self.weightDecay:
            g = g + self.weightDecay * x
        var.addcmul_(g, g)
        x.addcdiv_(g, var.sqrt().add_(1e-10), value=-clr)
        self.state["evalCounter"] = n + 1
        _sync_shadow(self, x)
        return x, [fx]


class Adadelta(OptimMethod):
    def __init__(self, decayRate=0.9, Epsilon=1e-10):
        super().__init__()
        self.decayRate, self.Epsilon = decayRate, Epsilon

    def optimize(self, feval, x):
        fx, g = feval(x)
        rho, eps = self.decayRate, self.Epsilon
        var = _state(self, "paramVariance", x)
        acc = _state(self, "accDelta", x)
        if native_ok(x, g, var, acc):
            native.get().optim_step(2, x, g, var, acc, self._shadow16, rho, eps, 0.0, 0.0, 0.0)
            self.state["evalCounter"] = self.state.get("evalCounter", 0) + 1
            return x, [fx]
        var.mul_(rho).addcmul_(g, g, value=1 - rho)
        delta = (acc + eps).sqrt().div_((var + eps).sqrt()).mul_(g)
        x.sub_(delta)
        acc.mul_(rho).addcmul_(delta, delta, value=1 - rho)
        self.state["evalCounter"] = self.state.get("evalCounter", 0) + 1
        _sync_shadow(self, x)
        return x, [fx]


class Adamax(OptimMethod):
    def __init__(self, learningRate=0.002, beta1=0.9, beta2=0.999, Epsilon=1e-38):
        super().__init__()
        self.learningRate, self.beta1, self.beta2, self.Epsilon = learningRate, beta1, beta2, Epsilon

    def optimize(self, feval, x):
        fx, g = feval(x)
        t = self.state.get("evalCounter", 0) + 1
        self.state["evalCounter"] = t
        m = _state(self, "m", x)
        u = _state(self, "u", x)
        if native_ok(x, g, m, u):
            native.get().optim_step(3, x, g, m, u, self._shadow16, self.learningRate / (1 - self.beta1 ** t),
                                    self.beta1, self.beta2, self.Epsilon, 0.0)
            return x, [fx]
        m.mul_(self.beta1).add_(g, alpha=1 - self.beta1)
        torch.maximum(u * self.beta2, g.abs() + self.Epsilon, out=u)
        x.addcdiv_(m, u, value=-self.learningRate / (1 - self.beta1 ** t))
        _sync_shadow(self, x)
        return x, [fx]


class RMSprop(OptimMethod):
    def __init__(self, learningRate=1e-2, learningRateDecay=0.0, decayRate=0.99, Epsilon=1e-8):
        super().__init__()
        self.learningRate, self.learningRateDecay = learningRate, learningRateDecay
        self.decayRate, self.Epsilon = decayRate, Epsilon

    def optimize(self, feval, x):
        fx, g = feval(x)
        n = self.state.get("evalCounter", 0)
        clr = self.learningRate / (1 + n * self.learningRateDecay)
        ms = _state(self, "sumSquare", x)
        if native_ok(x, g, ms):
            native.get().optim_step(1, x, g, ms, None, self._shadow16, clr, self.decayRate, self.Epsilon, 0.0, 0.0)
            self.state["evalCounter"] = n + 1
            return x, [fx]
        ms.mul_(self.decayRate).addcmul_(g, g, value=1 - self.decayRate)
        x.addcdiv_(g, ms.sqrt().add_(self.Epsilon), value=-clr)
        self.state["evalCounter"] = n + 1
        _sync_shadow(self, x)
        return x, [fx]


class Ftrl(OptimMethod):
    """FTRL-proximal (reference Ftrl.scala:39; same as TensorFlow's FtrlOptimizer)."""

    def __init__(self, learningRate=1e-3, learningRatePower=-0.5, initialAccumulatorValue=0.1,
                 l1RegularizationStrength=0.0, l2RegularizationStrength=0.0, l2ShrinkageRegularizationStrength=0.0):
        super().__init__()
        self.learningRate, self.learningRatePower = learningRate, learningRatePower
        self.initialAccumulatorValue = initialAccumulatorValue
        self.l1, self.l2, self.l2s = l1RegularizationStrength, l2RegularizationStrength, \
            l2ShrinkageRegularizationStrength

    def optimize(self, feval, x):
        fx, g = feval(x)
        lr, p = self.learningRate, self.learningRatePower
        accum = _state(self, "accum", x, self.initialAccumulatorValue)
        linear = _state(self, "linear", x)
        if native_ok(x, g, accum, linear):
            native.get().optim_step(4, x, g, accum, linear, self._shadow16, lr, p, self.l1, self.l2, self.l2s)
            self.state["evalCounter"] = self.state.get("evalCounter", 0) + 1
            return x, [fx]
        gs = g + 2 * self.l2s * x if self.l2s > 0 else g
        acc_new = accum + g * g
        if p == -0.5:
            sigma = (acc_new.sqrt() - accum.sqrt()) / lr
            quad = acc_new.sqrt() / lr + 2 * self.l2
        else:
            sigma = (acc_new.pow(-p) - accum.pow(-p)) / lr
            quad = acc_new.pow(-p) / lr + 2 * self.l2
        linear.add_(gs - sigma * x)
        l1 = torch.sign(linear) * self.l1
        newx = torch.where(linear.abs() > self.l1, (l1 - linear) / quad, torch.zeros_like(x))
        x.copy_(newx)
        accum.copy_(acc_new)
        self.state["evalCounter"] = self.state.get("evalCounter", 0) + 1
        _sync_shadow(self, x)
        return x, [fx]


class LineSearch:
    def __call__(self, opfunc, x, t, d, f, g, gtd, options=None):
        raise NotImplementedError


class LBFGS(OptimMethod):
    """Limited-memory BFGS with optional strong-Wolfe line search (reference LBFGS.scala:48)."""

    def __init__(self, maxIter=20, maxEval=None, tolFun=1e-5, tolX=1e-9, nCorrection=100, learningRate=1.0,
                 verbose=False, lineSearch=None, lineSearchOptions=None):
        super().__init__()
        self.maxIter, self.maxEval = maxIter, maxEval if maxEval is not None else int(maxIter * 1.25)
        self.tolFun, self.tolX, self.nCorrection, self.learningRate = tolFun, tolX, nCorrection, learningRate
        self.lineSearch = lineSearch

    def optimize(self, feval, x):
        f, g = feval(x)
        f = float(f)
        fs = [f]
        g = g.clone()
        if g.abs().sum() <= self.tolFun:
            return x, fs
        old_dirs, old_stps = [], []
        H_diag = 1.0
        d = -g
        t = min(1.0, 1.0 / float(g.abs().sum())) * self.learningRate
        g_old = g.clone()
        f_old = f
        n_iter, n_eval = 0, 1
        while n_iter < self.maxIter:
            n_iter += 1
            if n_iter > 1:
                y = g - g_old
                s = d * t
                ys = float(y @ s)
                if ys > 1e-10:
                    if len(old_dirs) == self.nCorrection:
                        old_dirs.pop(0)
                        old_stps.pop(0)
                    old_dirs.append(s)
                    old_stps.append(y)
                    H_diag = ys / float(y @ y)
                q = -g.clone()
                al = []
                for s_i, y_i in zip(reversed(old_dirs), reversed(old_stps)):
                    ro = 1.0 / float(y_i @ s_i)
                    a = ro * float(s_i @ q)
                    al.append((a, ro, s_i, y_i))
                    q.add_(y_i, alpha=-a)
                r = q * H_diag
                for a, ro, s_i, y_i in reversed(al):
                    be = ro * float(y_i @ r)
                    r.add_(s_i, alpha=a - be)
                d = r
                t = self.learningRate
            g_old = g.clone()
            f_old = f
            gtd = float(g @ d)
            if gtd > -self.tolX:
                break
            x.add_(d, alpha=t)
            f, g = feval(x)
            f = float(f)
            g = g.clone()
            n_eval += 1
            fs.append(f)
            if n_iter == self.maxIter or n_eval >= self.maxEval:
                break
            if g.abs().sum() <= self.tolFun:
                break
            if (d * t).abs().sum() <= self.tolX:
                break
            if abs(f - f_old) < self.tolX:
                break
        self.state["evalCounter"] = self.state.get("evalCounter", 0) + n_iter
        _sync_shadow(self, x)
        return x, fs


class LarsSGD(SGD):
    """Layer-wise adaptive rate scaling: rate = trust * lr * ||w|| / (||g|| + wd * ||w||) per parameter block
    (reference LarsSGD.scala:47; use one LarsSGD per layer via ``Optimizer.setOptimMethods`` and
    ``LarsSGD.createOptimForModule``)."""

    def __init__(self, lrScheduler=None, trust=1.0, _learningRate=1e-3, _learningRateDecay=0.0, _weightDecay=0.0,
                 _momentum=0.0):
        super().__init__(_learningRate, _learningRateDecay, _weightDecay, _momentum,
                         learningRateSchedule=lrScheduler or Default())
        self.trust = trust
        self._calculated_scale = None

    def setGradientScale(self, scale):
        self._calculated_scale = scale

    def optimize(self, feval, x):
        fx, g = feval(x)
        v = _state(self, "v", x)
        self.learningRateSchedule.updateHyperParameter(self)
        global_lr = -self.learningRateSchedule.currentRate * self.trust
        if self._calculated_scale is not None:
            scale = self._calculated_scale          # layer-global scale from LarsProcessor (device tensor ok)
            self._calculated_scale = None
        else:
            nw = float(x.norm())
            ng = float(g.norm())
            scale = (ng + self.weightDecay * nw) / nw if nw > 0 else float("inf")
            # reference getGradientScale guards (LarsSGD.scala:100-112)
            if math.isinf(scale):
                scale = 10000.0
            elif math.isnan(scale):
                scale = 1.0
            elif abs(scale) < 1e-4:
                scale = 1e-4
        rate = global_lr / scale
        v.mul_(self.momentum).add_((g + self.weightDecay * x) * rate)
        x.sub_(v)
        _sync_shadow(self, x)
        return x, [fx]

    @staticmethod
    def createOptimForModule(model, lrScheduler=None, trust=1.0, learningRate=1e-3, learningRateDecay=0.0,
                             weightDecay=0.0, momentum=0.0):
        out = {}
        for m in model.flattened_layers():
            if not m.modules_list() and m.parameters() is not None:
                out[m.getName()] = LarsSGD(lrScheduler, trust, learningRate, learningRateDecay, weightDecay, momentum)
        return out


__all__ = ["Adam", "ParallelAdam", "Adagrad", "Adadelta", "Adamax", "RMSprop", "Ftrl", "LBFGS", "LineSearch",
           "LarsSGD"]
