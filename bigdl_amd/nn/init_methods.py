"""Initialization methods (reference: S/nn/InitializationMethod.scala — Zeros, Ones, ConstInitMethod,
RandomUniform, RandomNormal, Xavier, MsraFiller, BilinearFiller; VariableFormat fan-in/out rules)."""
import math

import torch

from ..utils.random_generator import RNG


class VariableFormat:
    """How fan-in / fan-out are read from a weight shape."""

    DEFAULT = "default"          # (out, in, ...) — conv OIHW / linear (out, in)
    ONE_D = "one_d"
    IN_OUT = "in_out"
    OUT_IN = "out_in"
    GP_OUT_IN_KW_KH = "gp_out_in_kw_kh"

    @staticmethod
    def fans(shape, fmt=None):
        shape = list(shape)
        if len(shape) == 1:
            return shape[0], shape[0]
        if fmt == VariableFormat.IN_OUT:
            return shape[0], shape[1]
        receptive = 1
        for d in shape[2:]:
            receptive *= d
        return shape[1] * receptive, shape[0] * receptive


class InitializationMethod:
    def init(self, t, fmt=None):
        raise NotImplementedError

    def __call__(self, t, fmt=None):
        return self.init(t, fmt)


class Zeros(InitializationMethod):
    def init(self, t, fmt=None):
        return t.zero_()


class Ones(InitializationMethod):
    def init(self, t, fmt=None):
        return t.fill_(1.0)


class ConstInitMethod(InitializationMethod):
    def __init__(self, value):
        self.value = value

    def init(self, t, fmt=None):
        return t.fill_(self.value)


class RandomUniform(InitializationMethod):
    """U(lower, upper); with no bounds: U(-1/sqrt(fanIn), 1/sqrt(fanIn)) (reference default)."""

    def __init__(self, lower=None, upper=None):
        self.lower, self.upper = lower, upper

    def init(self, t, fmt=None):
        if self.lower is None:
            fan_in, _ = VariableFormat.fans(t.shape, fmt)
            std = 1.0 / math.sqrt(max(fan_in, 1))
            lo, hi = -std, std
        else:
            lo, hi = self.lower, self.upper
        t.copy_(RNG.uniform(lo, hi, tuple(t.shape)).to(t.device, t.dtype))
        return t


class RandomNormal(InitializationMethod):
    def __init__(self, mean=0.0, stdv=1.0):
        self.mean, self.stdv = mean, stdv

    def init(self, t, fmt=None):
        t.copy_(RNG.normal(self.mean, self.stdv, tuple(t.shape)).to(t.device, t.dtype))
        return t


class Xavier(InitializationMethod):
    def __init__(self, varianceNormAverage=True):
        self.avg = varianceNormAverage

    def init(self, t, fmt=None):
        fan_in, fan_out = VariableFormat.fans(t.shape, fmt)
        n = (fan_in + fan_out) / 2.0 if self.avg else fan_in
        stdv = math.sqrt(3.0 / n)
        t.copy_(RNG.uniform(-stdv, stdv, tuple(t.shape)).to(t.device, t.dtype))
        return t


class MsraFiller(InitializationMethod):
    """He init: N(0, sqrt(2/n)), n = fanIn (varianceNormAverage=False) or average of fans."""

    def __init__(self, varianceNormAverage=True):
        self.avg = varianceNormAverage

    def init(self, t, fmt=None):
        fan_in, fan_out = VariableFormat.fans(t.shape, fmt)
        n = (fan_in + fan_out) / 2.0 if self.avg else fan_out
        std = math.sqrt(2.0 / max(n, 1))
        t.copy_(RNG.normal(0.0, std, tuple(t.shape)).to(t.device, t.dtype))
        return t


class BilinearFiller(InitializationMethod):
    def init(self, t, fmt=None):
        kh, kw = t.shape[-2], t.shape[-1]
        f = math.ceil(kw / 2.0)
        c = (2 * f - 1 - f % 2) / (2.0 * f)
        w = torch.zeros(kh, kw)
        for i in range(kh):
            for j in range(kw):
                w[i, j] = (1 - abs(j / f - c)) * (1 - abs(i / f - c))
        t.copy_(w.expand_as(t))
        return t


__all__ = ["VariableFormat", "InitializationMethod", "Zeros", "Ones", "ConstInitMethod", "RandomUniform",
           "RandomNormal", "Xavier", "MsraFiller", "BilinearFiller"]
