"""Activation / element-wise layers.

Reference (S/nn/*.scala): ReLU 42 (= Threshold(0, 0)), ReLU6, Threshold 421, BinaryThreshold, LeakyReLU, PReLU,
RReLU, SReLU, ELU, Sigmoid, HardSigmoid, Tanh, HardTanh, TanhShrink, SoftPlus, SoftSign, SoftShrink,
HardShrink, LogSigmoid, SoftMax, SoftMin, LogSoftMax, Exp, Log, Sqrt, Square, Abs, Power, Clamp,
AddConstant, MulConstant, Negative, GradientReversal, Mul, Add, CMul, CAdd, Scale.

ReLU has an explicit native path (csrc/elementwise.hip, and is fused into the producing conv / BN on the
GPU engine — see nn/fusion.py); the point-wise activations below run native forward / backward kernels on the GPU
(csrc/activation.hip, ``_NativeActivation``); the rest derive their backward from a functional forward.
"""
import torch
import torch.nn.functional as F

from .. import ops
from .abstractnn import AutogradModule, TensorModule
from .init_methods import RandomUniform

BF16 = torch.bfloat16
CL = torch.channels_last


class ReLU(TensorModule):
    def __init__(self, ip=False):
        super().__init__()
        self.inplace = ip
        self.passthrough = False   # set by nn.fusion when the producer already applied the ReLU

    def updateOutput(self, input):
        if self.passthrough:
            return input
        if input.is_cuda and input.dtype == BF16 and _dense(input):
            return ops.relu_gpu(input, out=input if self.inplace else None)
        return torch.relu(input)

    def updateGradInput(self, input, gradOutput):
        if self.passthrough:
            return gradOutput
        out = self.output
        if out.is_cuda and out.dtype == BF16 and _dense(out):
            return ops.relu_bwd_gpu(gradOutput, out)
        return gradOutput * (out > 0).to(gradOutput.dtype)


def _dense(t):
    return t.is_contiguous() or (t.dim() == 4 and t.is_contiguous(memory_format=CL))


# kind codes of csrc/activation.hip
_NATIVE_KIND = {"Tanh": 0, "Sigmoid": 1, "ELU": 2, "LeakyReLU": 3, "ReLU6": 4, "SoftPlus": 5, "SoftSign": 6,
                "HardTanh": 7, "HardSigmoid": 8, "LogSigmoid": 9, "TanhShrink": 10, "SoftShrink": 11,
                "HardShrink": 12, "Threshold": 13, "Exp": 14, "Log": 15, "Sqrt": 16, "Square": 17, "Abs": 18}


class _NativeActivation(AutogradModule):
    """Point-wise layer with a native GPU forward / backward (csrc/activation.hip) for dense bf16 / fp32 device
    tensors; anything else (CPU, other dtypes, strided views) takes the autograd path of ``fn``."""

    _kind = None

    def _native_args(self):
        return 0.0, 0.0

    def _native_ok(self, x):
        return (isinstance(x, torch.Tensor) and x.is_cuda and x.dtype in (BF16, torch.float32) and _dense(x)
                and self._kind is not None)

    def updateOutput(self, input):
        if self._native_ok(input):
            from ..ops import native

            a, b = self._native_args()
            y = torch.empty_like(input)
            native.get().act_fwd(input, y, _NATIVE_KIND[self._kind], float(a), float(b))
            self._ag = None
            self._native_x = input
            return y
        self._native_x = None
        return super().updateOutput(input)

    def updateGradInput(self, input, gradOutput):
        x = getattr(self, "_native_x", None)
        if x is not None:
            from ..ops import native

            a, b = self._native_args()
            y = self.output
            g = gradOutput.to(x.dtype)
            if g.stride() != x.stride():
                g = g.contiguous(memory_format=CL) if x.dim() == 4 and not x.is_contiguous() else g.contiguous()
            dx = torch.empty_like(x)
            native.get().act_bwd(x, y, g, dx, _NATIVE_KIND[self._kind], float(a), float(b))
            self._pending_param_grads = None
            return dx
        return super().updateGradInput(input, gradOutput)


class Threshold(_NativeActivation):
    _kind = "Threshold"

    def _native_args(self):
        return self.threshold, self.value

    def __init__(self, th=1e-6, v=0.0, ip=False):
        super().__init__()
        self.threshold, self.value, self.inplace = th, v, ip

    def fn(self, x):
        return torch.where(x > self.threshold, x, torch.full_like(x, self.value))


class BinaryThreshold(AutogradModule):
    def __init__(self, th=1e-6, ip=False):
        super().__init__()
        self.threshold = th

    def fn(self, x):
        return (x > self.threshold).to(x.dtype)


class ReLU6(_NativeActivation):
    _kind = "ReLU6"

    def __init__(self, inplace=False):
        super().__init__()

    def fn(self, x):
        return torch.clamp(x, 0.0, 6.0)


class LeakyReLU(_NativeActivation):
    _kind = "LeakyReLU"

    def _native_args(self):
        return self.negval, 0.0

    def __init__(self, negval=0.01, inplace=False):
        super().__init__()
        self.negval = negval

    def fn(self, x):
        return F.leaky_relu(x, self.negval)


class ELU(_NativeActivation):
    _kind = "ELU"

    def _native_args(self):
        return self.alpha, 0.0

    def __init__(self, alpha=1.0, inplace=False):
        super().__init__()
        self.alpha = alpha

    def fn(self, x):
        return F.elu(x, self.alpha)


class PReLU(AutogradModule):
    def __init__(self, nOutputPlane=0):
        super().__init__()
        self.nOutputPlane = nOutputPlane
        self.register_parameter("weight", "gradWeight", torch.full((max(nOutputPlane, 1),), 0.25))

    def fn(self, x):
        w = self.weight.to(x.dtype)
        if self.nOutputPlane == 0:
            return torch.where(x > 0, x, w[0] * x)
        shape = [1, -1] + [1] * (x.dim() - 2) if x.dim() > 1 else [-1]
        return torch.where(x > 0, x, w.view(shape) * x)


class RReLU(AutogradModule):
    def __init__(self, lower=1.0 / 8, upper=1.0 / 3, inplace=False):
        super().__init__()
        self.lower, self.upper = lower, upper

    def fn(self, x):
        if self.train:
            a = torch.empty_like(x).uniform_(self.lower, self.upper)
            return torch.where(x >= 0, x, x * a)
        return torch.where(x >= 0, x, x * ((self.lower + self.upper) / 2))


class SReLU(AutogradModule):
    """S-shaped ReLU with learnable (tLeft, aLeft, tRight, aRight) per feature."""

    def __init__(self, shape, sharedAxes=None):
        super().__init__()
        shape = tuple(shape)
        self.register_parameter("weight", "gradWeight", torch.zeros(shape))          # tLeft
        self.register_parameter("aLeft", "gradALeft", torch.empty(shape).uniform_(0, 1))
        self.register_parameter("tRight", "gradTRight", torch.empty(shape).uniform_(0, 5))
        self.register_parameter("aRight", "gradARight", torch.ones(shape))

    def fn(self, x):
        tl, al, tr, ar = self.weight, self.aLeft, self.tRight, self.aRight
        tr_abs = tl + tr.abs()
        y = torch.where(x >= tr_abs, tr_abs + ar * (x - tr_abs), x)
        return torch.where(x <= tl, tl + al * (x - tl), y)


class Sigmoid(_NativeActivation):
    _kind = "Sigmoid"

    def fn(self, x):
        return torch.sigmoid(x)


class HardSigmoid(_NativeActivation):
    _kind = "HardSigmoid"

    def fn(self, x):
        return torch.clamp(0.2 * x + 0.5, 0.0, 1.0)


class Tanh(_NativeActivation):
    _kind = "Tanh"

    def fn(self, x):
        return torch.tanh(x)


class HardTanh(_NativeActivation):
    _kind = "HardTanh"

    def _native_args(self):
        return self.minValue, self.maxValue

    def __init__(self, minValue=-1.0, maxValue=1.0, inplace=False):
        super().__init__()
        self.minValue, self.maxValue = minValue, maxValue

    def fn(self, x):
        return torch.clamp(x, self.minValue, self.maxValue)


class Clamp(HardTanh):
    def __init__(self, min, max):
        super().__init__(min, max)


class TanhShrink(_NativeActivation):
    _kind = "TanhShrink"

    def fn(self, x):
        return x - torch.tanh(x)


class SoftPlus(_NativeActivation):
    _kind = "SoftPlus"

    def _native_args(self):
        return self.beta, 0.0

    def __init__(self, beta=1.0):
        super().__init__()
        self.beta = beta

    def fn(self, x):
        return F.softplus(x, self.beta, 20.0)


class SoftSign(_NativeActivation):
    _kind = "SoftSign"

    def fn(self, x):
        return x / (1 + x.abs())


class SoftShrink(_NativeActivation):
    _kind = "SoftShrink"

    def _native_args(self):
        return self.lambd, 0.0

    def __init__(self, lambd=0.5):
        super().__init__()
        self.lambd = lambd

    def fn(self, x):
        return F.softshrink(x, self.lambd)


class HardShrink(_NativeActivation):
    _kind = "HardShrink"

    def _native_args(self):
        return self.lambd, 0.0

    def __init__(self, lambd=0.5):
        super().__init__()
        self.lambd = lambd

    def fn(self, x):
        return F.hardshrink(x, self.lambd)


class LogSigmoid(_NativeActivation):
    _kind = "LogSigmoid"

    def fn(self, x):
        return F.logsigmoid(x)


def _softmax_dim(x, pos_dim):
    if pos_dim is not None and pos_dim >= 0:
        return pos_dim
    return 0 if x.dim() in (1, 3) else 1


class SoftMax(AutogradModule):
    def __init__(self, pos=None):
        super().__init__()
        self.pos = pos

    def fn(self, x):
        from ..ops import nnk

        return nnk.softmax(x, _softmax_dim(x, self.pos)).to(x.dtype)    # GPU, last dim: native (ops/nnk.py)


class SoftMin(AutogradModule):
    def fn(self, x):
        from ..ops import nnk

        return nnk.softmax(-x, _softmax_dim(x, None)).to(x.dtype)


class LogSoftMax(AutogradModule):
    def fn(self, x):
        from ..ops import nnk

        return nnk.log_softmax(x).to(x.dtype)          # last dim; GPU: one wave per row (csrc/nn_misc.hip)


class Exp(_NativeActivation):
    _kind = "Exp"

    def fn(self, x):
        return torch.exp(x)


class Log(_NativeActivation):
    _kind = "Log"

    def fn(self, x):
        return torch.log(x)


class Sqrt(_NativeActivation):
    _kind = "Sqrt"

    def fn(self, x):
        return torch.sqrt(x)


class Square(_NativeActivation):
    _kind = "Square"

    def fn(self, x):
        return x * x


class Abs(_NativeActivation):
    _kind = "Abs"

    def fn(self, x):
        return x.abs()


class Power(AutogradModule):
    """y = (shift + scale * x) ^ power."""

    def __init__(self, power, scale=1.0, shift=0.0):
        super().__init__()
        self.power, self.scale, self.shift = power, scale, shift

    def fn(self, x):
        return torch.pow(self.shift + self.scale * x, self.power)


class AddConstant(AutogradModule):
    def __init__(self, constant_scalar, inplace=False):
        super().__init__()
        self.constant_scalar = constant_scalar

    def fn(self, x):
        return x + self.constant_scalar


class MulConstant(AutogradModule):
    def __init__(self, scalar, inplace=False):
        super().__init__()
        self.scalar = scalar

    def fn(self, x):
        return x * self.scalar


class Negative(AutogradModule):
    def __init__(self, inplace=False):
        super().__init__()

    def fn(self, x):
        return -x


class GradientReversal(TensorModule):
    def __init__(self, the_lambda=1.0):
        super().__init__()
        self.the_lambda = the_lambda

    def updateOutput(self, input):
        return input

    def updateGradInput(self, input, gradOutput):
        return -self.the_lambda * gradOutput


class Identity(TensorModule):
    def updateOutput(self, input):
        return input

    def updateGradInput(self, input, gradOutput):
        return gradOutput


class Echo(TensorModule):
    """Prints activations and gradients passing through (debugging, reference Echo.scala); ``feval`` /
    ``beval`` replace the printing with callbacks ``fn(module, tensor)``."""

    def __init__(self, feval=None, beval=None):
        super().__init__()
        self.feval = feval
        self.beval = beval

    def updateOutput(self, input):
        if self.feval is not None:
            self.feval(self, input)
        else:
            print(f"{self.getName()} : Activation size is {_shape(input)}")
        return input

    def updateGradInput(self, input, gradOutput):
        if self.beval is not None:
            self.beval(self, gradOutput)
        else:
            print(f"{self.getName()} : Gradient size is {_shape(gradOutput)}")
        return gradOutput


def _shape(a):
    return tuple(a.shape) if isinstance(a, torch.Tensor) else a


class Mul(AutogradModule):
    """Multiply by a single learnable scalar."""

    def __init__(self):
        super().__init__()
        self.register_parameter("weight", "gradWeight", torch.empty(1))
        self.reset()

    def reset(self):
        RandomUniform(-1.0, 1.0).init(self.weight)

    def fn(self, x):
        return x * self.weight.to(x.dtype)


class Add(AutogradModule):
    """Add a learnable bias vector of size inputSize."""

    def __init__(self, inputSize, scaleB=1.0):
        super().__init__()
        self.register_parameter("bias", "gradBias", torch.empty(inputSize))
        self.scaleB = scaleB
        RandomUniform(-1.0 / inputSize ** 0.5, 1.0 / inputSize ** 0.5).init(self.bias)

    def fn(self, x):
        return x + self.bias.to(x.dtype).view((1,) * (x.dim() - 1) + (-1,)) if x.dim() > 1 else x + self.bias


class CMul(AutogradModule):
    """Component-wise multiply by a learnable tensor broadcast to the input (reference CMul.scala)."""

    def __init__(self, size, wRegularizer=None):
        super().__init__()
        self.size = tuple(size)
        self.wRegularizer = wRegularizer
        self.register_parameter("weight", "gradWeight", torch.empty(self.size))
        n = 1
        for s in self.size:
            n *= s
        RandomUniform(-1.0 / n ** 0.5, 1.0 / n ** 0.5).init(self.weight)

    def fn(self, x):
        w = self.weight.to(x.dtype)
        if w.dim() < x.dim():
            w = w.view((1,) * (x.dim() - w.dim()) + tuple(w.shape))
        return x * w


class CAdd(AutogradModule):
    def __init__(self, size, bRegularizer=None):
        super().__init__()
        self.size = tuple(size)
        self.bRegularizer = bRegularizer
        self.register_parameter("bias", "gradBias", torch.empty(self.size))
        n = 1
        for s in self.size:
            n *= s
        RandomUniform(-1.0 / n ** 0.5, 1.0 / n ** 0.5).init(self.bias)

    def fn(self, x):
        b = self.bias.to(x.dtype)
        if b.dim() < x.dim():
            b = b.view((1,) * (x.dim() - b.dim()) + tuple(b.shape))
        return x + b


class Scale(AutogradModule):
    """CMul followed by CAdd with the same broadcast shape (Caffe Scale layer)."""

    def __init__(self, size):
        super().__init__()
        self.size = tuple(size)
        self.register_parameter("weight", "gradWeight", torch.ones(self.size))
        self.register_parameter("bias", "gradBias", torch.zeros(self.size))

    def fn(self, x):
        w, b = self.weight.to(x.dtype), self.bias.to(x.dtype)
        if w.dim() < x.dim():
            shape = (1,) * (x.dim() - w.dim()) + tuple(w.shape)
            w, b = w.view(shape), b.view(shape)
        return x * w + b


__all__ = [n for n in list(globals()) if n[0].isupper() and n not in ("F", "BF16", "CL")]
