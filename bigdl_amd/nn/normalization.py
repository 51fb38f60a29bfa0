"""Normalization layers.

Reference: S/nn/BatchNormalization.scala:51 (447 LoC), SpatialBatchNormalization.scala (2,062 LoC; NCHW train
fwd :1211, bwd :1048), LayerNormalization.scala, SpatialCrossMapLRN.scala:43, SpatialWithinChannelLRN.scala,
Normalize.scala, NormalizeScale.scala, SpatialContrastive/Divisive/SubtractiveNormalization.scala.

GPU engine: (Spatial)BatchNormalization runs on csrc/batchnorm.hip. Statistics come for free from the conv
epilogue when a conv feeds the BN (``x._bn_stats``), the ReLU of a conv-BN-ReLU chain and the residual add +
ReLU of a ResNet block are fused into the apply pass (flags set by nn.fusion), and sync-BN across replicas
(reference ParameterSynchronizer, S/utils/ParameterSynchronizer.scala:25-106) is an RCCL all-reduce of the
packed [sum, sumsq] / [sum dy, sum dy*xhat] buffers between the reduce and apply phases.
"""
import math
import os

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import bn as bnops
from .abstractnn import AutogradModule, TensorModule, _t_begin, _t_end
from .init_methods import Ones, RandomUniform, Zeros

_ZMASK = os.environ.get("BIGDL_BN_ZMASK", "1") != "0"
# BIGDL_BN_DEFER=0: always materialise a training BN + ReLU output, even where nn.fusion found a consumer that applies
# it on load (ConvArgs::pre). See nn.fusion._defer_consumer for which consumers each level defers to.
_DEFER = [os.environ.get("BIGDL_BN_DEFER", "1") != "0"]
CL = torch.channels_last
BF16 = torch.bfloat16


class BatchNormalization(TensorModule):
    """BN over dim 2 (1-based) of (N, C) or (N, C, H, W) input."""

    def __init__(self, nOutput, eps=1e-5, momentum=0.1, affine=True, initWeight=None, initBias=None,
                 initGradWeight=None, initGradBias=None, dataFormat="NCHW"):
        super().__init__()
        self.nOutput = nOutput
        self.eps = eps
        self.momentum = momentum
        self.affine = affine
        self.dataFormat = dataFormat
        self.fuse_relu = False
        self.sync_fn = None          # sync-BN hook: fn(buffer[2C] fp32, count) -> total count
        if affine:
            self.register_parameter("weight", "gradWeight", torch.empty(nOutput))
            self.register_parameter("bias", "gradBias", torch.empty(nOutput))
        else:
            self.weight = self.bias = self.gradWeight = self.gradBias = None
        self.runningMean = torch.zeros(nOutput)
        self.runningVar = torch.ones(nOutput)
        self._buffers = ["runningMean", "runningVar"]
        self.saveMean = None
        self.saveStd = None
        self.weightInitMethod = RandomUniform(0.0, 1.0) if affine else None
        self.biasInitMethod = Zeros()
        self.reset()
        if initWeight is not None and affine:
            self.weight.copy_(torch.as_tensor(initWeight))
        if initBias is not None and affine:
            self.bias.copy_(torch.as_tensor(initBias))
        if initGradWeight is not None and affine:
            self.gradWeight.copy_(torch.as_tensor(initGradWeight))
        if initGradBias is not None and affine:
            self.gradBias.copy_(torch.as_tensor(initGradBias))

    def reset(self):
        if self.affine:
            with torch.no_grad():
                self.weightInitMethod.init(self.weight)
                self.biasInitMethod.init(self.bias)
        self.runningMean.zero_()
        self.runningVar.fill_(1.0)

    def setParallism(self, n):
        """Reference API (S/nn/BatchNormalization.scala:72-76) — enables sync-BN across the job."""
        from ..parallel.sync_bn import make_sync_fn

        self.sync_fn = make_sync_fn() if n and n > 1 else None
        return self

    def _to_nchw(self, x):
        if self.dataFormat == "NHWC" and x.dim() == 4:
            return x.permute(0, 3, 1, 2)
        return x

    def _from_nchw(self, y):
        if self.dataFormat == "NHWC" and y.dim() == 4:
            return y.permute(0, 2, 3, 1)
        return y

    def _gpu_ok(self, x):
        if not x.is_cuda or self.nOutput % 8 != 0:
            return False
        if x.dim() == 4:
            return True
        return x.dim() == 2

    def _prep_gpu(self, x):
        if x.dim() == 4:
            if x.dtype != BF16 or not x.is_contiguous(memory_format=CL):
                x = x.to(BF16, memory_format=CL)
        else:
            if x.dtype != BF16 or not x.is_contiguous():
                x = x.to(BF16).contiguous()
        return x

    def updateOutput(self, input, residual=None):
        if residual is None:     # a Graph's fused residual add (nn.fusion._fuse_graph_training)
            residual = self.__dict__.pop("_graph_residual", None)
        x = self._to_nchw(input)
        if self._gpu_ok(x):
            stats = getattr(input, "_bn_stats", None) if self.train else None
            x = self._prep_gpu(x)
            res = residual
            if res is not None and (res.dtype != BF16 or res.stride() != x.stride()):
                res = res.to(BF16).contiguous(memory_format=CL if x.dim() == 4 else torch.contiguous_format)
            # with a residual the ReLU mask is not a function of x: the apply pass stores it as one sign bit per
            # element, which the backward reads instead of the output itself (BIGDL_BN_ZMASK=0: read the output)
            zm = None
            if self.train and self.fuse_relu and res is not None and x.shape[1] % 8 == 0 and _ZMASK:
                zm = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device)
            if (self.train and self.fuse_relu and res is None and getattr(self, "_defer_ok", False) and _DEFER[0]
                    and x.dim() == 4 and self.dataFormat == "NCHW"):
                # the only consumer applies relu(x * scale + shift) on load: no apply pass, no output tensor
                # (nn.fusion plans this for BN -> ReLU -> conv / max pool)
                sm, si, aff = bnops.bn_prepare_gpu(x, self.weight, self.bias, self.runningMean, self.runningVar,
                                                   self.eps, self.momentum, stats=stats, sync_fn=self.sync_fn)
                self.saveMean, self.saveStd = sm, si
                self._aff, self._zm, self._xin = aff, None, x
                y = bnops.deferred(x, aff)
                y._bn_bwd = (self, x, sm, aff, False)
                return y
            y, sm, si, aff = bnops.bn_forward_gpu(x, self.weight, self.bias, self.runningMean, self.runningVar,
                                                   self.eps, self.momentum, self.train, stats=stats, res=res,
                                                   relu=self.fuse_relu, sync_fn=self.sync_fn if self.train else None,
                                                   zm=zm)
            self.saveMean, self.saveStd = sm, si
            # without a residual the ReLU mask is a function of x: backward recomputes it from (scale, shift)
            self._aff = aff if (self.fuse_relu and res is None) else None
            self._zm = zm
            self._xin = x
            if self.train and self.fuse_relu:
                # lets a consuming conv reduce this BN's backward statistics in its dgrad epilogue (nn.fusion)
                # (no reference to y itself: y -> _bn_bwd -> y was a reference cycle that kept every such output alive
                # until a GC pass, growing the caching allocator by ~5 GB per ResNet-50 step; the consuming conv's
                # input IS y, so it supplies the post-ReLU tensor itself)
                # last element: the sign mask, else whether the ReLU mask must come from y (a residual add)
                y._bn_bwd = (self, x, sm, self._aff, zm if zm is not None else res is not None)
            return self._from_nchw(y)
        xf = x.float()
        y, mean, invstd = bnops.bn_forward_cpu(xf, self.weight, self.bias, self.runningMean, self.runningVar, self.eps,
                                               self.momentum, self.train,
                                               sync_fn=self.sync_fn if self.train else None)
        if residual is not None:
            y = y + residual.float()
        if self.fuse_relu:
            y = torch.relu(y)
        self.saveMean, self.saveStd = mean, invstd
        self._xin = xf
        return self._from_nchw(y.to(input.dtype) if input.is_floating_point() else y)

    def _direct_grads(self):
        return (not self._frozen) and self.affine and self.scaleW == 1.0 and self.scaleB == 1.0

    def backward_fused(self, input, gradOutput, need_dres=False, sec=None):
        """GPU backward that also returns the residual-branch gradient (used by the fused ResNet block)."""
        gz = self._to_nchw(gradOutput)
        x = self._xin
        if gz.dtype != BF16 or gz.stride() != x.stride():
            gz = gz.to(BF16).contiguous(memory_format=CL if x.dim() == 4 else torch.contiguous_format)
        aff = getattr(self, "_aff", None)
        zm = getattr(self, "_zm", None)
        z = self._to_nchw(self.output) if (self.fuse_relu and aff is None and zm is None) else None
        direct = self._direct_grads()
        dg = self.gradWeight if direct else (torch.zeros_like(self.runningMean) if self.affine else None)
        db = self.gradBias if direct else (torch.zeros_like(self.runningMean) if self.affine else None)
        pre = getattr(gradOutput, "_bn_red", None)
        red = pre[1] if (pre is not None and pre[0] is self and self.train) else None
        graph_res = getattr(self, "_graph_dres", False)
        dx, dres = bnops.bn_backward_gpu(gz, z, x, self.saveMean, self.saveStd, self.weight, dg, db,
                                         training=self.train, need_dres=need_dres or graph_res,
                                         sync_fn=self.sync_fn if self.train else None, aff=aff, red=red, zm=zm,
                                         sec=sec)
        if graph_res:
            self._dres = dres
        if not direct and self.affine and not self._frozen:
            self.gradWeight.add_(dg, alpha=self.scaleW)
            self.gradBias.add_(db, alpha=self.scaleB)
        return self._from_nchw(dx), dres

    def backward(self, input, gradOutput):
        t0 = _t_begin(gradOutput)
        x = self._to_nchw(input)
        if self._gpu_ok(x):
            self.gradInput, _ = self.backward_fused(input, gradOutput)
        else:
            self.gradInput = self.updateGradInput(input, gradOutput)
            if not self._frozen:
                self.accGradParameters(input, gradOutput)
        _t_end(self, t0, "backward_time")
        return self.gradInput

    def _cpu_grads(self, gradOutput):
        gy = self._to_nchw(gradOutput).float()
        if self.fuse_relu:
            gy = gy * (self._to_nchw(self.output) > 0)
        return bnops.bn_backward_cpu(self._xin, gy, self.saveMean, self.saveStd, self.weight, self.train,
                                     sync_fn=self.sync_fn if self.train else None)

    def updateGradInput(self, input, gradOutput):
        x = self._to_nchw(input)
        if self._gpu_ok(x):
            dx, _ = self.backward_fused(input, gradOutput)
            return dx
        gx, dg, db = self._cpu_grads(gradOutput)
        self._pending = (dg, db)
        return self._from_nchw(gx.to(input.dtype))

    def accGradParameters(self, input, gradOutput):
        if not self.affine:
            return
        if input.is_cuda and self._gpu_ok(self._to_nchw(input)):
            return  # folded into backward_fused
        pend = getattr(self, "_pending", None)
        if pend is None:
            _, dg, db = self._cpu_grads(gradOutput)
        else:
            dg, db = pend
        self.gradWeight.add_(dg.to(self.gradWeight.device), alpha=self.scaleW)
        self.gradBias.add_(db.to(self.gradBias.device), alpha=self.scaleB)
        self._pending = None

    def __repr__(self):
        return f"{type(self).__name__}[{self.nOutput}, eps={self.eps}, momentum={self.momentum}, affine={self.affine}]"


class SpatialBatchNormalization(BatchNormalization):
    pass


class LayerNormalization(AutogradModule):
    def __init__(self, hiddenSize, eps=1e-6):
        super().__init__()
        self.hiddenSize, self.eps = hiddenSize, eps
        self.register_parameter("weight", "gradWeight", torch.ones(hiddenSize))
        self.register_parameter("bias", "gradBias", torch.zeros(hiddenSize))

    def fn(self, x):
        from ..ops.norm import layer_norm

        xf = x.float()
        y = layer_norm(xf, self.weight, self.bias, self.eps)     # native kernels on the GPU engine
        return y.to(x.dtype)


class SpatialCrossMapLRN(AutogradModule):
    """Cross-channel LRN: y = x / (k + alpha/size * sum_{window} x^2)^beta (reference :43)."""

    def __init__(self, size=5, alpha=1.0, beta=0.75, k=1.0, format="NCHW"):
        super().__init__()
        self.size, self.alpha, self.beta, self.k, self.format = size, alpha, beta, k, format

    def fn(self, x):
        from ..ops import nnk

        xf = x.float()
        if self.format == "NHWC":
            xf = xf.permute(0, 3, 1, 2)
        y = nnk.lrn(xf, self.size, self.alpha, self.beta, self.k)     # GPU: csrc/nn_misc.hip lrn kernels
        if self.format == "NHWC":
            y = y.permute(0, 2, 3, 1)
        return y.to(x.dtype)


class SpatialWithinChannelLRN(AutogradModule):
    def __init__(self, size=5, alpha=1.0, beta=0.75):
        super().__init__()
        self.size, self.alpha, self.beta = size, alpha, beta

    def fn(self, x):
        xf = x.float()
        p = (self.size - 1) // 2
        if xf.is_cuda and xf.dim() == 4:          # GPU: N-d window kernel (csrc/pool_nd.hip)
            from ..ops.pool_nd import pool2d_explicit

            oh, ow = xf.shape[2] + 2 * p - self.size + 1, xf.shape[3] + 2 * p - self.size + 1
            sq = pool2d_explicit(xf * xf, (self.size, self.size), (1, 1), (p, p), (oh, ow), False, True)
        else:
            sq = F.avg_pool2d(xf * xf, self.size, 1, p, count_include_pad=True)
        return (xf / (1 + self.alpha * sq) ** self.beta).to(x.dtype)


class Normalize(AutogradModule):
    """Lp-normalise each sample (reference Normalize.scala)."""

    def __init__(self, p=2.0, eps=1e-10):
        super().__init__()
        self.p, self.eps = p, eps

    def fn(self, x):
        xf = x.float()
        flat = xf.reshape(xf.shape[0], -1) if xf.dim() > 1 else xf.unsqueeze(0)
        if math.isinf(self.p):
            n = flat.abs().max(dim=1, keepdim=True).values
        else:
            n = flat.abs().pow(self.p).sum(dim=1, keepdim=True).pow(1.0 / self.p)
        return (flat / (n + self.eps)).reshape(xf.shape).to(x.dtype)


class NormalizeScale(AutogradModule):
    """L2-normalise across channels then scale per channel (SSD conv4_3 norm)."""

    def __init__(self, p, scale, size, wRegularizer=None, eps=1e-10):
        super().__init__()
        self.p, self.eps = p, eps
        self.register_parameter("weight", "gradWeight", torch.full(tuple(size), float(scale)))

    def fn(self, x):
        xf = x.float()
        n = xf.abs().pow(self.p).sum(dim=1, keepdim=True).pow(1.0 / self.p)
        return (xf / (n + self.eps) * self.weight).to(x.dtype)


def _gauss_kernel(n):
    k = torch.tensor([math.exp(-((i - (n - 1) / 2) ** 2) / (2 * (n / 4.0) ** 2)) for i in range(n)])
    return torch.outer(k, k) / torch.outer(k, k).sum()


class SpatialSubtractiveNormalization(AutogradModule):
    def __init__(self, nInputPlane=1, kernel=None):
        super().__init__()
        self.nInputPlane = nInputPlane
        self.kernel = torch.as_tensor(kernel).float() if kernel is not None else torch.ones(9, 9)
        if self.kernel.dim() == 1:
            self.kernel = torch.outer(self.kernel, self.kernel)
        self.kernel = self.kernel / (self.kernel.sum() * nInputPlane)

    def _mean(self, xf):
        k = self.kernel.to(xf.device)
        kh, kw = k.shape
        w = k.expand(1, self.nInputPlane, kh, kw)
        from ..ops import conv_fn

        m = conv_fn.conv2d(xf, w, None, (1, 1), (kh // 2, kw // 2))        # GPU: native implicit GEMM
        ones = torch.ones(1, self.nInputPlane, xf.shape[2], xf.shape[3], device=xf.device)
        coef = conv_fn.conv2d(ones, w, None, (1, 1), (kh // 2, kw // 2))
        return m / coef

    def fn(self, x):
        xf = x.float()
        sq = xf.dim() == 3
        if sq:
            xf = xf.unsqueeze(0)
        y = xf - self._mean(xf)
        return (y.squeeze(0) if sq else y).to(x.dtype)


class SpatialDivisiveNormalization(SpatialSubtractiveNormalization):
    def __init__(self, nInputPlane=1, kernel=None, threshold=1e-4, thresval=1e-4):
        super().__init__(nInputPlane, kernel)
        self.threshold, self.thresval = threshold, thresval

    def fn(self, x):
        xf = x.float()
        sq = xf.dim() == 3
        if sq:
            xf = xf.unsqueeze(0)
        std = self._mean(xf * xf).clamp_min(0).sqrt()
        mstd = std.mean(dim=(1, 2, 3), keepdim=True)
        div = torch.maximum(std, mstd)
        div = torch.where(div > self.threshold, div, torch.full_like(div, self.thresval))
        y = xf / div
        return (y.squeeze(0) if sq else y).to(x.dtype)


class SpatialContrastiveNormalization(AutogradModule):
    def __init__(self, nInputPlane=1, kernel=None, threshold=1e-4, thresval=1e-4):
        super().__init__()
        self.sub = SpatialSubtractiveNormalization(nInputPlane, kernel)
        self.div = SpatialDivisiveNormalization(nInputPlane, kernel, threshold, thresval)

    def fn(self, x):
        return self.div.fn(self.sub.fn(x))


__all__ = ["BatchNormalization", "SpatialBatchNormalization", "LayerNormalization", "SpatialCrossMapLRN",
           "SpatialWithinChannelLRN", "Normalize", "NormalizeScale", "SpatialSubtractiveNormalization",
           "SpatialDivisiveNormalization", "SpatialContrastiveNormalization"]
