"""Pooling layers. Reference: S/nn/SpatialMaxPooling.scala:62, SpatialAveragePooling.scala:62,
VolumetricMaxPooling.scala, VolumetricAveragePooling.scala, TemporalMaxPooling.scala; primitives in
NNPrimitive.scala:654-1051. GPU engine: 2D NHWC kernels in csrc/elementwise.hip, 3D / temporal pooling on the
N-d window kernels of csrc/pool_nd.hip."""
import os

import torch
import torch.nn.functional as F

from ..ops import bn as bnops
from ..ops import pool as P
from ..ops import pool_nd as PN
from .abstractnn import AutogradModule, TensorModule

# BIGDL_POOL_BN_RED=0: the stem BN's backward reduction runs as its own pass instead of inside the pool backward
_POOL_BN_RED = os.environ.get("BIGDL_POOL_BN_RED", "1") != "0"

BF16 = torch.bfloat16
CL = torch.channels_last


def _same(inp, k, s):
    out = -(-inp // s)
    total = max((out - 1) * s + k - inp, 0)
    return total // 2


def _gpu_ok(x):
    return x.is_cuda and x.dim() == 4 and x.shape[1] % 8 == 0


def _prep(x):
    if x.dtype != BF16 or not x.is_contiguous(memory_format=CL):
        x = x.to(BF16, memory_format=CL)
    return x


class SpatialMaxPooling(TensorModule):
    def __init__(self, kW, kH, dW=None, dH=None, padW=0, padH=0, format="NCHW"):
        super().__init__()
        self.kW, self.kH = kW, kH
        self.dW, self.dH = dW if dW is not None else kW, dH if dH is not None else kH
        self.padW, self.padH = padW, padH
        self.format = format
        self.ceilMode = False

    def ceil(self):
        self.ceilMode = True
        return self

    def floor(self):
        self.ceilMode = False
        return self

    def _pads(self, H, W):
        if self.padW == -1 and self.padH == -1:
            return _same(H, self.kH, self.dH), _same(W, self.kW, self.dW)
        return self.padH, self.padW

    def updateOutput(self, input):
        pre = getattr(input, "_bn_pre", None)
        if pre is not None and not (self.format == "NCHW" and input.dim() == 4 and _gpu_ok(input)
                                    and _prep(input) is input):
            input, pre = bnops.materialize(input), None
        x = input.permute(0, 3, 1, 2) if self.format == "NHWC" else input
        sq = x.dim() == 3
        if sq:
            x = x.unsqueeze(0)
        ph, pw = self._pads(x.shape[2], x.shape[3])
        if _gpu_ok(x):
            # a deferred BN + ReLU input (nn.fusion: the ResNet stem) is applied inside the pooling kernel
            y, self._idx = P.maxpool_fwd_gpu(_prep(x), self.kH, self.kW, self.dH, self.dW, ph, pw, self.ceilMode,
                                             pre=pre)
        elif x.is_cuda:       # any channel count / dtype / layout: N-d window kernel over N*C planes
            geo, osh = PN.pool2d_geo(x.shape, self.kH, self.kW, self.dH, self.dW, ph, pw, self.ceilMode)
            y, self._idx = PN.pool_nd_fwd(x.contiguous(), osh, geo, True)
        else:
            y, self._idx = F.max_pool2d(x, (self.kH, self.kW), (self.dH, self.dW), (ph, pw),
                                        ceil_mode=self.ceilMode, return_indices=True)
        y = y.squeeze(0) if sq else y
        return y.permute(0, 2, 3, 1) if self.format == "NHWC" else y

    def updateGradInput(self, input, gradOutput):
        x = input.permute(0, 3, 1, 2) if self.format == "NHWC" else input
        g = gradOutput.permute(0, 3, 1, 2) if self.format == "NHWC" else gradOutput
        sq = x.dim() == 3
        if sq:
            x, g = x.unsqueeze(0), g.unsqueeze(0)
        ph, pw = self._pads(x.shape[2], x.shape[3])
        bn_src = getattr(input, "_bn_bwd", None) if _POOL_BN_RED else None
        if _gpu_ok(x) and bn_src is not None and bn_src[0].train and not sq:
            # the input is a training BN's ReLU output (the ResNet stem): reduce that BN's backward statistics here
            gi, red = P.maxpool_bwd_bnred_gpu(_prep(g), self._idx, x.shape, self.kH, self.kW, self.dH, self.dW, ph, pw,
                                              bn_src)
            if red is not None:
                gi._bn_red = (bn_src[0], red)
        elif _gpu_ok(x):
            gi = P.maxpool_bwd_gpu(_prep(g), self._idx, x.shape, self.kH, self.kW, self.dH, self.dW, ph, pw)
        elif x.is_cuda:
            geo, _ = PN.pool2d_geo(x.shape, self.kH, self.kW, self.dH, self.dW, ph, pw, self.ceilMode)
            gi = PN.pool_nd_bwd(g, self._idx, x.shape, geo, True, dtype=x.dtype)
        else:
            # overlapping windows must SUM their gradients (max_unpool2d would overwrite): use autograd
            xr = x.detach().float().requires_grad_(True)
            with torch.enable_grad():
                y = F.max_pool2d(xr, (self.kH, self.kW), (self.dH, self.dW), (ph, pw), ceil_mode=self.ceilMode)
            gi = torch.autograd.grad(y, xr, g.float())[0].to(x.dtype)
        gi = gi.squeeze(0) if sq else gi
        return gi.permute(0, 2, 3, 1) if self.format == "NHWC" else gi

    def __repr__(self):
        return f"SpatialMaxPooling({self.kW}, {self.kH}, {self.dW}, {self.dH}, {self.padW}, {self.padH})"


class SpatialAveragePooling(TensorModule):
    def __init__(self, kW, kH, dW=1, dH=1, padW=0, padH=0, globalPooling=False, ceilMode=False,
                 countIncludePad=True, divide=True, format="NCHW"):
        super().__init__()
        self.kW, self.kH, self.dW, self.dH, self.padW, self.padH = kW, kH, dW, dH, padW, padH
        self.globalPooling, self.ceilMode, self.countIncludePad, self.divide = (globalPooling, ceilMode,
                                                                                countIncludePad, divide)
        self.format = format

    def ceil(self):
        self.ceilMode = True
        return self

    def floor(self):
        self.ceilMode = False
        return self

    def _geom(self, x):
        if self.globalPooling:
            return x.shape[2], x.shape[3], 1, 1, 0, 0
        if self.padW == -1 and self.padH == -1:
            return (self.kH, self.kW, self.dH, self.dW, _same(x.shape[2], self.kH, self.dH),
                    _same(x.shape[3], self.kW, self.dW))
        return self.kH, self.kW, self.dH, self.dW, self.padH, self.padW

    def updateOutput(self, input):
        x = input.permute(0, 3, 1, 2) if self.format == "NHWC" else input
        sq = x.dim() == 3
        if sq:
            x = x.unsqueeze(0)
        kh, kw, sh, sw, ph, pw = self._geom(x)
        if _gpu_ok(x) and self.divide:
            y = P.avgpool_fwd_gpu(_prep(x), kh, kw, sh, sw, ph, pw, self.ceilMode, self.countIncludePad)
        elif x.is_cuda:
            geo, osh = PN.pool2d_geo(x.shape, kh, kw, sh, sw, ph, pw, self.ceilMode)
            y, _ = PN.pool_nd_fwd(x.contiguous(), osh, geo, False, self.countIncludePad)
            if not self.divide:
                y = y * (kh * kw)
        else:
            y = F.avg_pool2d(x, (kh, kw), (sh, sw), (ph, pw), self.ceilMode, self.countIncludePad)
            if not self.divide:
                y = y * (kh * kw)
        y = y.squeeze(0) if sq else y
        return y.permute(0, 2, 3, 1) if self.format == "NHWC" else y

    def updateGradInput(self, input, gradOutput):
        x = input.permute(0, 3, 1, 2) if self.format == "NHWC" else input
        g = gradOutput.permute(0, 3, 1, 2) if self.format == "NHWC" else gradOutput
        sq = x.dim() == 3
        if sq:
            x, g = x.unsqueeze(0), g.unsqueeze(0)
        kh, kw, sh, sw, ph, pw = self._geom(x)
        if _gpu_ok(x) and self.divide:
            gi = P.avgpool_bwd_gpu(_prep(g), x.shape, kh, kw, sh, sw, ph, pw, self.countIncludePad)
        elif x.is_cuda:
            geo, _ = PN.pool2d_geo(x.shape, kh, kw, sh, sw, ph, pw, self.ceilMode)
            gi = PN.pool_nd_bwd(g * (kh * kw) if not self.divide else g, None, x.shape, geo, False,
                                self.countIncludePad, dtype=x.dtype)
        else:
            xr = x.detach().float().requires_grad_(True)
            with torch.enable_grad():
                y = F.avg_pool2d(xr, (kh, kw), (sh, sw), (ph, pw), self.ceilMode, self.countIncludePad)
                if not self.divide:
                    y = y * (kh * kw)
            gi = torch.autograd.grad(y, xr, g.float())[0].to(x.dtype)
        gi = gi.squeeze(0) if sq else gi
        return gi.permute(0, 2, 3, 1) if self.format == "NHWC" else gi


class VolumetricMaxPooling(AutogradModule):
    def __init__(self, kT, kW, kH, dT=None, dW=None, dH=None, padT=0, padW=0, padH=0):
        super().__init__()
        self.k = (kT, kH, kW)
        self.s = (dT or kT, dH or kH, dW or kW)
        self.p = (padT, padH, padW)
        self.ceilMode = False

    def ceil(self):
        self.ceilMode = True
        return self

    def fn(self, x):
        return PN.pool3d(x, self.k, self.s, self.p, self.ceilMode, max_mode=True)


class VolumetricAveragePooling(AutogradModule):
    def __init__(self, kT, kW, kH, dT=None, dW=None, dH=None, padT=0, padW=0, padH=0, countIncludePad=True,
                 ceilMode=False):
        super().__init__()
        self.k = (kT, kH, kW)
        self.s = (dT or kT, dH or kH, dW or kW)
        self.p = (padT, padH, padW)
        self.countIncludePad, self.ceilMode = countIncludePad, ceilMode

    def fn(self, x):
        return PN.pool3d(x, self.k, self.s, self.p, self.ceilMode, max_mode=False, count_pad=self.countIncludePad)


class TemporalMaxPooling(AutogradModule):
    """Max over time of (batch, frames, features) input (reference TemporalMaxPooling.scala)."""

    def __init__(self, kW, dW=None):
        super().__init__()
        self.kW, self.dW = kW, dW if dW is not None else kW

    def fn(self, x):
        return PN.temporal_max_pool(x, self.kW, self.dW)


__all__ = ["SpatialMaxPooling", "SpatialAveragePooling", "VolumetricMaxPooling", "VolumetricAveragePooling",
           "TemporalMaxPooling"]
