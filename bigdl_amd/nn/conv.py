"""Convolution layers.

Reference: S/nn/SpatialConvolution.scala (983 LoC; updateOutput :253-362, updateGradInput :364-426,
accGradParameters :435-520), SpatialShareConvolution.scala, SpatialDilatedConvolution.scala:58,
SpatialFullConvolution.scala:71, SpatialSeparableConvolution.scala:54, VolumetricConvolution.scala:51,
VolumetricFullConvolution.scala, TemporalConvolution.scala:49, LocallyConnected1D/2D.scala,
SpatialConvolutionMap.scala.

GPU engine: SpatialConvolution / SpatialShareConvolution / SpatialDilatedConvolution run on the
implicit-GEMM MFMA kernels (csrc/conv_igemm.hip): forward with fused bias (+ BatchNorm statistics when a
BN follows — see nn/fusion.py), data gradient through the same kernel family, weight gradient
accumulated in fp32 straight into the flat gradient buffer. Constructor argument order follows the
reference (kernelW before kernelH, strides / pads W before H).
"""
import math

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import bn as bnops
from ..ops import conv as cv
from ..ops import conv_fn
from ..ops import side_stream
from .abstractnn import AutogradModule, TensorModule, _t_begin, _t_end
from .init_methods import RandomUniform, Zeros

CL = torch.channels_last
BF16 = torch.bfloat16


def _same_pad(inp, k, s, d=1):
    out = -(-inp // s)
    total = max((out - 1) * s + (k - 1) * d + 1 - inp, 0)
    return total // 2, total - total // 2


class SpatialConvolution(TensorModule):
    def __init__(self, nInputPlane, nOutputPlane, kernelW, kernelH, strideW=1, strideH=1, padW=0, padH=0,
                 nGroup=1, propagateBack=True, wRegularizer=None, bRegularizer=None, initWeight=None,
                 initBias=None, initGradWeight=None, initGradBias=None, withBias=True, format="NCHW",
                 dilationW=1, dilationH=1):
        super().__init__()
        assert nInputPlane % nGroup == 0 and nOutputPlane % nGroup == 0
        self.nInputPlane, self.nOutputPlane = nInputPlane, nOutputPlane
        self.kernelW, self.kernelH = kernelW, kernelH
        self.strideW, self.strideH = strideW, strideH
        self.padW, self.padH = padW, padH
        self.dilationW, self.dilationH = dilationW, dilationH
        self.nGroup = nGroup
        self.propagateBack = propagateBack
        self.withBias = withBias
        self.format = format
        self.wRegularizer, self.bRegularizer = wRegularizer, bRegularizer
        self.emit_stats = False      # set by nn.fusion when a BatchNorm consumes this conv's output
        self.fuse_relu = False
        self._fuse_out = self._fuse_addend = None
        self.register_parameter("weight", "gradWeight",
                                torch.empty(nOutputPlane, nInputPlane // nGroup, kernelH, kernelW))
        if withBias:
            self.register_parameter("bias", "gradBias", torch.empty(nOutputPlane))
        else:
            self.bias = None
            self.gradBias = None
        self.weightInitMethod = RandomUniform()
        self.biasInitMethod = RandomUniform()
        self.reset()
        if initWeight is not None:
            self.weight.copy_(torch.as_tensor(initWeight).reshape(self.weight.shape))
        if initBias is not None and withBias:
            self.bias.copy_(torch.as_tensor(initBias).reshape(self.bias.shape))
        if initGradWeight is not None:
            self.gradWeight.copy_(torch.as_tensor(initGradWeight).reshape(self.weight.shape))
        if initGradBias is not None and withBias:
            self.gradBias.copy_(torch.as_tensor(initGradBias).reshape(self.bias.shape))

    def reset(self):
        fan_in = self.nInputPlane // self.nGroup * self.kernelH * self.kernelW
        stdv = 1.0 / math.sqrt(fan_in)
        with torch.no_grad():
            if isinstance(self.weightInitMethod, RandomUniform) and self.weightInitMethod.lower is None:
                RandomUniform(-stdv, stdv).init(self.weight)
            else:
                self.weightInitMethod.init(self.weight)
            if self.bias is not None:
                if isinstance(self.biasInitMethod, RandomUniform) and self.biasInitMethod.lower is None:
                    RandomUniform(-stdv, stdv).init(self.bias)
                else:
                    self.biasInitMethod.init(self.bias)
        self._w16 = {} if not self._w16_managed else self._w16

    def _place(self, attr, t):
        if t.dim() == 4 and t.is_cuda:
            return t.contiguous(memory_format=CL)
        return t.contiguous()

    # ---------------------------------------------------------------- geometry
    def _pads(self, H, W):
        if self.padW == -1 and self.padH == -1:
            ph = _same_pad(H, self.kernelH, self.strideH, self.dilationH)[0]
            pw = _same_pad(W, self.kernelW, self.strideW, self.dilationW)[0]
            return ph, pw
        return self.padH, self.padW

    def _same_extra(self, H, W):
        """Extra bottom/right zero rows when TF-style SAME padding is asymmetric (pad total odd)."""
        if not (self.padW == -1 and self.padH == -1):
            return 0, 0
        bh, ah = _same_pad(H, self.kernelH, self.strideH, self.dilationH)
        bw, aw = _same_pad(W, self.kernelW, self.strideW, self.dilationW)
        return ah - bh, aw - bw

    def _prep(self, x):
        """(input padded for asymmetric SAME, symmetric pads, extra rows, extra cols)."""
        H, W = x.shape[2], x.shape[3]
        ph, pw = self._pads(H, W)
        eh, ew = self._same_extra(H, W)
        if eh or ew:
            x = F.pad(x, (0, ew, 0, eh))
            if x.is_cuda:
                x = x.contiguous(memory_format=CL)
        return x, ph, pw, eh, ew

    def _nchw(self, x):
        if self.format == "NHWC":
            return x.permute(0, 3, 1, 2)
        return x

    def _fmt_out(self, y):
        if self.format == "NHWC":
            return y.permute(0, 2, 3, 1)
        return y

    # ---------------------------------------------------------------- forward
    def _pre_ok(self, x):
        """A deferred BN + ReLU input (ops/bn.py deferred) goes to the GEMM as is (applied on load or materialised by
        the binding) on the plain NCHW path: no SAME padding copy, no pair-view stem, no grouped / fused-graph output."""
        if not (x.is_cuda and x.dim() == 4 and self.format == "NCHW" and self.nGroup == 1
                and x.shape[1] == self.nInputPlane and x.shape[1] % 8 == 0 and x.dtype == BF16
                and x.is_contiguous(memory_format=CL)):
            return False
        if self._same_extra(x.shape[2], x.shape[3]) != (0, 0) or self._pair_path(x):
            return False
        return getattr(self, "_fuse_out", None) is None and getattr(self, "_fuse_addend", None) is None

    def updateOutput(self, input):
        if getattr(input, "_bn_pre", None) is not None and not self._pre_ok(input):
            input = bnops.materialize(input)
        x = self._nchw(input)
        squeeze = x.dim() == 3
        if squeeze:
            x = x.unsqueeze(0)
        x, ph, pw, _, _ = self._prep(x)
        if x.is_cuda and self.nGroup == 1:
            y = self._fwd_gpu(x, ph, pw)
        elif x.is_cuda:
            y = self._fwd_gpu_grouped(x, ph, pw)
        else:
            y = F.conv2d(x.float(), self.weight, self.bias, (self.strideH, self.strideW), (ph, pw),
                         (self.dilationH, self.dilationW), self.nGroup)
            if self.fuse_relu:
                y = torch.relu(y)
        if squeeze:
            y = y.squeeze(0)
        return self._fmt_out(y)

    def _w16_padded(self):
        w16 = self.w16("weight")
        if w16.shape[1] % 8 != 0:
            w16 = cv.weight_krsc_bf16(w16.float())
        return w16

    def _pair_path(self, x):
        return (cv.pair_ok(x.shape[1], (self.strideH, self.strideW), (self.dilationH, self.dilationW), self.nGroup)
                and self.nInputPlane == x.shape[1] and getattr(self, "_fuse_out", None) is None
                and getattr(self, "_fuse_addend", None) is None)

    def _fwd_gpu_pairs(self, x, ph, pw):
        """<= 4 input channels, width stride 2 (image stems): pixel-pair packed implicit GEMM (ops/conv.py,
        csrc/stem.hip) — 2 width taps per 16-byte granule instead of 1 pixel padded to 8 channels."""
        R, S, sh = self.kernelH, self.kernelW, self.strideH
        OH, OW, S2, _, _ = cv.pair_geometry(x.shape[2], x.shape[3], R, S, sh, ph, pw)
        xp = cv.to_pairs_bf16(x, R, S, sh, ph, pw)
        self._xpair = (xp, tuple(x.shape), ph, pw)
        self._x16 = None
        wp = cv.pair_weight(self.w16("weight"))
        stats = None
        if self.emit_stats and self.train and self.nOutputPlane % 8 == 0:
            stats = bnops.new_stats(self.nOutputPlane, x.device)
        y = cv.conv2d_pairs_fwd(xp, wp, self.bias, self.nOutputPlane, OH, OW, R, S2, sh, relu=self.fuse_relu,
                                stats=stats)
        if stats is not None:
            y._bn_stats = stats
        self._geom = (x.shape, ph, pw)
        return y

    def _wgrad_gpu_pairs(self, x, gy16):
        xp, shape, ph, pw = self._xpair
        R, S, K = self.kernelH, self.kernelW, self.nOutputPlane
        S2 = (S + 1) // 2
        dwp = ops.zeros(K, R * S2 * 8, device=x.device)
        db = None
        if self.bias is not None:
            db = self.gradBias if self.scaleB == 1.0 else ops.zeros(K, device=x.device)
        cv.conv2d_pairs_wgrad(gy16, xp, R, S2, self.strideH, dwp, db)
        ops.native.get().pair_wgrad_add(dwp, self.gradWeight, float(self.scaleW))
        if db is not None and db is not self.gradBias:
            self.gradBias.add_(db, alpha=self.scaleB)

    def _fwd_gpu(self, x, ph, pw):
        self._xpair = None
        self._x16_pre = None
        pre = getattr(x, "_bn_pre", None)
        if self._pair_path(x) and self.nOutputPlane % 8 == 0 and pre is None:
            return self._fwd_gpu_pairs(x, ph, pw)
        x16 = cv.to_nhwc_bf16(x)
        self._x16 = x16
        w16 = self._w16_padded()
        stats = None
        if self.emit_stats and self.train and self.nOutputPlane % 8 == 0:
            stats = bnops.new_stats(self.nOutputPlane, x.device)
        # inference graph fusion (nn.fusion.fuse_graph_for_inference): output straight into a concat slice
        # and / or a residual addend summed in the epilogue; set by the graph right before this call
        out, addend = getattr(self, "_fuse_out", None), getattr(self, "_fuse_addend", None)
        self._fuse_out = self._fuse_addend = None
        y = cv.conv2d_fwd(x16, w16, self.bias, (self.strideH, self.strideW), (ph, pw),
                          (self.dilationH, self.dilationW), relu=self.fuse_relu, stats=stats, out=out,
                          addend=addend, pre=pre)
        if pre is not None:
            # applied on load: the weight gradient re-applies it (on its own stream); else the binding materialised it
            y, mat = y
            if mat is None:
                self._x16_pre = pre
            else:
                self._x16 = mat
        if stats is not None:
            y._bn_stats = stats
        self._geom = (x.shape, ph, pw)
        return y

    def _direct_groups(self):
        """Groups with <= 16 input channels (depthwise, ResNeXt-style) run the direct grouped kernels
        (csrc/grouped_conv.hip): one launch per pass for all groups."""
        return self.nGroup > 1 and self.nInputPlane // self.nGroup <= 16

    def _geo_g(self, ph, pw):
        return [self.strideH, self.strideW, ph, pw, self.dilationH, self.dilationW, self.nGroup]

    def _fwd_gpu_grouped(self, x, ph, pw):
        G = self.nGroup
        cin, cout = self.nInputPlane // G, self.nOutputPlane // G
        if self._direct_groups():
            xf = x.float().contiguous()
            OH = cv.out_size(x.shape[2], self.kernelH, self.strideH, ph, self.dilationH)
            OW = cv.out_size(x.shape[3], self.kernelW, self.strideW, pw, self.dilationW)
            y = xf.new_empty(x.shape[0], self.nOutputPlane, OH, OW)
            ops.native.get().gconv(0, xf, self.weight.float().contiguous(),
                                   self.bias.float().contiguous() if self.bias is not None else None, y,
                                   self._geo_g(ph, pw))
            if self.fuse_relu:
                y.relu_()
            self._xf = xf
            self._geom = (x.shape, ph, pw)
            return y.to(BF16).contiguous(memory_format=CL)
        outs = []
        w = self.weight
        self._x16 = cv.to_nhwc_bf16(x) if x.shape[1] % 8 == 0 else None
        for g in range(G):
            xg = cv.to_nhwc_bf16(x[:, g * cin:(g + 1) * cin].contiguous(memory_format=CL))
            wg = cv.weight_krsc_bf16(w[g * cout:(g + 1) * cout])
            bg = self.bias[g * cout:(g + 1) * cout] if self.bias is not None else None
            outs.append(cv.conv2d_fwd(xg, wg, bg, (self.strideH, self.strideW), (ph, pw),
                                      (self.dilationH, self.dilationW), relu=self.fuse_relu))
        self._geom = (x.shape, ph, pw)
        return torch.cat(outs, dim=1).contiguous(memory_format=CL)

    # ---------------------------------------------------------------- backward
    def updateGradInput(self, input, gradOutput):
        if not self.propagateBack:
            return None
        x = self._nchw(input)
        gy = self._nchw(gradOutput)
        squeeze = x.dim() == 3
        if squeeze:
            x, gy = x.unsqueeze(0), gy.unsqueeze(0)
        H, W = x.shape[2], x.shape[3]
        x, ph, pw, eh, ew = self._prep(x)
        if gy.is_cuda:
            gy = self._relu_mask(gy)
            once = getattr(self, "_dgrad_bn_once", False)
            self._dgrad_bn_once = False
            bn_src = getattr(input, "_bn_bwd", None) if (getattr(self, "_dgrad_bn_ok", False) or once) else None
            if bn_src is not None and not torch.is_tensor(bn_src[4]):
                # flag -> the BN's post-ReLU output, which is this conv's input (a tensor there is its sign mask)
                bn_src = bn_src[:4] + ((input if bn_src[4] else None),)
            gi = self._dgrad_gpu(x, gy, ph, pw, None if (squeeze or eh or ew or self.format != "NCHW") else bn_src)
        else:
            gy = self._relu_mask(gy)
            gi = torch.nn.grad.conv2d_input(x.shape, self.weight, gy.float(), (self.strideH, self.strideW),
                                            (ph, pw), (self.dilationH, self.dilationW), self.nGroup)
        if eh or ew:
            gi = gi[:, :, :H, :W]
            if gi.is_cuda:
                gi = gi.contiguous(memory_format=CL)
        if squeeze:
            gi = gi.squeeze(0)
        return self._fmt_out(gi)

    def _relu_mask(self, gy):
        if not self.fuse_relu:
            return gy
        if gy.is_cuda and gy.dtype == BF16:
            return ops.relu_bwd_gpu(gy.contiguous(memory_format=CL), self.output)
        return gy * (self.output > 0)

    def _dgrad_gpu(self, x, gy, ph, pw, bn_src=None):
        gy16 = gy if (gy.dtype == BF16 and gy.is_contiguous(memory_format=CL)) else gy.to(BF16, memory_format=CL)
        if self.nGroup == 1:
            w16 = self._w16_padded()
            if gy16.shape[1] % 8:   # output channels not a multiple of 8: zero-pad K for the GEMM
                gy16 = cv.pad_dim(gy16, 1)
                w16 = cv.pad_dim(w16, 0)
            wt = getattr(self, "_wt_cache", None)
            if getattr(self, "_wt_stamp", None) != cv.WT_STAMP[0] or wt is None or \
                    tuple(wt.shape) != (w16.shape[1], w16.shape[2], w16.shape[3], w16.shape[0]):
                wt = cv.transpose_w(w16)        # not batched by TrainStep this step (or padded K)
            Cp = w16.shape[1]
            xs = (x.shape[0], Cp, x.shape[2], x.shape[3])
            addend = getattr(self, "_dgrad_addend", None)
            self._dgrad_addend = None
            addend_zm = None
            if isinstance(addend, tuple):       # (gradient, sign mask): add gradient where the mask bit is set
                addend, addend_zm = addend
            if addend is not None and Cp != x.shape[1]:
                raise RuntimeError("dgrad addend requires unpadded channels")
            bn = None
            if bn_src is not None and Cp == x.shape[1]:
                # the input is a training BN's output: reduce that BN's backward statistics in our epilogue
                bnmod, bx, bmean, baff, bz = bn_src
                bzm = None
                if bz is not None and bz.dtype == torch.uint8:
                    bz, bzm = None, bz
                bn = {"x": bx, "z": bz, "zm": bzm, "mean": bmean, "aff": baff,
                      "red": bnops.new_stats(Cp, gy16.device)}
            gi = cv.conv2d_dgrad(gy16, wt, xs, (self.strideH, self.strideW), (ph, pw),
                                 (self.dilationH, self.dilationW), addend=addend, bn=bn, addend_zm=addend_zm)
            if Cp != x.shape[1]:
                gi = gi[:, : x.shape[1]].contiguous(memory_format=CL)
            elif bn is not None and bn.get("done"):
                gi._bn_red = (bnmod, bn["red"])
            return gi
        G = self.nGroup
        cin, cout = self.nInputPlane // G, self.nOutputPlane // G
        if self._direct_groups():
            gyf = gy.float().contiguous()
            dx = torch.empty(x.shape[0], self.nInputPlane, x.shape[2], x.shape[3], device=gy.device)
            ops.native.get().gconv(1, dx, self.weight.float().contiguous(), None, gyf, self._geo_g(ph, pw))
            return dx.to(BF16).contiguous(memory_format=CL)
        parts = []
        for g in range(G):
            wg = cv.pad_dim(cv.weight_krsc_bf16(self.weight[g * cout:(g + 1) * cout]), 0)
            gyg = cv.pad_dim(gy16[:, g * cout:(g + 1) * cout].contiguous(memory_format=CL), 1)
            xs = (x.shape[0], wg.shape[1], x.shape[2], x.shape[3])
            gi = cv.conv2d_dgrad(gyg, cv.transpose_w(wg), xs, (self.strideH, self.strideW), (ph, pw),
                                 (self.dilationH, self.dilationW))
            parts.append(gi[:, :cin])
        return torch.cat(parts, dim=1).contiguous(memory_format=CL)

    def backward(self, input, gradOutput):
        side = None if self._frozen else side_stream.stream_for(gradOutput)
        if side is None:
            return super().backward(input, gradOutput)
        t0 = _t_begin(gradOutput)
        self.gradInput = self.updateGradInput(input, gradOutput)
        # weight gradient on the side stream, concurrent with the data-gradient chain (ops/side_stream.py)
        side_stream.begin(side)
        with torch.cuda.stream(side):
            self.accGradParameters(input, gradOutput)
            self._apply_regularizers()
        side_stream.keep(side, input, gradOutput, self.output, getattr(self, "_x16", None),
                         *(getattr(self, "_xpair", None) or (None,))[:1])
        _t_end(self, t0, "backward_time")
        return self.gradInput

    def accGradParameters(self, input, gradOutput):
        x = self._nchw(input)
        gy = self._nchw(gradOutput)
        if x.dim() == 3:
            x, gy = x.unsqueeze(0), gy.unsqueeze(0)
        x, ph, pw, _, _ = self._prep(x)
        if gy.is_cuda:
            gy = self._relu_mask(gy) if self.fuse_relu and not getattr(self, "_masked_cached", False) else gy
            self._wgrad_gpu(x, gy, ph, pw)
            return
        gy = self._relu_mask(gy).float()
        gw = torch.nn.grad.conv2d_weight(x.float(), self.weight.shape, gy, (self.strideH, self.strideW), (ph, pw),
                                         (self.dilationH, self.dilationW), self.nGroup)
        self.gradWeight.add_(gw, alpha=self.scaleW)
        if self.bias is not None:
            self.gradBias.add_(gy.sum(dim=(0, 2, 3)), alpha=self.scaleB)

    def _wgrad_gpu(self, x, gy, ph, pw):
        gy16 = gy if (gy.dtype == BF16 and gy.is_contiguous(memory_format=CL)) else gy.to(BF16, memory_format=CL)
        xpair = getattr(self, "_xpair", None)
        if (xpair is not None and xpair[1] == tuple(x.shape) and xpair[2:] == (ph, pw) and self.nGroup == 1
                and self.gradWeight.dtype == torch.float32):
            self._wgrad_gpu_pairs(x, gy16)
            return
        x16 = getattr(self, "_x16", None)
        pre = None
        if x16 is None or x16.shape[0] != x.shape[0] or x16.shape[2:] != x.shape[2:]:
            x16 = cv.to_nhwc_bf16(bnops.materialize(x))
        elif getattr(self, "_x16_pre", None) is not None:
            # the forward applied a deferred BN + ReLU on load: the weight gradient applies it too (halo 3x3 kernel) or
            # gets it materialised on the weight-gradient stream
            pre = self._x16_pre
        st, pd, dl = (self.strideH, self.strideW), (ph, pw), (self.dilationH, self.dilationW)
        if self.nGroup != 1 and self._direct_groups():
            xf = getattr(self, "_xf", None)
            if xf is None or xf.shape != x.shape:
                xf = x.float().contiguous()
            dw = ops.zeros(self.weight.shape, device=x.device)
            db = ops.zeros(self.nOutputPlane, device=x.device) if self.bias is not None else None
            ops.native.get().gconv(2, xf, dw, db, gy.float().contiguous(), self._geo_g(pd[0], pd[1]))
            self.gradWeight.add_(dw, alpha=self.scaleW)
            if db is not None:
                self.gradBias.add_(db, alpha=self.scaleB)
            return
        if self.nGroup != 1:
            G = self.nGroup
            cin, cout = self.nInputPlane // G, self.nOutputPlane // G
            for g in range(G):
                xg = cv.to_nhwc_bf16(x[:, g * cin:(g + 1) * cin].contiguous(memory_format=CL))
                gyg = cv.pad_dim(gy16[:, g * cout:(g + 1) * cout].contiguous(memory_format=CL), 1)
                dw = ops.zeros(gyg.shape[1], xg.shape[1], self.kernelH, self.kernelW, device=x.device,
                               memory_format=CL)
                db = ops.zeros(gyg.shape[1], device=x.device) if self.bias is not None else None
                cv.conv2d_wgrad(gyg, xg, dw, db, st, pd, dl)
                self.gradWeight[g * cout:(g + 1) * cout].add_(dw[:cout, :cin], alpha=self.scaleW)
                if db is not None:
                    self.gradBias[g * cout:(g + 1) * cout].add_(db[:cout], alpha=self.scaleB)
            return
        K = self.nOutputPlane
        direct = (x16.shape[1] == self.nInputPlane and K % 8 == 0 and self.scaleW == 1.0 and self.scaleB == 1.0
                  and self.gradWeight.is_contiguous(memory_format=CL))
        if pre is not None and not direct:
            x16 = bnops.materialize(bnops.deferred(x16, pre))
        if direct:
            cv.conv2d_wgrad(gy16, x16, self.gradWeight, self.gradBias, st, pd, dl, pre=pre)
        else:
            gyp = cv.pad_dim(gy16, 1)
            dw = ops.zeros(gyp.shape[1], x16.shape[1], self.kernelH, self.kernelW, device=x.device,
                           memory_format=CL)
            db = ops.zeros(gyp.shape[1], device=x.device) if self.bias is not None else None
            cv.conv2d_wgrad(gyp, x16, dw, db, st, pd, dl)
            self.gradWeight.add_(dw[:K, : self.nInputPlane], alpha=self.scaleW)
            if db is not None:
                self.gradBias.add_(db[:K], alpha=self.scaleB)

    def clearState(self):
        super().clearState()
        self._x16 = None
        self._x16_pre = None
        self._xpair = None
        return self

    def __repr__(self):
        return (f"SpatialConvolution({self.nInputPlane} -> {self.nOutputPlane}, {self.kernelW} x {self.kernelH}, "
                f"{self.strideW}, {self.strideH}, {self.padW}, {self.padH})")


class SpatialShareConvolution(SpatialConvolution):
    """Reference shares im2col buffers across layers to save host memory (ResNet ``optnet``). On the GPU
    engine there is no im2col buffer at all (implicit GEMM), so this is SpatialConvolution."""


class SpatialDilatedConvolution(SpatialConvolution):
    def __init__(self, nInputPlane, nOutputPlane, kW, kH, dW=1, dH=1, padW=0, padH=0, dilationW=1, dilationH=1,
                 wRegularizer=None, bRegularizer=None):
        super().__init__(nInputPlane, nOutputPlane, kW, kH, dW, dH, padW, padH, wRegularizer=wRegularizer,
                         bRegularizer=bRegularizer, dilationW=dilationW, dilationH=dilationH)


class SpatialFullConvolution(AutogradModule):
    """Transposed convolution (deconvolution). Weight (nInputPlane, nOutputPlane/nGroup, kH, kW)."""

    def __init__(self, nInputPlane, nOutputPlane, kW, kH, dW=1, dH=1, padW=0, padH=0, adjW=0, adjH=0, nGroup=1,
                 noBias=False, wRegularizer=None, bRegularizer=None):
        super().__init__()
        self.nInputPlane, self.nOutputPlane = nInputPlane, nOutputPlane
        self.kW, self.kH, self.dW, self.dH = kW, kH, dW, dH
        self.padW, self.padH, self.adjW, self.adjH, self.nGroup = padW, padH, adjW, adjH, nGroup
        self.wRegularizer, self.bRegularizer = wRegularizer, bRegularizer
        self.register_parameter("weight", "gradWeight", torch.empty(nInputPlane, nOutputPlane // nGroup, kH, kW))
        if not noBias:
            self.register_parameter("bias", "gradBias", torch.empty(nOutputPlane))
        else:
            self.bias = None
        self.reset()

    def reset(self):
        stdv = 1.0 / math.sqrt(self.kW * self.kH * self.nInputPlane)
        RandomUniform(-stdv, stdv).init(self.weight)
        if self.bias is not None:
            RandomUniform(-stdv, stdv).init(self.bias)

    def fn(self, x):
        if isinstance(x, torch.Tensor):
            adj = (self.adjH, self.adjW)
        else:  # Table(input, sizeTensor)
            x = x[1]
            adj = (self.adjH, self.adjW)
        if x.is_cuda and self.nGroup == 1:     # the native data-gradient kernel (ops/conv_fn.py)
            return conv_fn.conv_transpose2d(x.float(), self.weight, self.bias, (self.dH, self.dW),
                                            (self.padH, self.padW), adj)
        return F.conv_transpose2d(x.to(self.weight.dtype), self.weight, self.bias, (self.dH, self.dW),
                                  (self.padH, self.padW), adj, self.nGroup)


class SpatialSeparableConvolution(AutogradModule):
    def __init__(self, nInputChannel, nOutputChannel, depthMultiplier, kW, kH, sW=1, sH=1, pW=0, pH=0,
                 hasBias=True, dataFormat="NCHW", wRegularizer=None, bRegularizer=None, pRegularizer=None):
        super().__init__()
        self.cin, self.cout, self.dm = nInputChannel, nOutputChannel, depthMultiplier
        self.k, self.s, self.p = (kH, kW), (sH, sW), (pH, pW)
        self.dataFormat = dataFormat
        self.register_parameter("depthWeight", "depthGradWeight", torch.empty(nInputChannel * depthMultiplier, 1, kH, kW))
        self.register_parameter("pointWeight", "pointGradWeight",
                                torch.empty(nOutputChannel, nInputChannel * depthMultiplier, 1, 1))
        if hasBias:
            self.register_parameter("bias", "gradBias", torch.zeros(nOutputChannel))
        else:
            self.bias = None
        self.reset()

    def reset(self):
        RandomUniform().init(self.depthWeight)
        RandomUniform().init(self.pointWeight)

    def fn(self, x):
        if self.dataFormat == "NHWC":
            x = x.permute(0, 3, 1, 2)
        # depthwise half on the direct grouped kernel, pointwise half on the MFMA GEMM
        y = conv_fn.group_conv2d(x.to(self.depthWeight.dtype), self.depthWeight, None, self.s, self.p,
                                 groups=self.cin)
        y = conv_fn.conv2d(y, self.pointWeight, self.bias)        # pointwise half on the MFMA GEMM
        return y.permute(0, 2, 3, 1) if self.dataFormat == "NHWC" else y


class SpatialConvolutionMap(AutogradModule):
    """Convolution with an explicit connection table (rows: (inputPlane, outputPlane), 1-based)."""

    def __init__(self, connTable, kW, kH, dW=1, dH=1, padW=0, padH=0):
        super().__init__()
        ct = torch.as_tensor(connTable, dtype=torch.long)
        self.connTable = ct
        self.nInputPlane = int(ct[:, 0].max())
        self.nOutputPlane = int(ct[:, 1].max())
        self.kW, self.kH, self.dW, self.dH, self.padW, self.padH = kW, kH, dW, dH, padW, padH
        self.register_parameter("weight", "gradWeight", torch.empty(ct.shape[0], kH, kW))
        self.register_parameter("bias", "gradBias", torch.empty(self.nOutputPlane))
        mask = torch.zeros(self.nOutputPlane, self.nInputPlane, 1, 1)
        for i, o in ct.tolist():
            mask[o - 1, i - 1] = 1
        self._mask = mask
        self.reset()

    @staticmethod
    def full(nin, nout):
        return [[i, o] for o in range(1, nout + 1) for i in range(1, nin + 1)]

    @staticmethod
    def oneToOne(n):
        return [[i, i] for i in range(1, n + 1)]

    def reset(self):
        stdv = 1.0 / math.sqrt(self.kW * self.kH * self.nInputPlane)
        RandomUniform(-stdv, stdv).init(self.weight)
        RandomUniform(-stdv, stdv).init(self.bias)

    def fn(self, x):
        W = torch.zeros(self.nOutputPlane, self.nInputPlane, self.kH, self.kW, dtype=self.weight.dtype,
                        device=self.weight.device)
        idx_o = self.connTable[:, 1].to(self.weight.device) - 1
        idx_i = self.connTable[:, 0].to(self.weight.device) - 1
        W = W.index_put((idx_o, idx_i), self.weight)
        return conv_fn.conv2d(x.to(W.dtype), W, self.bias, (self.dH, self.dW), (self.padH, self.padW))


class VolumetricConvolution(AutogradModule):
    def __init__(self, nInputPlane, nOutputPlane, kT, kW, kH, dT=1, dW=1, dH=1, padT=0, padW=0, padH=0,
                 withBias=True, wRegularizer=None, bRegularizer=None):
        super().__init__()
        self.k, self.s, self.p = (kT, kH, kW), (dT, dH, dW), (padT, padH, padW)
        self.nInputPlane, self.nOutputPlane = nInputPlane, nOutputPlane
        self.wRegularizer, self.bRegularizer = wRegularizer, bRegularizer
        self.register_parameter("weight", "gradWeight", torch.empty(nOutputPlane, nInputPlane, kT, kH, kW))
        if withBias:
            self.register_parameter("bias", "gradBias", torch.empty(nOutputPlane))
        else:
            self.bias = None
        self.reset()

    def reset(self):
        stdv = 1.0 / math.sqrt(self.k[0] * self.k[1] * self.k[2] * self.nInputPlane)
        RandomUniform(-stdv, stdv).init(self.weight)
        if self.bias is not None:
            RandomUniform(-stdv, stdv).init(self.bias)

    def fn(self, x):
        if self.p == (-1, -1, -1):
            pads = [_same_pad(x.shape[2 + i], self.k[i], self.s[i]) for i in range(3)]
            x = F.pad(x, (pads[2][0], pads[2][1], pads[1][0], pads[1][1], pads[0][0], pads[0][1]))
            p = 0
        else:
            p = self.p
        if isinstance(p, int):
            p = (p, p, p)
        return conv_fn.conv3d(x.to(self.weight.dtype), self.weight, self.bias, self.s, p)


class VolumetricFullConvolution(AutogradModule):
    def __init__(self, nInputPlane, nOutputPlane, kT, kW, kH, dT=1, dW=1, dH=1, padT=0, padW=0, padH=0, adjT=0,
                 adjW=0, adjH=0, nGroup=1, noBias=False, wRegularizer=None, bRegularizer=None):
        super().__init__()
        self.k, self.s, self.p, self.adj, self.g = (kT, kH, kW), (dT, dH, dW), (padT, padH, padW), (adjT, adjH, adjW), nGroup
        self.register_parameter("weight", "gradWeight", torch.empty(nInputPlane, nOutputPlane // nGroup, kT, kH, kW))
        if not noBias:
            self.register_parameter("bias", "gradBias", torch.empty(nOutputPlane))
        else:
            self.bias = None
        stdv = 1.0 / math.sqrt(kT * kW * kH * nInputPlane)
        RandomUniform(-stdv, stdv).init(self.weight)
        if self.bias is not None:
            RandomUniform(-stdv, stdv).init(self.bias)

    def fn(self, x):
        if x.is_cuda and self.g == 1:           # native 2-D transposed conv per temporal tap (ops/conv_fn.py)
            return conv_fn.conv_transpose3d(x.float(), self.weight, self.bias, self.s, self.p, self.adj)
        return F.conv_transpose3d(x.to(self.weight.dtype), self.weight, self.bias, self.s, self.p, self.adj, self.g)


class TemporalConvolution(AutogradModule):
    """1-D convolution over (batch, frames, inputFrameSize) (reference TemporalConvolution.scala:49)."""

    def __init__(self, inputFrameSize, outputFrameSize, kernelW, strideW=1, propagateBack=True,
                 wRegularizer=None, bRegularizer=None, initWeight=None, initBias=None):
        super().__init__()
        self.inputFrameSize, self.outputFrameSize, self.kernelW, self.strideW = (inputFrameSize, outputFrameSize,
                                                                                  kernelW, strideW)
        self.wRegularizer, self.bRegularizer = wRegularizer, bRegularizer
        self.register_parameter("weight", "gradWeight", torch.empty(outputFrameSize, inputFrameSize * kernelW))
        self.register_parameter("bias", "gradBias", torch.empty(outputFrameSize))
        stdv = 1.0 / math.sqrt(kernelW * inputFrameSize)
        RandomUniform(-stdv, stdv).init(self.weight)
        RandomUniform(-stdv, stdv).init(self.bias)
        if initWeight is not None:
            self.weight.copy_(torch.as_tensor(initWeight).reshape(self.weight.shape))
        if initBias is not None:
            self.bias.copy_(torch.as_tensor(initBias).reshape(self.bias.shape))

    def fn(self, x):
        squeeze = x.dim() == 2
        if squeeze:
            x = x.unsqueeze(0)
        w = self.weight.view(self.outputFrameSize, self.kernelW, self.inputFrameSize).permute(0, 2, 1)
        y = conv_fn.conv1d(x.to(w.dtype).transpose(1, 2), w, self.bias, self.strideW).transpose(1, 2)
        return y.squeeze(0) if squeeze else y


class LocallyConnected2D(AutogradModule):
    def __init__(self, nInputPlane, inputWidth, inputHeight, nOutputPlane, kernelW, kernelH, strideW=1, strideH=1,
                 padW=0, padH=0, propagateBack=True, wRegularizer=None, bRegularizer=None, withBias=True,
                 format="NCHW"):
        super().__init__()
        self.cin, self.cout = nInputPlane, nOutputPlane
        self.k, self.s, self.p = (kernelH, kernelW), (strideH, strideW), (padH, padW)
        self.oh = (inputHeight + 2 * padH - kernelH) // strideH + 1
        self.ow = (inputWidth + 2 * padW - kernelW) // strideW + 1
        self.format = format
        L = self.oh * self.ow
        self.register_parameter("weight", "gradWeight", torch.empty(L, nOutputPlane, nInputPlane * kernelH * kernelW))
        if withBias:
            self.register_parameter("bias", "gradBias", torch.empty(L, nOutputPlane))
        else:
            self.bias = None
        stdv = 1.0 / math.sqrt(kernelW * kernelH * nInputPlane)
        RandomUniform(-stdv, stdv).init(self.weight)
        if self.bias is not None:
            RandomUniform(-stdv, stdv).init(self.bias)

    def fn(self, x):
        if self.format == "NHWC":
            x = x.permute(0, 3, 1, 2)
        if x.is_cuda:
            # one GEMM per output location, batched: cols [L][N][C*kh*kw] x W [L][O][C*kh*kw] on the native MFMA
            # kernel (ops/bmm.py); patches gathered with Tensor.unfold views (no im2col kernel)
            from ..ops.bmm import matmul

            N = x.shape[0]
            ph, pw = self.p
            xp = torch.constant_pad_nd(x.float(), (pw, pw, ph, ph)) if (ph or pw) else x.float()
            pat = xp.unfold(2, self.k[0], self.s[0]).unfold(3, self.k[1], self.s[1])   # N, C, OH, OW, kh, kw
            cols = pat.permute(2, 3, 0, 1, 4, 5).reshape(self.oh * self.ow, N, -1)      # L, N, C*kh*kw
            y = matmul(cols, self.weight.transpose(1, 2))                               # L, N, O
            if self.bias is not None:
                y = y + self.bias.unsqueeze(1)
            y = y.permute(1, 2, 0).reshape(N, self.cout, self.oh, self.ow)
            return y.permute(0, 2, 3, 1) if self.format == "NHWC" else y
        cols = F.unfold(x.to(self.weight.dtype), self.k, padding=self.p, stride=self.s)   # N, CKK, L
        y = torch.einsum("nkl,lok->nol", cols, self.weight)
        if self.bias is not None:
            y = y + self.bias.t().unsqueeze(0)
        y = y.reshape(x.shape[0], self.cout, self.oh, self.ow)
        return y.permute(0, 2, 3, 1) if self.format == "NHWC" else y


class LocallyConnected1D(AutogradModule):
    def __init__(self, nInputFrame, inputFrameSize, outputFrameSize, kernelW, strideW=1, propagateBack=True,
                 wRegularizer=None, bRegularizer=None):
        super().__init__()
        self.nOut = (nInputFrame - kernelW) // strideW + 1
        self.kW, self.sW, self.inS, self.outS = kernelW, strideW, inputFrameSize, outputFrameSize
        self.register_parameter("weight", "gradWeight", torch.empty(self.nOut, outputFrameSize, inputFrameSize * kernelW))
        self.register_parameter("bias", "gradBias", torch.empty(self.nOut, outputFrameSize))
        stdv = 1.0 / math.sqrt(kernelW * inputFrameSize)
        RandomUniform(-stdv, stdv).init(self.weight)
        RandomUniform(-stdv, stdv).init(self.bias)

    def fn(self, x):
        squeeze = x.dim() == 2
        if squeeze:
            x = x.unsqueeze(0)
        win = x.to(self.weight.dtype).unfold(1, self.kW, self.sW)          # N, L, in, kW
        win = win.permute(0, 1, 3, 2).reshape(x.shape[0], self.nOut, -1)
        if x.is_cuda:     # batched over output frames on the native MFMA GEMM (ops/bmm.py)
            from ..ops.bmm import matmul

            y = matmul(win.transpose(0, 1), self.weight.transpose(1, 2)).transpose(0, 1) + self.bias
            return y.squeeze(0) if squeeze else y
        y = torch.einsum("nlk,lok->nlo", win, self.weight) + self.bias
        return y.squeeze(0) if squeeze else y


__all__ = ["SpatialConvolution", "SpatialShareConvolution", "SpatialDilatedConvolution", "SpatialFullConvolution",
           "SpatialSeparableConvolution", "SpatialConvolutionMap", "VolumetricConvolution",
           "VolumetricFullConvolution", "TemporalConvolution", "LocallyConnected1D", "LocallyConnected2D"]
