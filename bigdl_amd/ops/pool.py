"""Pooling ops. GPU: csrc/elementwise.hip (NHWC bf16, 8 channels per lane, gather-form backward).

Reference: NNPrimitive.maxPoolingForwardFloat / BackwardFloat (S/nn/NNPrimitive.scala:654-936),
S/nn/SpatialMaxPooling.scala:62, S/nn/SpatialAveragePooling.scala:62.
"""
import torch

from . import native
from .conv import out_size

CL = torch.channels_last


def pool_out(H, W, kh, kw, sh, sw, ph, pw, ceil):
    return out_size(H, kh, sh, ph, 1, ceil), out_size(W, kw, sw, pw, 1, ceil)


def maxpool_fwd_gpu(x, kh, kw, sh, sw, ph, pw, ceil=False, pre=None):
    """``pre`` ([2C] scale | shift): x is a deferred BatchNorm + ReLU output (ops/bn.py deferred), applied on load by
    the fixed 3x3/2 kernel (materialised first by the binding otherwise)."""
    N, C, H, W = x.shape
    OH, OW = pool_out(H, W, kh, kw, sh, sw, ph, pw, ceil)
    y = torch.empty((N, C, OH, OW), dtype=x.dtype, device=x.device, memory_format=CL)
    idx = torch.empty((N, C, OH, OW), dtype=torch.uint8, device=x.device, memory_format=CL)
    native.get().maxpool_fwd(x, y, idx, [N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw], pre)
    return y, idx


def maxpool_bwd_gpu(dy, idx, x_shape, kh, kw, sh, sw, ph, pw):
    N, C, H, W = x_shape
    OH, OW = dy.shape[2], dy.shape[3]
    dy = dy.contiguous(memory_format=CL)
    dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=CL)
    native.get().maxpool_bwd(dy, idx, dx, [N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw])
    return dx


def maxpool_bwd_bnred_gpu(dy, idx, x_shape, kh, kw, sh, sw, ph, pw, bn_src):
    """maxpool_bwd_gpu that also accumulates the backward reduction of the training BN whose ReLU output is the pool's
    input (``bn_src`` = that output's ``_bn_bwd``: module, BN input, mean, [scale | shift], sign mask or flag).
    Returns (dx, red) with red the BN's slotted statistics, or (dx, None) when the fused kernel does not apply."""
    from . import bn as bnops

    bnmod, bx, mean, aff, zm = bn_src
    zm = zm if torch.is_tensor(zm) else None
    N, C, H, W = x_shape
    OH, OW = dy.shape[2], dy.shape[3]
    if (zm is None) == (aff is None) or tuple(bx.shape) != (N, C, H, W) or bx.dtype != torch.bfloat16 \
            or not bx.is_contiguous(memory_format=CL):
        return maxpool_bwd_gpu(dy, idx, x_shape, kh, kw, sh, sw, ph, pw), None
    dy = dy.contiguous(memory_format=CL)
    dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=CL)
    red = bnops.new_stats(C, dy.device)
    if not native.get().maxpool_bwd_bnred(dy, idx, dx, [N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw], bx, mean, aff,
                                          zm, red):
        native.get().maxpool_bwd(dy, idx, dx, [N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw])
        return dx, None
    return dx, red


def avgpool_fwd_gpu(x, kh, kw, sh, sw, ph, pw, ceil=False, count_pad=True):
    N, C, H, W = x.shape
    OH, OW = pool_out(H, W, kh, kw, sh, sw, ph, pw, ceil)
    y = torch.empty((N, C, OH, OW), dtype=x.dtype, device=x.device, memory_format=CL)
    native.get().avgpool_fwd(x, y, [N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw], bool(count_pad))
    return y


def avgpool_bwd_gpu(dy, x_shape, kh, kw, sh, sw, ph, pw, count_pad=True):
    N, C, H, W = x_shape
    OH, OW = dy.shape[2], dy.shape[3]
    dy = dy.contiguous(memory_format=CL)
    dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=CL)
    native.get().avgpool_bwd(dy, dx, [N, H, W, C, OH, OW, kh, kw, sh, sw, ph, pw], bool(count_pad))
    return dx
