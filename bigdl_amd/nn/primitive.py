"""Convolution / pooling primitives (reference S/nn/NNPrimitive.scala:108-1771: im2col / col2im (with dilation),
vol2col / col2vol, unfoldedCopy / unfoldedAcc for volumetric conv, max / avg pooling loops, temporal pooling).

The GPU engine never materialises these (its convolutions are implicit GEMMs that generate the im2col addresses
inside the MFMA kernels, csrc/conv_igemm.hip); these are the explicit CPU forms of the same index maps, used by
the CPU engine's reference paths and kept for API parity (e.g. hand-built im2col + GEMM layers).
Layout: im2col of an input [C, H, W] is [C*kH*kW, oH*oW] (row = (c, kh, kw), column = output pixel).
"""
import torch
import torch.nn.functional as F


def out_size(n, k, s, p, d=1):
    return (n + 2 * p - d * (k - 1) - 1) // s + 1


def im2col(x, kW, kH, dW=1, dH=1, padW=0, padH=0, dilationW=1, dilationH=1):
    """[C, H, W] or [N, C, H, W] -> [(N,) C*kH*kW, oH*oW]."""
    batched = x.dim() == 4
    xb = x if batched else x.unsqueeze(0)
    cols = F.unfold(xb, (kH, kW), dilation=(dilationH, dilationW), padding=(padH, padW), stride=(dH, dW))
    return cols if batched else cols[0]


def col2im(cols, C, H, W, kW, kH, dW=1, dH=1, padW=0, padH=0, dilationW=1, dilationH=1):
    """Adjoint of im2col: overlapping patches are summed (col2imFloat :279)."""
    batched = cols.dim() == 3
    cb = cols if batched else cols.unsqueeze(0)
    out = F.fold(cb, (H, W), (kH, kW), dilation=(dilationH, dilationW), padding=(padH, padW), stride=(dH, dW))
    return out if batched else out[0]


def vol2col(x, kT, kW, kH, dT=1, dW=1, dH=1, pT=0, pW=0, pH=0):
    """[C, T, H, W] -> [C*kT*kH*kW, oT*oH*oW] (vol2colFloat :1612)."""
    xp = F.pad(x, (pW, pW, pH, pH, pT, pT))
    u = xp.unfold(1, kT, dT).unfold(2, kH, dH).unfold(3, kW, dW)       # C, oT, oH, oW, kT, kH, kW
    C, oT, oH, oW = u.shape[:4]
    return u.permute(0, 4, 5, 6, 1, 2, 3).reshape(C * kT * kH * kW, oT * oH * oW)


def col2vol(cols, C, T, H, W, kT, kW, kH, dT=1, dW=1, dH=1, pT=0, pW=0, pH=0):
    """Adjoint of vol2col (col2volFloat :1719), computed through autograd of vol2col."""
    x = torch.zeros(C, T, H, W, dtype=cols.dtype, requires_grad=True)
    with torch.enable_grad():
        y = vol2col(x, kT, kW, kH, dT, dW, dH, pT, pW, pH)
        (g,) = torch.autograd.grad(y, x, cols)
    return g


def max_pooling_forward(x, kW, kH, dW, dH, padW=0, padH=0, ceil=False):
    """Returns (output, 1-based flat argmax indices within each input plane) like maxPoolingForwardFloat :654."""
    y, idx = F.max_pool2d(x, (kH, kW), (dH, dW), (padH, padW), ceil_mode=ceil, return_indices=True)
    return y, idx + 1


def max_pooling_backward(gy, idx, input_shape):
    """Scatter gradients to the argmax positions (maxPoolingBackwardFloat :714)."""
    H, W = input_shape[-2:]
    return F.max_unpool2d(gy, idx - 1, gy.shape[-2:], output_size=(H, W)) if gy.dim() == 4 else \
        F.max_unpool2d(gy.unsqueeze(0), (idx - 1).unsqueeze(0), gy.shape[-2:], output_size=(H, W))[0]


def temporal_max_pooling(x, kW, dW):
    """[T, F] (or [N, T, F]) max over time windows (NNPrimitive temporal pooling :996)."""
    xt = x.transpose(-1, -2)
    y, idx = F.max_pool1d(xt, kW, dW, return_indices=True)
    return y.transpose(-1, -2), idx.transpose(-1, -2) + 1


__all__ = ["im2col", "col2im", "vol2col", "col2vol", "max_pooling_forward", "max_pooling_backward",
           "temporal_max_pooling", "out_size"]
