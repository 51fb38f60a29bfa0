"""N-d pooling and nearest up-sampling on the GPU engine (csrc/pool_nd.hip), with CPU fallbacks.

Reference: S/nn/VolumetricMaxPooling.scala, S/nn/VolumetricAveragePooling.scala, S/nn/TemporalMaxPooling.scala,
S/nn/UpSampling1D.scala, S/nn/UpSampling2D.scala, S/nn/UpSampling3D.scala.

Every layout is handed to the kernels as a dense [B][D][H][W][C] view (C innermost): channels-first tensors are
B = N*C with C = 1, channels-last / sequence tensors keep their channel (feature) axis innermost. No layout copies
are made for contiguous inputs. CUDA tensors of bf16 / fp32 always take the native kernels (they fail loudly if the
extension is missing); other dtypes run in fp32 and are cast back. CPU tensors use torch.
"""
import torch
import torch.nn.functional as F

from . import native
from .conv import out_size

_NATIVE_DTYPES = (torch.float32, torch.bfloat16)


def _native_ok(x):
    return x.is_cuda


def _as_native(x):
    x = x.contiguous()
    return x if x.dtype in _NATIVE_DTYPES else x.float()


def pool_nd_fwd(x, out_shape, geo, max_mode, count_pad=True):
    """Raw forward over a dense view: returns (y, idx or None); y has x's dtype."""
    dt = x.dtype
    xn = _as_native(x)
    y = torch.empty(out_shape, dtype=xn.dtype, device=x.device)
    idx = torch.empty(out_shape, dtype=torch.int32, device=x.device) if max_mode else None
    native.get().poolnd_fwd(xn, y, idx, geo, bool(max_mode), bool(count_pad))
    return y.to(dt), idx


def pool_nd_bwd(gy, idx, x_shape, geo, max_mode, count_pad=True, dtype=None):
    """Raw backward (gather over covering windows): returns dx of x_shape."""
    dt = dtype or gy.dtype
    ndt = dt if dt in _NATIVE_DTYPES else torch.float32
    g = gy.to(ndt).contiguous()
    dx = torch.empty(x_shape, dtype=ndt, device=gy.device)
    native.get().poolnd_bwd(g, idx, dx, geo, bool(max_mode), bool(count_pad))
    return dx.to(dt)


class _PoolNdFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, out_shape, geo, max_mode, count_pad):
        y, idx = pool_nd_fwd(x, out_shape, geo, max_mode, count_pad)
        ctx.geo, ctx.max_mode, ctx.count_pad, ctx.x_shape, ctx.dt = geo, max_mode, count_pad, x.shape, x.dtype
        if max_mode:
            ctx.save_for_backward(idx)
        return y

    @staticmethod
    def backward(ctx, gy):
        idx = ctx.saved_tensors[0] if ctx.max_mode else None
        return pool_nd_bwd(gy, idx, ctx.x_shape, ctx.geo, ctx.max_mode, ctx.count_pad, ctx.dt), None, None, None, None


class _UpsampleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, out_shape, geo):
        dt = x.dtype
        xn = _as_native(x)
        y = torch.empty(out_shape, dtype=xn.dtype, device=x.device)
        native.get().upsample_nearest(xn, y, geo, False)
        ctx.geo, ctx.x_shape, ctx.ndt, ctx.dt = geo, x.shape, xn.dtype, dt
        return y.to(dt)

    @staticmethod
    def backward(ctx, gy):
        g = gy.to(ctx.ndt).contiguous()
        dx = torch.empty(ctx.x_shape, dtype=ctx.ndt, device=gy.device)
        native.get().upsample_nearest(g, dx, ctx.geo, True)
        return dx.to(ctx.dt), None, None


def pool2d_geo(x_shape, kh, kw, sh, sw, ph, pw, ceil=False):
    """(geo, out_shape) of a 2D window over an NCHW tensor seen as B = N*C planes (any channel count)."""
    N, C, H, W = x_shape
    OH, OW = out_size(H, kh, sh, ph, 1, ceil), out_size(W, kw, sw, pw, 1, ceil)
    return [N * C, 1, H, W, 1, 1, OH, OW, 1, kh, kw, 1, sh, sw, 0, ph, pw], (N, C, OH, OW)


def pool2d_explicit(x, k, s, pad_begin, out_hw, max_mode, count_pad):
    """Differentiable 2D pooling of an NCHW CUDA tensor with explicit output size and leading pads (windows are
    clipped to the input, so trailing / asymmetric padding needs no copy): TF SAME / VALID pooling."""
    N, C, H, W = x.shape
    geo = [N * C, 1, H, W, 1, 1, out_hw[0], out_hw[1], 1, k[0], k[1], 1, s[0], s[1], 0, pad_begin[0], pad_begin[1]]
    return _PoolNdFn.apply(x.contiguous(), (N, C, out_hw[0], out_hw[1]), geo, max_mode, count_pad)


def pool3d(x, k, s, p, ceil=False, max_mode=True, count_pad=True):
    """Max / average pooling of an NCDHW (or CDHW) tensor; k, s, p are (t, h, w) triples."""
    if not _native_ok(x):
        if max_mode:
            return F.max_pool3d(x, k, s, p, ceil_mode=ceil)
        return F.avg_pool3d(x, k, s, p, ceil, count_pad)
    sq = x.dim() == 4
    if sq:
        x = x.unsqueeze(0)
    N, C, D, H, W = x.shape
    OD, OH, OW = (out_size(n, kk, ss, pp, 1, ceil) for n, kk, ss, pp in zip((D, H, W), k, s, p))
    geo = [N * C, D, H, W, 1, OD, OH, OW, *k, *s, *p]
    y = _PoolNdFn.apply(x, (N, C, OD, OH, OW), geo, max_mode, count_pad)
    return y.squeeze(0) if sq else y


def temporal_max_pool(x, kW, dW):
    """Max over time windows of a (batch, frames, features) or (frames, features) sequence."""
    sq = x.dim() == 2
    if sq:
        x = x.unsqueeze(0)
    if not _native_ok(x):
        y = F.max_pool1d(x.transpose(1, 2), kW, dW).transpose(1, 2)
    else:
        N, T, Fd = x.shape
        OT = (T - kW) // dW + 1
        geo = [N, 1, 1, T, Fd, 1, 1, OT, 1, 1, kW, 1, 1, dW, 0, 0, 0]
        y = _PoolNdFn.apply(x, (N, OT, Fd), geo, True, True)
    return y.squeeze(0) if sq else y


def upsample_nearest(x, factors, channels_last=False, sequence=False):
    """Nearest up-sampling by integer factors.

    sequence=True: x is (batch, steps, features) and factors = (length,).
    channels_last=True: x is NHWC and factors = (h, w).
    otherwise x is N C <spatial...> with one factor per spatial axis (1 to 3 of them).
    """
    factors = tuple(int(f) for f in factors)
    if not _native_ok(x):
        if sequence:
            return x.repeat_interleave(factors[0], dim=1)
        if channels_last:
            return x.repeat_interleave(factors[0], 1).repeat_interleave(factors[1], 2)
        for i, f in enumerate(factors):
            x = x.repeat_interleave(f, 2 + i)
        return x
    if sequence:
        N, T, Fd = x.shape
        geo = [N, 1, 1, T, Fd, 1, 1, T * factors[0], 1, 1, factors[0], 1, 1, 1, 0, 0, 0]
        return _UpsampleFn.apply(x, (N, T * factors[0], Fd), geo)
    if channels_last:
        N, H, W, C = x.shape
        fh, fw = factors
        geo = [N, 1, H, W, C, 1, H * fh, W * fw, 1, fh, fw, 1, 1, 1, 0, 0, 0]
        return _UpsampleFn.apply(x, (N, H * fh, W * fw, C), geo)
    N, C = x.shape[:2]
    sp = list(x.shape[2:])
    fs = list(factors)
    while len(sp) < 3:                       # pad to (D, H, W) with unit axes in front
        sp.insert(0, 1)
        fs.insert(0, 1)
    D, H, W = sp
    kd, kh, kw = fs
    geo = [N * C, D, H, W, 1, D * kd, H * kh, W * kw, kd, kh, kw, 1, 1, 1, 0, 0, 0]
    out_shape = (N, C) + tuple(n * f for n, f in zip(x.shape[2:], factors))
    return _UpsampleFn.apply(x, out_shape, geo)


__all__ = ["pool_nd_fwd", "pool_nd_bwd", "pool2d_geo", "pool2d_explicit", "pool3d", "temporal_max_pool", "upsample_nearest"]
