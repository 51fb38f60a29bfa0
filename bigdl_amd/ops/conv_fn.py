"""Differentiable convolutions on the native implicit-GEMM kernels (csrc/conv_igemm.hip) for the long tail of
conv-shaped layers that are written as autograd functions (``AutogradModule.fn``): transposed ("full")
convolution, temporal (1-D) convolution, connection-table convolution, the pointwise half of separable
convolution and volumetric (3-D) convolution — so none of them falls back to a vendor library on the GPU.

Every function takes / returns fp32 NCHW tensors like the layers' reference math; inside, activations run as
bf16 NHWC with channels zero-padded to multiples of 8 (the kernels' 16-byte granule) and fp32 accumulation.

    conv2d(x, w, b, stride, pad, dil)           y = x (*) w        fwd: NT GEMM, bwd: dgrad + wgrad kernels
    conv_transpose2d(x, w, b, stride, pad, adj) y = x (*)^T w      fwd: the dgrad kernel, bwd: fwd + wgrad
    conv3d(x, w, b, stride, pad)                sum over the kT taps of 2-D convs on depth-gathered batches

Reference: S/nn/SpatialConvolution.scala, SpatialFullConvolution.scala:71, TemporalConvolution.scala,
SpatialConvolutionMap.scala, SpatialSeparableConvolution.scala:54, VolumetricConvolution.scala:51.
"""
import torch
import torch.nn.functional as F

from . import conv as cv


def _zeros(*shape, **kw):
    from . import zeros

    return zeros(*shape, **kw)

BF16 = torch.bfloat16
CL = torch.channels_last


def _p8(n):
    return -(-n // 8) * 8


def _act16(x, C8):
    """fp32/bf16 NCHW -> bf16 NHWC with C padded to C8."""
    y = x.to(BF16).contiguous(memory_format=CL)
    if C8 != x.shape[1]:
        y = F.pad(y, (0, 0, 0, 0, 0, C8 - x.shape[1])).contiguous(memory_format=CL)
    return y


def _w16(w, K8, C8):
    """(K, C, R, S) -> bf16 KRSC (channels_last) padded to (K8, C8, R, S)."""
    K, C = w.shape[0], w.shape[1]
    w = w.to(BF16)
    if K8 != K or C8 != C:
        w = F.pad(w, (0, 0, 0, 0, 0, C8 - C, 0, K8 - K))
    return w.contiguous(memory_format=CL)


def _out_size(H, k, s, p, d):
    return (H + 2 * p - d * (k - 1) - 1) // s + 1


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dil):
        K, C = w.shape[0], w.shape[1]
        C8, K8 = _p8(C), _p8(K)
        x16 = _act16(x, C8)
        w16 = _w16(w, K8, C8)
        bias = None
        if b is not None:
            bias = b.float() if K8 == K else F.pad(b.float(), (0, K8 - K))
        y = cv.conv2d_fwd(x16, w16, bias, stride, pad, dil)
        ctx.save_for_backward(x16, w16)
        ctx.geo = (stride, pad, dil, K, C, x.shape, b is not None)
        return y[:, :K].float().contiguous()

    @staticmethod
    def backward(ctx, gy):
        x16, w16 = ctx.saved_tensors
        stride, pad, dil, K, C, xshape, has_b = ctx.geo
        K8, C8 = w16.shape[0], w16.shape[1]
        gy16 = _act16(gy, K8)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gi = cv.conv2d_dgrad(gy16, cv.transpose_w(w16), (xshape[0], C8, xshape[2], xshape[3]), stride, pad, dil)
            gx = gi[:, :C].float().contiguous()
        if ctx.needs_input_grad[1] or (has_b and ctx.needs_input_grad[2]):
            dw = _zeros(w16.shape, device=gy.device, memory_format=CL)
            db = _zeros(K8, device=gy.device) if has_b else None
            cv.conv2d_wgrad(gy16, x16, dw, db, stride, pad, dil)
            gw = dw[:K, :C].contiguous()
            gb = db[:K] if has_b else None
        return gx, gw, gb, None, None, None


def conv2d(x, w, b=None, stride=(1, 1), pad=(0, 0), dil=(1, 1)):
    """Native 2-D convolution (fp32 NCHW in / out). Falls back to torch on the CPU engine."""
    if not x.is_cuda:
        return F.conv2d(x, w, b, stride, pad, dil)
    return _Conv2d.apply(x, w, b, tuple(stride), tuple(pad), tuple(dil))


class _ConvT2d(torch.autograd.Function):
    """y = conv_transpose(x, w): exactly the data gradient of the conv that maps y's shape to x's with weight w
    (w: [Cin, Cout, kh, kw] is that conv's [K, C, R, S])."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, adj):
        Cin, Cout, kh, kw = w.shape
        N, _, H, W = x.shape
        OH = (H - 1) * stride[0] - 2 * pad[0] + kh + adj[0]
        OW = (W - 1) * stride[1] - 2 * pad[1] + kw + adj[1]
        K8, C8 = _p8(Cin), _p8(Cout)
        x16 = _act16(x, K8)
        w16 = _w16(w, K8, C8)
        y16 = cv.conv2d_dgrad(x16, cv.transpose_w(w16), (N, C8, OH, OW), stride, pad)
        y = y16[:, :Cout].float()
        if b is not None:
            y = y + b.view(1, -1, 1, 1)
        ctx.save_for_backward(x16, w16)
        ctx.geo = (stride, pad, Cin, Cout, b is not None)
        return y.contiguous()

    @staticmethod
    def backward(ctx, gy):
        x16, w16 = ctx.saved_tensors
        stride, pad, Cin, Cout, has_b = ctx.geo
        K8, C8 = w16.shape[0], w16.shape[1]
        gy16 = _act16(gy, C8)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            # the forward of the underlying conv (input = gy, output grid = x's)
            gi = cv.conv2d_fwd(gy16, w16, None, stride, pad)
            gx = gi[:, :Cin, :x16.shape[2], :x16.shape[3]].float().contiguous()
        if ctx.needs_input_grad[1]:
            dw = _zeros(w16.shape, device=gy.device, memory_format=CL)
            cv.conv2d_wgrad(x16, gy16, dw, None, stride, pad)
            gw = dw[:Cin, :Cout].contiguous()
        if has_b and ctx.needs_input_grad[2]:
            gb = gy.sum(dim=(0, 2, 3))
        return gx, gw, gb, None, None, None


def conv_transpose2d(x, w, b=None, stride=(1, 1), pad=(0, 0), adj=(0, 0)):
    if not x.is_cuda:
        return F.conv_transpose2d(x, w, b, stride, pad, adj)
    return _ConvT2d.apply(x, w, b, tuple(stride), tuple(pad), tuple(adj))


def linear(x, w, b=None):
    """y = x W^T + b over the last dimension on the MFMA GEMM kernels (a 1x1 convolution over the rows): the
    projections of layers written as autograd functions (attention, generic recurrent cells). CPU: torch."""
    if not x.is_cuda:
        return F.linear(x, w, b)
    lead = x.shape[:-1]
    rows = x.reshape(-1, x.shape[-1])
    y = conv2d(rows.view(rows.shape[0], rows.shape[1], 1, 1), w.view(w.shape[0], w.shape[1], 1, 1), b)
    return y.view(*lead, w.shape[0])


class _GroupConv(torch.autograd.Function):
    """Grouped / depthwise convolution in one launch per pass (csrc/grouped_conv.hip), fp32 NCHW."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dil, groups):
        from . import native

        x, w = x.float().contiguous(), w.float().contiguous()
        N, C, H, W = x.shape
        K, _, R, S = w.shape
        OH = (H + 2 * pad[0] - dil[0] * (R - 1) - 1) // stride[0] + 1
        OW = (W + 2 * pad[1] - dil[1] * (S - 1) - 1) // stride[1] + 1
        y = x.new_empty(N, K, OH, OW)
        geo = [stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], groups]
        native.get().gconv(0, x, w, b.float().contiguous() if b is not None else None, y, geo)
        ctx.save_for_backward(x, w)
        ctx.geo, ctx.has_b = geo, b is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        from . import native

        x, w = ctx.saved_tensors
        gy = gy.float().contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            native.get().gconv(1, gx, w, None, gy, ctx.geo)
        if ctx.needs_input_grad[1] or (ctx.has_b and ctx.needs_input_grad[2]):
            gw = torch.zeros_like(w)
            gb = torch.zeros(w.shape[0], device=x.device) if ctx.has_b else None
            native.get().gconv(2, x, gw, gb, gy, ctx.geo)
        return gx, gw, gb, None, None, None, None


def group_conv2d(x, w, b=None, stride=(1, 1), pad=(0, 0), dil=(1, 1), groups=1):
    """Grouped convolution: direct kernel when groups carry little reduction depth (depthwise, <= 16 input
    channels per group), else the implicit-GEMM conv per group writing its channel slice."""
    if not x.is_cuda:
        return F.conv2d(x, w, b, stride, pad, dil, groups)
    if groups == 1:
        return conv2d(x, w, b, stride, pad, dil)
    cin_g = x.shape[1] // groups
    if cin_g <= 16:
        return _GroupConv.apply(x, w, b, tuple(stride), tuple(pad), tuple(dil), groups)
    cout_g = w.shape[0] // groups
    outs = [conv2d(x[:, g * cin_g:(g + 1) * cin_g], w[g * cout_g:(g + 1) * cout_g],
                   b[g * cout_g:(g + 1) * cout_g] if b is not None else None, stride, pad, dil) for g in range(groups)]
    return torch.cat(outs, 1)


def conv1d(x, w, b=None, stride=1):
    """x: [N, C, L], w: [K, C, kW] -> [N, K, L'] as a 2-D convolution over a height-1 image."""
    if not x.is_cuda:
        return F.conv1d(x, w, b, stride)
    return conv2d(x.unsqueeze(2), w.unsqueeze(2), b, (1, stride), (0, 0)).squeeze(2)


def conv_transpose3d(x, w, b=None, stride=(1, 1, 1), pad=(0, 0, 0), adj=(0, 0, 0)):
    """x: [N, Cin, T, H, W], w: [Cin, Cout, kT, kH, kW]. Input frame t feeds output frames t*sT + kt - pT: each
    temporal tap kt is a native 2-D transposed convolution of all frames (folded into the batch), scattered into
    the output frames with index_add (the adjoint of conv3d's depth gather)."""
    if not x.is_cuda:
        return F.conv_transpose3d(x, w, b, stride, pad, adj)
    N, Cin, T, H, W = x.shape
    _, Cout, kT, kH, kW = w.shape
    sT, sH, sW = stride
    pT, pH, pW = pad
    OT = (T - 1) * sT - 2 * pT + kT + adj[0]
    L = max((T - 1) * sT + kT, pT + OT)                 # padded temporal extent
    xs = x.permute(0, 2, 1, 3, 4).reshape(N * T, Cin, H, W)
    y = None
    for kt in range(kT):
        part = conv_transpose2d(xs, w[:, :, kt], None, (sH, sW), (pH, pW), (adj[1], adj[2]))
        OH, OW = part.shape[2], part.shape[3]
        if y is None:
            y = part.new_zeros(N, L, Cout, OH, OW)
        idx = torch.arange(T, device=x.device) * sT + kt
        y = y.index_add(1, idx, part.view(N, T, Cout, OH, OW))
    y = y[:, pT:pT + OT].permute(0, 2, 1, 3, 4)
    if b is not None:
        y = y + b.view(1, -1, 1, 1, 1)
    return y.contiguous()


def conv3d(x, w, b=None, stride=(1, 1, 1), pad=(0, 0, 0)):
    """x: [N, C, T, H, W], w: [K, C, kT, kH, kW]. Each temporal tap kt is a 2-D convolution of the depth slices
    t*sT + kt - pT (zero outside) folded into the batch; the kT partial outputs are summed."""
    if not x.is_cuda:
        return F.conv3d(x, w, b, stride, pad)
    N, C, T, H, W = x.shape
    K, _, kT, kH, kW = w.shape
    sT, sH, sW = stride
    pT, pH, pW = pad
    OT = (T + 2 * pT - kT) // sT + 1
    xp = F.pad(x, (0, 0, 0, 0, pT, pT)) if pT else x
    y = None
    for kt in range(kT):
        idx = torch.arange(OT, device=x.device) * sT + kt
        xs = xp.index_select(2, idx).permute(0, 2, 1, 3, 4).reshape(N * OT, C, H, W)
        part = conv2d(xs, w[:, :, kt], b if kt == 0 else None, (sH, sW), (pH, pW))
        y = part if y is None else y + part
    OH, OW = y.shape[2], y.shape[3]
    return y.view(N, OT, K, OH, OW).permute(0, 2, 1, 3, 4).contiguous()
