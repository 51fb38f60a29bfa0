"""TensorFlow-semantics operations as modules (the reference's ``nn/ops`` + ``nn/tf`` op families).

Reference: S/nn/ops/*.scala (71 files: Operation base :32, element-wise math / comparison / logical ops,
reductions, Gather, OneHot, Pad, Slice, Tile, TopK, InTopK, SegmentSum, BatchMatMul, DepthwiseConv2D,
Dilation2D, ResizeBilinear, RandomUniform, TruncatedNormal, CrossEntropy, feature-column ops),
S/nn/tf/*.scala (18 files: BiasAdd, Shape, StridedSlice, SplitAndSelect, ArrayOps (Pack/Unpack/Concat/...),
ControlDependency, NoOp, Assert, StateOps (Variable/Assign), ImageOps, ParsingOps).

Design: one table ``OPS`` maps a TF op name to ``fn(inputs, attrs) -> tensor | list`` written with torch ops on the
tensors' device, so an imported graph runs on the GPU engine unchanged. ``TFOp`` wraps one table entry as a module:
inputs that were constant in the source graph are baked in (``consts``: position -> tensor buffer), the rest arrive
as the module input (a tensor, or a Table when several). Floating-point ops back-propagate through torch autograd;
integer / boolean ops are forward-only like the reference's ``Operation``. Multi-output ops return a Table.
Named classes (``Gather``, ``OneHot``, ``StridedSlice``, ...) are thin constructors over ``TFOp``.
"""
import math

import torch
import torch.nn.functional as F

from ..utils.table import Table
from .abstractnn import AutogradModule

# TF DataType enum -> torch dtype (None: string / resource)
TF_DTYPES = {"DT_FLOAT": torch.float32, "DT_DOUBLE": torch.float64, "DT_INT32": torch.int32, "DT_UINT8": torch.uint8,
             "DT_INT16": torch.int16, "DT_INT8": torch.int8, "DT_STRING": None, "DT_INT64": torch.int64,
             "DT_BOOL": torch.bool, "DT_BFLOAT16": torch.bfloat16, "DT_HALF": torch.float16,
             "DT_UINT16": torch.int32, "DT_UINT32": torch.int64, "DT_UINT64": torch.int64}


def _i(t):
    return [int(v) for v in (t.reshape(-1).tolist() if isinstance(t, torch.Tensor) else list(t))]


def _axis(t, rank):
    a = int(t.reshape(-1)[0]) if isinstance(t, torch.Tensor) else int(t)
    return a + rank if a < 0 else a


def _bcast(a, b):
    if isinstance(a, torch.Tensor) and isinstance(b, torch.Tensor):
        if a.dtype != b.dtype:
            dt = torch.promote_types(a.dtype, b.dtype)
            a, b = a.to(dt), b.to(dt)
        if a.device != b.device:
            b = b.to(a.device)
    return a, b


def _bin(fn):
    def run(x, at):
        a, b = _bcast(x[0], x[1])
        return fn(a, b)
    return run


def _un(fn):
    return lambda x, at: fn(x[0])


def _reduce(fn):
    def run(x, at):
        t = x[0]
        keep = bool(at.get("keep_dims", at.get("keepdims", False)))
        axes = sorted({a + t.dim() if a < 0 else a for a in _i(x[1])}) if len(x) > 1 else list(range(t.dim()))
        if not axes:
            return t
        return fn(t, axes, keep)
    return run


def _sum(t, axes, keep):
    return t.sum(dim=axes, keepdim=keep)


def _prod(t, axes, keep):
    for a in sorted(axes, reverse=True):
        t = t.prod(dim=a, keepdim=keep)
    return t


def _amax(t, axes, keep):
    return t.amax(dim=axes, keepdim=keep)


def _amin(t, axes, keep):
    return t.amin(dim=axes, keepdim=keep)


def _mean(t, axes, keep):
    return t.float().mean(dim=axes, keepdim=keep).to(t.dtype) if not t.is_floating_point() else t.mean(dim=axes,
                                                                                                       keepdim=keep)


def _all(t, axes, keep):
    t = t.bool()
    for a in sorted(axes, reverse=True):
        t = t.all(dim=a, keepdim=keep)
    return t


def _any(t, axes, keep):
    t = t.bool()
    for a in sorted(axes, reverse=True):
        t = t.any(dim=a, keepdim=keep)
    return t


def _nchw(x, fmt):
    return x.permute(0, 3, 1, 2) if fmt == "NHWC" else x


def _back(x, fmt):
    return x.permute(0, 2, 3, 1) if fmt == "NHWC" else x


def _hw(v, fmt):
    v = _i(v)
    return (v[1], v[2]) if fmt == "NHWC" else (v[2], v[3])


def _same_pads(n, k, s, d=1):
    out = -(-n // s)
    total = max((out - 1) * s + (k - 1) * d + 1 - n, 0)
    return total // 2, total - total // 2


def _conv2d(x, at):
    inp, w = x[0], x[1]
    fmt = at.get("data_format", "NHWC")
    sh, sw = _hw(at.get("strides", [1, 1, 1, 1]), fmt)
    dh, dw = _hw(at.get("dilations", [1, 1, 1, 1]), fmt)
    xi = _nchw(inp, fmt)
    wt = w.permute(3, 2, 0, 1).to(xi.dtype)          # HWIO -> OIHW
    if at.get("padding", "VALID") == "SAME":
        ph = _same_pads(xi.shape[2], wt.shape[2], sh, dh)
        pw = _same_pads(xi.shape[3], wt.shape[3], sw, dw)
        xi = F.pad(xi, (pw[0], pw[1], ph[0], ph[1]))
    if xi.is_cuda:                                     # native implicit GEMM (ops/conv_fn.py)
        from ..ops import conv_fn

        y = conv_fn.conv2d(xi.float(), wt.float(), None, (sh, sw), (0, 0), (dh, dw)).to(xi.dtype)
    else:
        y = F.conv2d(xi, wt, None, (sh, sw), 0, (dh, dw))
    return _back(y, fmt)


def _depthwise(x, at):
    inp, w = x[0], x[1]
    fmt = at.get("data_format", "NHWC")
    sh, sw = _hw(at.get("strides", [1, 1, 1, 1]), fmt)
    xi = _nchw(inp, fmt)
    kh, kw, cin, mult = w.shape
    wt = w.permute(2, 3, 0, 1).reshape(cin * mult, 1, kh, kw).to(xi.dtype)
    if at.get("padding", "VALID") == "SAME":
        ph, pw = _same_pads(xi.shape[2], kh, sh), _same_pads(xi.shape[3], kw, sw)
        xi = F.pad(xi, (pw[0], pw[1], ph[0], ph[1]))
    if xi.is_cuda:                                     # one-launch grouped / depthwise kernel
        from ..ops import conv_fn

        return _back(conv_fn.group_conv2d(xi.float(), wt.float(), None, (sh, sw), (0, 0), (1, 1), cin).to(xi.dtype), fmt)
    return _back(F.conv2d(xi, wt, None, (sh, sw), 0, 1, cin), fmt)


def _conv2d_transpose(x, at):
    """Conv2DBackpropInput(input_sizes, filter, out_backprop): the transposed convolution."""
    sizes, w, dy = _i(x[0]), x[1], x[2]
    fmt = at.get("data_format", "NHWC")
    sh, sw = _hw(at.get("strides", [1, 1, 1, 1]), fmt)
    g = _nchw(dy, fmt)
    wt = w.permute(3, 2, 0, 1).to(g.dtype)             # OIHW of the forward conv
    H, W = (sizes[1], sizes[2]) if fmt == "NHWC" else (sizes[2], sizes[3])
    kh, kw = wt.shape[2], wt.shape[3]
    if at.get("padding", "VALID") == "SAME":
        ph, pw = _same_pads(H, kh, sh), _same_pads(W, kw, sw)
    else:
        ph, pw = (0, 0), (0, 0)
    Hp, Wp = H + ph[0] + ph[1], W + pw[0] + pw[1]
    oh = Hp - ((g.shape[2] - 1) * sh + kh)
    ow = Wp - ((g.shape[3] - 1) * sw + kw)
    if g.is_cuda:                                      # the native data-gradient kernel
        from ..ops import conv_fn

        y = conv_fn.conv_transpose2d(g.float(), wt.float(), None, (sh, sw), (0, 0), (oh, ow)).to(g.dtype)
    else:
        y = F.conv_transpose2d(g, wt, None, (sh, sw), 0, (oh, ow))
    y = y[:, :, ph[0]: ph[0] + H, pw[0]: pw[0] + W]
    return _back(y, fmt)


def tf_pool2d(xi, kind, k, s, same):
    """TF max / avg pooling of an NCHW tensor (SAME: output ceil(H/s), leading pad (total)//2, averages exclude
    the padding). GPU: the N-d window kernel with explicit leading pads (csrc/pool_nd.hip); CPU: torch."""
    H, W = xi.shape[2], xi.shape[3]
    if same:
        ph, pw = _same_pads(H, k[0], s[0]), _same_pads(W, k[1], s[1])
        oh, ow = -(-H // s[0]), -(-W // s[1])
    else:
        ph, pw = (0, 0), (0, 0)
        oh, ow = (H - k[0]) // s[0] + 1, (W - k[1]) // s[1] + 1
    if xi.is_cuda:
        from ..ops.pool_nd import pool2d_explicit

        return pool2d_explicit(xi, k, s, (ph[0], pw[0]), (oh, ow), kind == "max", False)
    pads = (pw[0], pw[1], ph[0], ph[1])
    if kind == "max":
        return F.max_pool2d(F.pad(xi, pads, value=float("-inf")), k, s)
    num = F.avg_pool2d(F.pad(xi, pads), k, s)
    den = F.avg_pool2d(F.pad(torch.ones_like(xi[:, :1]), pads), k, s)
    return num / den


def _pool(kind):
    def run(x, at):
        fmt = at.get("data_format", "NHWC")
        kh, kw = _hw(at["ksize"], fmt)
        sh, sw = _hw(at["strides"], fmt)
        xi = _nchw(x[0], fmt)
        if xi.is_cuda:
            return _back(tf_pool2d(xi, kind, (kh, kw), (sh, sw), at.get("padding", "VALID") == "SAME"), fmt)
        if at.get("padding", "VALID") == "SAME":
            ph, pw = _same_pads(xi.shape[2], kh, sh), _same_pads(xi.shape[3], kw, sw)
            pads = (pw[0], pw[1], ph[0], ph[1])
            if kind == "max":
                y = F.max_pool2d(F.pad(xi, pads, value=float("-inf")), (kh, kw), (sh, sw))
            else:
                num = F.avg_pool2d(F.pad(xi, pads), (kh, kw), (sh, sw))
                den = F.avg_pool2d(F.pad(torch.ones_like(xi[:, :1]), pads), (kh, kw), (sh, sw))
                y = num / den
        else:
            y = F.max_pool2d(xi, (kh, kw), (sh, sw)) if kind == "max" else F.avg_pool2d(xi, (kh, kw), (sh, sw))
        return _back(y, fmt)
    return run


def _fused_bn(x, at):
    t, scale, offset, mean, var = x[:5]
    fmt = at.get("data_format", "NHWC")
    eps = float(at.get("epsilon", 1e-3))
    xi = _nchw(t, fmt)
    if at.get("is_training", True) and (mean.numel() == 0 or True) and at.get("is_training", True):
        m = xi.mean(dim=(0, 2, 3))
        v = xi.var(dim=(0, 2, 3), unbiased=False)
    else:
        m, v = mean, var
    y = (xi - m[None, :, None, None]) * torch.rsqrt(v[None, :, None, None] + eps) * scale[None, :, None, None] + \
        offset[None, :, None, None]
    return [_back(y, fmt), m, v, m, v]


def _strided_slice(x, at):
    t = x[0]
    begin, end, strides = _i(x[1]), _i(x[2]), _i(x[3])
    bm, em = int(at.get("begin_mask", 0)), int(at.get("end_mask", 0))
    el, na, sa = int(at.get("ellipsis_mask", 0)), int(at.get("new_axis_mask", 0)), int(at.get("shrink_axis_mask", 0))
    idx, dim = [], 0
    n = len(begin)
    for i in range(n):
        if el & (1 << i):
            rest = t.dim() - (n - i - 1 - bin(na >> (i + 1)).count("1"))
            while dim < rest:
                idx.append(slice(None))
                dim += 1
            continue
        if na & (1 << i):
            idx.append(None)
            continue
        if sa & (1 << i):
            b = begin[i] + t.shape[dim] if begin[i] < 0 else begin[i]
            idx.append(b)
            dim += 1
            continue
        s = strides[i]
        b = None if bm & (1 << i) else begin[i]
        e = None if em & (1 << i) else end[i]
        if s < 0:
            size = t.shape[dim]
            b = size - 1 if b is None else (b + size if b < 0 else b)
            e = -1 if e is None else (e + size if e < 0 else e)
            rng = list(range(b, e, s))
            idx.append(torch.tensor(rng, dtype=torch.long, device=t.device) if rng else slice(0, 0))
        else:
            idx.append(slice(b, e, s))
        dim += 1
    out = t
    # apply one axis at a time so tensor indices do not broadcast against each other
    pos = 0
    for it in idx:
        if it is None:
            out = out.unsqueeze(pos)
            pos += 1
        elif isinstance(it, int):
            out = out.select(pos, it)
        elif isinstance(it, torch.Tensor):
            out = out.index_select(pos, it)
            pos += 1
        else:
            out = out[(slice(None),) * pos + (it,)]
            pos += 1
    return out


def _slice(x, at):
    t, begin, size = x[0], _i(x[1]), _i(x[2])
    idx = tuple(slice(b, None if s == -1 else b + s) for b, s in zip(begin, size))
    return t[idx]


def _pad(x, at, mode="constant"):
    t, p = x[0], x[1].reshape(-1, 2).tolist()
    value = float(x[2].reshape(-1)[0]) if len(x) > 2 else 0.0
    pads = []
    for a, b in reversed(p):
        pads += [int(a), int(b)]
    if mode == "constant":
        return F.pad(t, pads, value=value)
    m = at.get("mode", "REFLECT").lower()
    return F.pad(t.unsqueeze(0) if t.dim() < 3 else t, pads, mode="reflect" if m == "reflect" else "replicate")


def _onehot(x, at):
    idx, depth = x[0].long(), int(x[1].reshape(-1)[0])
    on = x[2].reshape(-1)[0] if len(x) > 2 else torch.tensor(1.0)
    off = x[3].reshape(-1)[0] if len(x) > 3 else torch.tensor(0.0)
    axis = int(at.get("axis", -1))
    valid = (idx >= 0) & (idx < depth)
    oh = F.one_hot(idx.clamp(0, depth - 1), depth) * valid.unsqueeze(-1)
    y = oh.to(on.dtype) * on + (1 - oh).to(on.dtype) * off
    if axis != -1:
        y = y.movedim(-1, axis)
    return y


def _gather(x, at):
    params, ind = x[0], x[1].long()
    axis = _axis(x[2], params.dim()) if len(x) > 2 else 0
    return params.index_select(axis, ind.reshape(-1)).reshape(params.shape[:axis] + ind.shape + params.shape[axis + 1:])


def _topk(x, at):
    k = int(x[1].reshape(-1)[0]) if len(x) > 1 else int(at.get("k", 1))
    v, i = torch.topk(x[0], k, dim=-1, largest=True, sorted=bool(at.get("sorted", True)))
    return [v, i.int()]


def _in_topk(x, at):
    pred, target = x[0], x[1].long()
    k = int(x[2].reshape(-1)[0]) if len(x) > 2 else int(at.get("k", 1))
    t = pred.gather(1, target[:, None])
    return (pred > t).sum(1) < k


def _segment_sum(x, at):
    data, seg = x[0], x[1].long()
    n = int(seg.max()) + 1 if seg.numel() else 0
    out = torch.zeros((n,) + tuple(data.shape[1:]), dtype=data.dtype, device=data.device)
    return out.index_add(0, seg, data)


def _softmax_xent(x, at):
    logits, labels = x[0], x[1]
    lsm = torch.log_softmax(logits, dim=-1)
    loss = -(labels * lsm).sum(-1)
    return [loss, torch.softmax(logits, -1) - labels]


def _sparse_softmax_xent(x, at):
    logits, labels = x[0], x[1].long()
    lsm = torch.log_softmax(logits, dim=-1)
    loss = -lsm.gather(-1, labels[..., None]).squeeze(-1)
    return [loss, torch.softmax(logits, -1) - F.one_hot(labels, logits.shape[-1]).to(logits.dtype)]


def _resize(mode):
    def run(x, at):
        t, size = x[0], _i(x[1])
        xi = t.permute(0, 3, 1, 2)
        if mode == "bilinear":
            if at.get("align_corners", False):
                y = F.interpolate(xi.float(), size=size, mode="bilinear", align_corners=True)
            else:      # TF1 legacy (half_pixel_centers=False): src = dst * in / out
                H, W = xi.shape[2], xi.shape[3]
                ys = torch.arange(size[0], device=t.device, dtype=torch.float32) * (H / size[0])
                xs = torch.arange(size[1], device=t.device, dtype=torch.float32) * (W / size[1])
                y0, x0 = ys.floor().long().clamp(max=H - 1), xs.floor().long().clamp(max=W - 1)
                y1, x1 = (y0 + 1).clamp(max=H - 1), (x0 + 1).clamp(max=W - 1)
                ly, lx = (ys - y0)[:, None], (xs - x0)[None, :]
                f = xi.float()
                top = f[:, :, y0][:, :, :, x0] * (1 - lx) + f[:, :, y0][:, :, :, x1] * lx
                bot = f[:, :, y1][:, :, :, x0] * (1 - lx) + f[:, :, y1][:, :, :, x1] * lx
                y = top * (1 - ly) + bot * ly
        else:
            y = F.interpolate(xi.float(), size=size, mode="nearest")
        return y.permute(0, 2, 3, 1).to(t.dtype)
    return run


def _dilation2d(x, at):
    """Grayscale morphological dilation: out = max_{dy,dx} x[y*s+dy*r, x*s+dx*r] + w[dy, dx]."""
    t, w = x[0], x[1]
    sh, sw = _i(at.get("strides", [1, 1, 1, 1]))[1:3]
    rh, rw = _i(at.get("rates", [1, 1, 1, 1]))[1:3]
    kh, kw, c = w.shape
    xi = t.permute(0, 3, 1, 2)
    ekh, ekw = (kh - 1) * rh + 1, (kw - 1) * rw + 1
    if at.get("padding", "VALID") == "SAME":
        ph, pw = _same_pads(xi.shape[2], ekh, sh), _same_pads(xi.shape[3], ekw, sw)
        xi = F.pad(xi, (pw[0], pw[1], ph[0], ph[1]), value=float("-inf"))
    cols = F.unfold(xi, (kh, kw), dilation=(rh, rw), stride=(sh, sw))       # N, C*kh*kw, L
    N = xi.shape[0]
    oh = (xi.shape[2] - ekh) // sh + 1
    ow = (xi.shape[3] - ekw) // sw + 1
    cols = cols.reshape(N, c, kh * kw, oh * ow) + w.permute(2, 0, 1).reshape(1, c, kh * kw, 1)
    return cols.amax(dim=2).reshape(N, c, oh, ow).permute(0, 2, 3, 1)


def _lrn(x, at):
    t = x[0].permute(0, 3, 1, 2)
    r = int(at.get("depth_radius", 5))
    bias, alpha, beta = float(at.get("bias", 1.0)), float(at.get("alpha", 1.0)), float(at.get("beta", 0.5))
    sq = F.pad((t * t).unsqueeze(1), (0, 0, 0, 0, r, r)).squeeze(1)
    s = sum(sq[:, i: i + t.shape[1]] for i in range(2 * r + 1))
    return (t / (bias + alpha * s) ** beta).permute(0, 2, 3, 1)


def _split(x, at):
    axis = _axis(x[0], x[1].dim())
    n = int(at.get("num_split", 1))
    return list(torch.chunk(x[1], n, dim=axis))


def _splitv(x, at):
    sizes = _i(x[1])
    axis = _axis(x[2], x[0].dim())
    if -1 in sizes:
        sizes[sizes.index(-1)] = x[0].shape[axis] - (sum(sizes) + 1)
    return list(torch.split(x[0], sizes, dim=axis))


def _concat_v2(x, at):
    ts = x[:-1]
    axis = _axis(x[-1], ts[0].dim())
    dt = ts[0].dtype
    return torch.cat([t.to(dt) for t in ts], dim=axis)


def _reshape(x, at):
    shape = _i(x[1])
    return x[0].reshape(shape)


def _range(x, at):
    a, b, d = [v.reshape(-1)[0].item() for v in x[:3]]
    dt = x[0].dtype
    return torch.arange(a, b, d, dtype=dt if dt.is_floating_point else torch.int64).to(dt)


def _fill(x, at):
    return torch.full(_i(x[0]), x[1].reshape(-1)[0].item(), dtype=x[1].dtype, device=x[1].device)


def _cast(x, at):
    dt = TF_DTYPES.get(at.get("DstT", "DT_FLOAT"), torch.float32)
    return x[0].to(dt)


def _rand_uniform(x, at):
    from ..utils.random_generator import RNG
    return RNG.uniform(0.0, 1.0, tuple(_i(x[0])))


def _trunc_normal(x, at):
    from ..utils.random_generator import RNG
    t = RNG.normal(0.0, 1.0, tuple(_i(x[0])))
    while True:
        bad = t.abs() > 2
        if not bool(bad.any()):
            return t
        t[bad] = RNG.normal(0.0, 1.0, (int(bad.sum()),))


def _select(x, at):
    c, a, b = x[0].bool(), x[1], x[2]
    if c.dim() == 1 and a.dim() > 1:
        c = c.reshape((-1,) + (1,) * (a.dim() - 1))
    return torch.where(c, a, b)


def _matmul(x, at):
    a, b = _bcast(x[0], x[1])
    if at.get("transpose_a", False):
        a = a.t()
    if at.get("transpose_b", False):
        b = b.t()
    return a @ b


def _batch_matmul(x, at):
    a, b = _bcast(x[0], x[1])
    if at.get("adj_x", False):
        a = a.transpose(-1, -2)
    if at.get("adj_y", False):
        b = b.transpose(-1, -2)
    return a @ b


def _bias_add(x, at):
    t, b = x[0], x[1]
    if at.get("data_format", "NHWC") == "NCHW" and t.dim() >= 3:
        return t + b.reshape((1, -1) + (1,) * (t.dim() - 2))
    return t + b


def _squeeze(x, at):
    dims = _i(at.get("squeeze_dims", [])) if at.get("squeeze_dims") is not None else []
    t = x[0]
    if not dims:
        return t.squeeze()
    for d in sorted([d + t.dim() if d < 0 else d for d in dims], reverse=True):
        t = t.squeeze(d)
    return t


def _expand_dims(x, at):
    d = int(x[1].reshape(-1)[0])
    return x[0].unsqueeze(d if d >= 0 else d + x[0].dim() + 1)


def _transpose(x, at):
    return x[0].permute(*_i(x[1]))


def _tile(x, at):
    return x[0].repeat(*_i(x[1]))


def _pack(x, at):
    axis = int(at.get("axis", 0))
    return torch.stack(list(x), dim=axis)


def _unpack(x, at):
    axis = int(at.get("axis", 0))
    return list(torch.unbind(x[0], dim=axis))


def _argmax(fn):
    def run(x, at):
        d = _axis(x[1], x[0].dim()) if len(x) > 1 else 0
        r = fn(x[0], dim=d)
        return r.to(TF_DTYPES.get(at.get("output_type", "DT_INT64"), torch.int64))
    return run


def _l2loss(x, at):
    return (x[0] * x[0]).sum() / 2


def _approx_eq(x, at):
    a, b = _bcast(x[0], x[1])
    return (a - b).abs() < float(at.get("tolerance", 1e-5))


def _floor_mod(a, b):
    return torch.remainder(a, b)


def _trunc_div(a, b):
    return torch.div(a, b, rounding_mode="trunc")


def _floor_div(a, b):
    return torch.div(a, b, rounding_mode="floor") if not a.is_floating_point() else torch.floor(a / b)


def _real_div(a, b):
    return a / b if a.is_floating_point() else torch.div(a, b, rounding_mode="trunc")


OPS = {
    # element-wise unary
    "Abs": _un(torch.abs), "Neg": _un(torch.neg), "Exp": _un(torch.exp), "Expm1": _un(torch.expm1),
    "Log": _un(torch.log), "Log1p": _un(torch.log1p), "Sqrt": _un(torch.sqrt), "Rsqrt": _un(torch.rsqrt),
    "Square": _un(torch.square), "Reciprocal": _un(torch.reciprocal), "Inv": _un(torch.reciprocal),
    "Sign": _un(torch.sign), "Floor": _un(torch.floor), "Ceil": _un(torch.ceil), "Round": _un(torch.round),
    "Rint": _un(torch.round), "Tanh": _un(torch.tanh), "Sigmoid": _un(torch.sigmoid), "Relu": _un(torch.relu),
    "Relu6": _un(lambda t: torch.clamp(t, 0, 6)), "Elu": _un(F.elu), "Selu": _un(F.selu),
    "Softplus": _un(F.softplus), "Softsign": _un(F.softsign), "Erf": _un(torch.erf), "Erfc": _un(torch.erfc),
    "Lgamma": _un(torch.lgamma), "Digamma": _un(torch.digamma), "IsFinite": _un(torch.isfinite),
    "IsInf": _un(torch.isinf), "IsNan": _un(torch.isnan), "LogicalNot": _un(torch.logical_not),
    "Sin": _un(torch.sin), "Cos": _un(torch.cos), "Identity": _un(lambda t: t), "StopGradient": _un(lambda t: t),
    "Snapshot": _un(lambda t: t), "ZerosLike": _un(torch.zeros_like), "OnesLike": _un(torch.ones_like),
    "Softmax": _un(lambda t: torch.softmax(t, -1)), "LogSoftmax": _un(lambda t: torch.log_softmax(t, -1)),
    "Shape": lambda x, at: torch.tensor(list(x[0].shape), dtype=TF_DTYPES.get(at.get("out_type", "DT_INT32"))),
    "Size": lambda x, at: torch.tensor(x[0].numel(), dtype=torch.int32),
    "Rank": lambda x, at: torch.tensor(x[0].dim(), dtype=torch.int32),
    # binary (broadcasting)
    "Add": _bin(torch.add), "AddV2": _bin(torch.add), "Sub": _bin(torch.sub), "Mul": _bin(torch.mul),
    "Div": _bin(_real_div), "RealDiv": _bin(_real_div), "FloorDiv": _bin(_floor_div), "FloorMod": _bin(_floor_mod),
    "Mod": _bin(torch.fmod), "TruncateDiv": _bin(_trunc_div), "TruncateMod": _bin(torch.fmod),
    "Pow": _bin(torch.pow), "Maximum": _bin(torch.maximum), "Minimum": _bin(torch.minimum),
    "SquaredDifference": _bin(lambda a, b: (a - b) ** 2), "Equal": _bin(torch.eq), "NotEqual": _bin(torch.ne),
    "Greater": _bin(torch.gt), "GreaterEqual": _bin(torch.ge), "Less": _bin(torch.lt), "LessEqual": _bin(torch.le),
    "LogicalAnd": _bin(torch.logical_and), "LogicalOr": _bin(torch.logical_or), "ApproximateEqual": _approx_eq,
    "BiasAdd": _bias_add, "BiasAddV1": _bias_add,
    # n-ary / shape
    "AddN": lambda x, at: sum(x[1:], x[0]), "ConcatV2": _concat_v2,
    "Concat": lambda x, at: torch.cat(list(x[1:]), dim=_axis(x[0], x[1].dim())),
    "Pack": _pack, "Unpack": _unpack, "Split": _split, "SplitV": _splitv, "Reshape": _reshape,
    "Squeeze": _squeeze, "ExpandDims": _expand_dims, "Transpose": _transpose, "Tile": _tile,
    "Pad": _pad, "PadV2": _pad, "MirrorPad": lambda x, at: _pad(x, at, "mirror"), "Slice": _slice,
    "StridedSlice": _strided_slice, "Fill": _fill, "Range": _range, "Cast": _cast, "Select": _select,
    "SelectV2": _select, "Gather": _gather, "GatherV2": _gather, "OneHot": _onehot,
    "BroadcastTo": lambda x, at: x[0].expand(*_i(x[1])),
    # reductions
    "Sum": _reduce(_sum), "Prod": _reduce(_prod), "Max": _reduce(_amax), "Min": _reduce(_amin),
    "Mean": _reduce(_mean), "All": _reduce(_all), "Any": _reduce(_any),
    "ArgMax": _argmax(torch.argmax), "ArgMin": _argmax(torch.argmin),
    # nn
    "MatMul": _matmul, "BatchMatMul": _batch_matmul, "BatchMatMulV2": _batch_matmul, "Conv2D": _conv2d,
    "DepthwiseConv2dNative": _depthwise, "Conv2DBackpropInput": _conv2d_transpose, "MaxPool": _pool("max"),
    "AvgPool": _pool("avg"), "FusedBatchNorm": _fused_bn, "FusedBatchNormV2": _fused_bn,
    "FusedBatchNormV3": _fused_bn, "LRN": _lrn, "SoftmaxCrossEntropyWithLogits": _softmax_xent,
    "SparseSoftmaxCrossEntropyWithLogits": _sparse_softmax_xent, "L2Loss": _l2loss,
    "ResizeBilinear": _resize("bilinear"), "ResizeNearestNeighbor": _resize("nearest"), "TopK": _topk,
    "TopKV2": _topk, "InTopK": _in_topk, "InTopKV2": _in_topk, "SegmentSum": _segment_sum, "Dilation2D": _dilation2d,
    # random
    "RandomUniform": _rand_uniform, "TruncatedNormal": _trunc_normal,
    "RandomStandardNormal": lambda x, at: __import__("bigdl_amd.utils.random_generator", fromlist=["RNG"]).RNG.normal(
        0.0, 1.0, tuple(_i(x[0]))),
    # control / misc
    "NoOp": lambda x, at: torch.zeros(0), "Assert": lambda x, at: x[0] if x else torch.zeros(0),
}

MULTI_OUTPUT = {"Unpack", "Split", "SplitV", "TopK", "TopKV2", "SoftmaxCrossEntropyWithLogits",
                "SparseSoftmaxCrossEntropyWithLogits", "FusedBatchNorm", "FusedBatchNormV2", "FusedBatchNormV3"}


def run_op(op, inputs, attrs):
    if op not in OPS:
        raise NotImplementedError(f"TensorFlow op {op} is not supported")
    return OPS[op](list(inputs), attrs)


class TFOp(AutogradModule):
    """One TF-semantics op. ``consts`` maps input positions to fixed tensors; the module input supplies the
    remaining positions in order (tensor for one, Table for several)."""

    def __init__(self, op, attrs=None, consts=None, n_inputs=None):
        super().__init__()
        if op not in OPS:
            raise NotImplementedError(f"TensorFlow op {op} is not supported")
        self.op = op
        self.attrs = dict(attrs or {})
        self.n_inputs = n_inputs
        self.const_pos = sorted((consts or {}).keys())
        self._buffers = []
        for p in self.const_pos:
            name = f"const{p}"
            setattr(self, name, consts[p])
            self._buffers.append(name)

    def _assemble(self, x):
        dyn = [] if x is None else ([x[i + 1] for i in range(x.length())] if isinstance(x, Table) else [x])
        n = self.n_inputs if self.n_inputs is not None else len(dyn) + len(self.const_pos)
        out, it = [], iter(dyn)
        for i in range(n):
            if i in self.const_pos:
                c = getattr(self, f"const{i}")
                if dyn and isinstance(c, torch.Tensor) and isinstance(dyn[0], torch.Tensor) and c.device != dyn[0].device:
                    c = c.to(dyn[0].device)
                out.append(c)
            else:
                out.append(next(it))
        return out

    def fn(self, x):
        r = run_op(self.op, self._assemble(x), self.attrs)
        if isinstance(r, (list, tuple)):
            t = Table()
            for i, v in enumerate(r):
                t[i + 1] = v
            return t
        return r

    def updateOutput(self, input):
        needs_grad = self.train and self._differentiable(input)
        if not needs_grad:
            self._ag = None
            with torch.no_grad():
                return self.fn(input)
        return super().updateOutput(input)

    @staticmethod
    def _differentiable(x):
        if isinstance(x, torch.Tensor):
            return x.is_floating_point()
        if isinstance(x, Table):
            return any(TFOp._differentiable(v) for _, v in x.items())
        return False

    def updateGradInput(self, input, gradOutput):
        if getattr(self, "_ag", None) is None:
            from .abstractnn import activity_apply
            return activity_apply(input, torch.zeros_like)
        return super().updateGradInput(input, gradOutput)

    def __repr__(self):
        return f"TFOp[{self.op}]"


def _named(op):
    def __init__(self, **attrs):
        TFOp.__init__(self, op, attrs)
    return type(op, (TFOp,), {"__init__": __init__, "__doc__": f"TF op ``{op}`` (see OPS)."})


# named constructors for the reference's ops / tf modules (nn/ops/*.scala, nn/tf/*.scala)
_NAMED = ["Gather", "OneHot", "StridedSlice", "Slice", "Tile", "Pad", "TopK", "InTopK", "SegmentSum", "BatchMatMul",
          "Dilation2D", "ResizeBilinear", "RandomUniform", "TruncatedNormal", "ArgMax", "Cast", "Rank", "Shape",
          "Equal", "NotEqual", "Greater", "GreaterEqual", "Less", "LessEqual", "LogicalAnd", "LogicalOr", "LogicalNot",
          "IsFinite", "IsInf", "IsNan", "Floor", "Ceil", "Round", "Rint", "Sign", "Inv", "Erf", "Erfc", "Lgamma",
          "Digamma", "Expm1", "FloorDiv", "FloorMod", "TruncateDiv", "SquaredDifference", "Maximum", "Minimum",
          "ApproximateEqual", "All", "Any", "Prod", "L2Loss", "BiasAdd", "Select", "Range", "Fill", "ExpandDims",
          "Squeeze", "Transpose", "Pack", "Unpack", "ConcatV2", "Split", "SplitV", "AddN", "NoOp", "Assert", "Mod",
          "Pow", "Rsqrt", "Reciprocal", "Softsign", "Softplus", "Relu6", "Elu"]
ops = type("ops", (), {n: _named(n) for n in _NAMED})      # ``tf_ops.ops.Gather(axis=...)``


class CrossEntropy(TFOp):
    """SoftmaxCrossEntropyWithLogits as a module (reference nn/ops/CrossEntropy.scala)."""

    def __init__(self):
        super().__init__("SoftmaxCrossEntropyWithLogits")


class DepthwiseConv2D(TFOp):
    def __init__(self, strideW=1, strideH=1, padW=0, padH=0, dataFormat="NHWC"):
        super().__init__("DepthwiseConv2dNative", {"strides": [1, strideH, strideW, 1] if dataFormat == "NHWC"
                                                   else [1, 1, strideH, strideW],
                                                   "padding": "SAME" if padW == -1 else "VALID",
                                                   "data_format": dataFormat})


__all__ = ["TFOp", "OPS", "run_op", "TF_DTYPES", "MULTI_OUTPUT", "ops", "CrossEntropy", "DepthwiseConv2D"]
