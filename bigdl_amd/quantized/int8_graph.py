"""Static int8 inference plan for a quantized nn.Graph on the GPU engine.

Reference: the MKL-DNN int8 inference path — S/nn/mkldnn/Fusion.scala:219-318 (int8 conv outputs requantized with
the next layer's calibrated scale, conv+sum / conv+relu fused in int8), S/nn/MklInt8Convertible.scala:53
(calibrated static per-tensor input / output scales), S/nn/mkldnn/JoinTable.scala:54 (concat branches write into
the consumer's memory), and the int8 pooling of the DNN engine.

Design (MI355X-first): activations that flow only between int8-capable layers stay int8 NHWC ``[N][H][W][Cp]``
(Cp = channels padded to 16, one 16-byte granule per MFMA lane) with one static scale per tensor. Every quantized
conv reads that buffer straight into LDS (csrc/quant.hip conv_i8_glds_kernel) and its epilogue dequantizes,
adds the bias, applies the ReLU and REQUANTIZES with the consumer tensor's scale — so no quantize pass, no amax
pass and no bf16 round trip remain between layers. Concats are one int8 buffer whose branches (convs, int8
pooling) write their channel slices in place. Max / average pooling run on int8 directly (same scale in and
out). The graph input is quantized once from fp32 NCHW; any consumer that cannot take int8 (softmax, a general
module, a graph output) gets a dequantized bf16 tensor.

Scales: a calibration batch is run through the quantized graph and the abs-max of every node output is recorded.
Tensors that must share a scale (a pool's input and output, a concat's inputs and output, pass-through ReLU /
dropout / flatten) form one class (union-find); the class scale is max |x| / 127 over its members.
"""
import os

import torch

from ..nn.activation import ReLU
from ..nn.dropout import Dropout
from ..nn.graph import Graph
from ..nn.pooling import SpatialAveragePooling, SpatialMaxPooling
from ..nn.table_ops import JoinTable
from ..ops import native
from ..ops.conv import _fwd_taps, out_size
from .modules import QuantizedLinear, QuantizedSpatialConvolution, quantize_act_gpu

BF16 = torch.bfloat16
CL = torch.channels_last


def _ceil16(c):
    return -(-c // 16) * 16


class I8Act:
    """An int8 activation: ``data`` int8 [N, H, W, Cp] (contiguous, pad channels zero), ``C`` real channels,
    ``scale`` (x = q * scale)."""

    __slots__ = ("data", "C", "scale")

    def __init__(self, data, C, scale):
        self.data, self.C, self.scale = data, C, scale

    @property
    def shape(self):
        N, H, W, _ = self.data.shape
        return (N, self.C, H, W)

    def dequantize(self):
        N, H, W, Cp = self.data.shape
        y = torch.empty((N, self.C, H, W), dtype=BF16, device=self.data.device, memory_format=CL)
        native.get().dequantize_rows(self.data, y, N * H * W, self.C, Cp, float(self.scale))
        return y


class I8Stem:
    """The graph input quantized straight into the width im2col of its only consumer, a small-channel stem conv
    (``quantize_wim2col_f32``): ``data`` int8 [N, H, OW, 32], ``x`` the fp32 input (for a float fallback)."""

    __slots__ = ("data", "x", "scale", "OW")

    def __init__(self, data, x, scale, OW):
        self.data, self.x, self.scale, self.OW = data, x, scale, OW

    @property
    def shape(self):
        return tuple(self.x.shape)


def _stem_ok(m):
    """A stem conv the width-im2col path takes: <= 4 input channels, <= 8 width taps, no width dilation."""
    import os

    return (os.environ.get("BIGDL_I8_STEM", "1") != "0" and _conv_ok(m) and m.nInputPlane <= 4
            and m.kernelW <= 8 and m.dilationW == 1 and m.dilationH == 1)


# BIGDL_I8_STEM_F32=0: quantize the image into the stem's width im2col first instead of inside the stem kernel
_STEM_F32 = os.environ.get("BIGDL_I8_STEM_F32", "1") != "0"


def _wim2col(x, OW, stem, pw, scale):
    N, _, H, _ = x.shape
    q = torch.empty((N, H, OW, 32), dtype=torch.int8, device=x.device)
    native.get().quantize_wim2col_f32(x, q, OW, stem.kernelW, stem.strideW, pw, float(scale))
    return q


def _stem_weight(m):
    """w'[k][r][e*4 + c] = w[k][r][e][c] (e < S, c < 4), cached on the module (its int8 weight does not change)."""
    w = m.weight
    key = (w.data_ptr(), w._version)
    c = getattr(m, "_i8_stem_w", None)
    if c is None or c[0] != key:
        K, R, S, _ = w.shape
        wp = torch.zeros(K, R, 8, 4, dtype=torch.int8, device=w.device)
        wp[:, :, :S, :] = w[..., :4]
        m._i8_stem_w = c = (key, wp.reshape(K, R * 32).contiguous())
    return c[1]


def _as_float(v):
    from ..utils.table import Table

    if isinstance(v, I8Act):
        return v.dequantize()
    if isinstance(v, I8Stem):
        return v.x
    if isinstance(v, Table):
        t = Table()
        for k, x in v.items():
            t[k] = _as_float(x)
        return t
    return v


class _UF:
    def __init__(self):
        self.p = {}

    def find(self, a):
        self.p.setdefault(a, a)
        while self.p[a] != a:
            self.p[a] = self.p[self.p[a]]
            a = self.p[a]
        return a

    def union(self, a, b):
        ra, rb = self.find(a), self.find(b)
        if ra != rb:
            self.p[ra] = rb


def _is_flatten(m):
    return type(m).__name__ in ("View", "Reshape", "InferReshape")


def _conv_ok(m):
    return isinstance(m, QuantizedSpatialConvolution) and m.nGroup == 1 and m.format == "NCHW"


def _pool_ok(m):
    if isinstance(m, SpatialMaxPooling):
        return m.format == "NCHW" and not (m.padW == -1 and m.padH == -1)
    if isinstance(m, SpatialAveragePooling):
        return m.format == "NCHW" and m.divide and not (m.padW == -1 and m.padH == -1)
    return False


def _pass_ok(m):
    return (isinstance(m, ReLU) and m.passthrough) or isinstance(m, Dropout) or type(m).__name__ == "Identity"


class Int8GraphPlan:
    """Builds and attaches the int8 runners of a quantized Graph (``node.fuse_run``)."""

    def __init__(self, g, calibration):
        self.g = g
        self.users = {}
        for n in g.order:
            for p in n.prevs:
                self.users.setdefault(p.id, []).append(n)
        self.amax = self._calibrate(calibration)
        self._find_residuals()
        self.int8 = {}
        self._classify()
        self._scales()
        self._attach()

    # ------------------------------------------------------------------ planning
    def _calibrate(self, x):
        for n in self.g.order:
            n.fuse_run = None
        with torch.no_grad():
            self.g.forward(x)
        amax = {}
        for nid, v in self.g._outs.items():
            if isinstance(v, torch.Tensor) and v.is_floating_point() and v.numel():
                amax[nid] = float(v.detach().abs().max())
        self.g._outs = {}
        return amax

    def _find_residuals(self):
        """CAddTable(conv, other) [-> ReLU] where the conv feeds only the add: the int8 conv epilogue adds the
        shortcut (int8, its own scale) and applies the ReLU (reference Fusion.scala conv + sum)."""
        self.res, self.res_conv, self.res_relu = {}, {}, {}
        for n in self.g.order:
            if not (type(n.element).__name__ == "CAddTable" and len(n.prevs) == 2
                    and all(k is None for k in n.prev_index)):
                continue
            for ci in (0, 1):
                c, o = n.prevs[ci], n.prevs[1 - ci]
                if c is o or not _conv_ok(c.element) or len(self.users.get(c.id, [])) != 1 or c.element.fuse_relu:
                    continue
                us = self.users.get(n.id, [])
                r = us[0] if (len(us) == 1 and isinstance(us[0].element, ReLU) and len(us[0].prevs) == 1) else None
                self.res[n.id] = (c, o, r, ci + 1)
                self.res_conv[c.id] = n.id
                if r is not None:
                    self.res_relu[r.id] = n.id
                break

    def _consumer_ok(self, n, c):
        m = c.element
        if any(k is not None for k in c.prev_index):
            return False
        if c.id in self.res:              # a planned residual add takes its conv and an int8 shortcut
            return True
        if c.id in self.res_relu:
            return True
        if _conv_ok(m) or _pool_ok(m) or _pass_ok(m):
            return len(c.prevs) == 1
        if isinstance(m, JoinTable):
            return True
        if _is_flatten(m):
            us = self.users.get(c.id, [])
            return bool(us) and all(isinstance(u.element, QuantizedLinear) for u in us)
        if isinstance(m, QuantizedLinear):
            return _is_flatten(n.element) or _pool_ok(n.element)
        return False

    def _classify(self):
        g = self.g
        outs = {o.id for o in g.output_nodes}
        for n in g.order:
            m = n.element
            if n.id in self.int8:          # set with its residual conv
                continue
            if n.id in self.res_conv:      # conv -> add [-> ReLU]: the block output decides for all three
                add = self.res_conv[n.id]
                c, o, r, _ = self.res[add]
                f = r if r is not None else [x for x in g.order if x.id == add][0]
                us = self.users.get(f.id, [])
                cap = f.id not in outs and bool(us) and all(self._consumer_ok(f, u) for u in us)
                for nid in (n.id, add) + ((r.id,) if r is not None else ()):
                    self.int8[nid] = cap
                continue
            us = self.users.get(n.id, [])
            if n.id in outs or not us or not all(self._consumer_ok(n, c) for c in us):
                self.int8[n.id] = False
                continue
            if n in g.inputs_nodes and not n.prevs:
                cap = True
            elif _conv_ok(m):
                cap = True
            elif (_pool_ok(m) or _pass_ok(m) or _is_flatten(m)) and len(n.prevs) == 1:
                cap = self.int8.get(n.prevs[0].id, False)
            elif isinstance(m, JoinTable):
                cap = any(self.int8.get(p.id, False) for p in n.prevs) and all(k is None for k in n.prev_index)
            else:
                cap = False
            self.int8[n.id] = cap

    def _scales(self):
        uf = _UF()
        for n in self.g.order:
            if not self.int8[n.id]:
                continue
            uf.find(n.id)
            m = n.element
            if n.id in self.res:
                c, o, r, _ = self.res[n.id]
                uf.union(n.id, c.id)
                if r is not None:
                    uf.union(r.id, n.id)
            elif n.id in self.res_relu:
                pass
            elif (_pool_ok(m) or _pass_ok(m) or _is_flatten(m)) and n.prevs:
                uf.union(n.id, n.prevs[0].id)
            elif isinstance(m, JoinTable):
                for p in n.prevs:
                    if self.int8.get(p.id, False):
                        uf.union(n.id, p.id)
        cls_amax = {}
        for nid, is8 in self.int8.items():
            if is8:
                r = uf.find(nid)
                cls_amax[r] = max(cls_amax.get(r, 0.0), self.amax.get(nid, 0.0))
        self.scale = {}
        for nid, is8 in self.int8.items():
            if is8:
                a = cls_amax[uf.find(nid)]
                self.scale[nid] = (a if a > 0 else 1.0) / 127.0

    # ------------------------------------------------------------------ runners
    def _attach(self):
        g = self.g
        self.join_of = {}          # producing node id -> (concat link, the concat input node it feeds)
        for n in g.order:
            if isinstance(n.element, JoinTable) and self.int8[n.id]:
                link = _I8Concat(self, n)
                for p in n.prevs:
                    self.join_of[p.id] = (link, p)
                    if isinstance(p.element, ReLU) and p.element.passthrough and len(p.prevs) == 1 \
                            and len(self.users.get(p.prevs[0].id, [])) == 1:
                        self.join_of[p.prevs[0].id] = (link, p)     # conv -> fused ReLU -> concat
        self.stash, self.fused = {}, {}
        extra = {}
        for add_id, (c, o, r, idx) in self.res.items():
            extra.setdefault(c.id, []).append(o)
        for n in g.order:
            m = n.element
            run = None
            n.fuse_pre = None
            if n.id in self.res_conv:
                o = self.res[self.res_conv[n.id]][1]
                n.fuse_pre = (lambda outs, x, _c=n.id, _o=o.id: self.stash.__setitem__(_c, outs[_o]))
            if n.id in self.res:
                run = self._add_runner(n)
            elif n.id in self.res_relu:
                run = self._res_relu_runner(n)
            elif n in g.inputs_nodes and not n.prevs:
                if self.int8[n.id]:
                    run = self._input_runner(n)
            elif _conv_ok(m):
                run = self._conv_runner(n)
            elif isinstance(m, QuantizedLinear):
                run = self._linear_runner(n)
            elif _pool_ok(m) and self.int8[n.id]:
                run = self._pool_runner(n)
            elif (_pass_ok(m) or _is_flatten(m)) and self.int8[n.id]:
                run = self._pass_runner(n)
            elif isinstance(m, JoinTable) and self.int8[n.id]:
                run = self.join_of_self(n)
            else:
                run = self._float_runner(n)
            n.fuse_run = run
        if extra:
            from ..nn.fusion import _topo_with_deps

            g.order = _topo_with_deps(g, extra)
            g.modules = [n.element for n in g.order]
        g._int8_plan = self

    def join_of_self(self, n):
        for link, _ in self.join_of.values():
            if link.node is n:
                return link.run_join
        raise RuntimeError("int8 plan: concat link missing")

    def _dest(self, n, N, H, W, C, dev):
        """Output buffer of node n's int8 result: its concat slice when one is planned, else a fresh buffer."""
        jl = self.join_of.get(n.id)
        if jl is not None:
            view = jl[0].slice_for(jl[1], N, H, W, C, dev)
            if view is not None:
                return view, True
        Cp = _ceil16(C)
        return _i8_buffer((N, H, W, Cp), C, dev), False

    def _input_runner(self, n):
        scale = self.scale[n.id]
        us = self.users.get(n.id, [])
        stem = us[0].element if len(us) == 1 and us[0].id not in self.res_conv and _stem_ok(us[0].element) else None

        def run(x):
            if not (isinstance(x, torch.Tensor) and x.is_cuda and x.dim() == 4 and x.dtype == torch.float32):
                return x
            x = x.contiguous()
            N, C, H, W = x.shape
            if stem is not None and C == stem.nInputPlane:
                ph, pw = stem._pads(H, W)
                OW = out_size(W, stem.kernelW, stem.strideW, pw, 1)
                if _STEM_F32 and C <= 3 and W == 224:
                    return I8Stem(None, x, scale, OW)     # quantized inside the stem kernel (or by stem_run)
                return I8Stem(_wim2col(x, OW, stem, pw, scale), x, scale, OW)
            q = _i8_buffer((N, H, W, _ceil16(C)), C, x.device)
            native.get().quantize_nchw_f32(x, q, _ceil16(C), float(scale))
            return I8Act(q, C, scale)
        return run

    def _residual_addend(self, n, N, OH, OW, K):
        """The int8 shortcut of a residual conv (quantized here when it arrived as a float tensor), or None."""
        a = self.stash.pop(n.id, None)
        add_id = self.res_conv[n.id]
        self.fused[add_id] = False
        if a is None or tuple(a.shape) != (N, K, OH, OW):
            return None
        if not isinstance(a, I8Act):
            if not (isinstance(a, torch.Tensor) and a.is_cuda and K % 8 == 0):
                return None
            o = self.res[add_id][1]
            sc = (self.amax.get(o.id, 0.0) or float(a.abs().max()) or 1.0) / 127.0
            q = _i8_buffer((N, OH, OW, _ceil16(K)), K, a.device)
            _quantize_into(a, q[..., :K], q.shape[3], sc)
            a = I8Act(q, K, sc)
        self.fused[add_id] = True
        return a

    def _add_runner(self, n):
        m = n.element
        idx = self.res[n.id][3]

        def run(x):
            if self.fused.get(n.id):
                return x[idx]
            return m.forward(_as_float(x))
        return run

    def _res_relu_runner(self, n):
        m = n.element
        add_id = self.res_relu[n.id]

        def run(x):
            if self.fused.get(add_id):
                return x
            return m.forward(_as_float(x))
        return run

    def _conv_runner(self, n):
        m = n.element
        out8 = self.int8[n.id]
        oscale = self.scale.get(n.id)
        residual = n.id in self.res_conv
        res_relu = residual and self.res[self.res_conv[n.id]][2] is not None

        def run(x):
            if isinstance(x, I8Stem):
                return stem_run(x)
            if not (isinstance(x, I8Act) or (isinstance(x, torch.Tensor) and x.is_cuda and x.dim() == 4)):
                return m.forward(_as_float(x))
            N, C, H, W = x.shape
            ph, pw = m._pads(H, W)
            R, S = m.kernelH, m.kernelW
            OH = out_size(H, R, m.strideH, ph, m.dilationH)
            OW = out_size(W, S, m.strideW, pw, m.dilationW)
            if isinstance(x, I8Act) and x.data.shape[3] == m.Cp:
                q, xs, xsc = x.data, None, float(x.scale)
            else:
                xf = _as_float(x)
                xn = xf.permute(0, 2, 3, 1)
                q, xs = quantize_act_gpu(xn.contiguous(), C, m.Cp, getattr(m, "inputAmax", None))
                xsc = 0.0
            K = m.nOutputPlane
            taps = _fwd_taps(R, S, ph, pw, m.dilationH, m.dilationW)
            geo = [N, H, W, m.Cp, OH, OW, m.strideH, m.strideW, R * S * m.Cp, K, K, OH, OW, 1, 1, 0, 0]
            add = self._residual_addend(n, N, OH, OW, K) if residual else None
            relu = m.fuse_relu or (add is not None and res_relu)
            ad, asc = (add.data, float(add.scale)) if add is not None else (None, 0.0)
            if out8 and (add is not None or not residual):
                dst, _ = self._dest(n, N, OH, OW, K, q.device)
                geo[10] = dst.stride(2)
                native.get().conv_i8(q, m.weight, dst, m.bias, xs, m.weightScale, geo, taps, relu, xsc,
                                     float(oscale), ad, asc)
                return I8Act(dst, K, oscale)
            y = torch.empty((N, K, OH, OW), dtype=BF16, device=q.device, memory_format=CL)
            native.get().conv_i8(q, m.weight, y, m.bias, xs, m.weightScale, geo, taps, relu, xsc, 0.0, ad, asc)
            return y

        def stem_run(x):
            # R x 1 convolution over the 32-byte width-im2col rows: height taps only, width stride 1
            N, C, H, W = x.shape
            ph, _ = m._pads(H, W)
            R, K = m.kernelH, m.nOutputPlane
            OH, OW = out_size(H, R, m.strideH, ph, 1), x.OW
            taps = _fwd_taps(R, 1, ph, 0, 1, 1)
            geo = [N, H, OW, 32, OH, OW, m.strideH, 1, R * 32, K, K, OH, OW, 1, 1, 0, 0]
            relu = m.fuse_relu
            wp = _stem_weight(m)
            dev = x.x.device
            if out8 and not residual:
                dst, _ = self._dest(n, N, OH, OW, K, dev)
                geo[10] = dst.stride(2)
                out_t, osc, ret = dst, float(oscale), I8Act(dst, K, oscale)
            else:
                out_t = torch.empty((N, K, OH, OW), dtype=BF16, device=dev, memory_format=CL)
                osc, ret = 0.0, out_t
            if x.data is None:
                # fp32 image straight into the stem kernel (the lanes quantize their own operands)
                if native.get().conv_i8_stem_f32(x.x, wp, out_t, m.bias, m.weightScale, geo, taps, relu,
                                                 float(x.scale), osc):
                    return ret
                _, pw = m._pads(H, W)
                x.data = _wim2col(x.x, OW, m, pw, x.scale)
            native.get().conv_i8(x.data, wp, out_t, m.bias, None, m.weightScale, geo, taps, relu, float(x.scale), osc,
                                 None, 0.0)
            return ret
        return run

    def _linear_runner(self, n):
        m = n.element

        def run(x):
            if isinstance(x, I8Act) and x.data.shape[1] == 1 and x.data.shape[2] == 1 and x.data.shape[3] == m.Kp \
                    and x.C == m.inputSize:
                B = x.data.shape[0]
                out = torch.empty(B, m.outputSize, dtype=torch.float32, device=x.data.device)
                geo = [B, 1, 1, m.Kp, 1, 1, 1, 1, m.Kp, m.outputSize, m.outputSize, 1, 1, 1, 1, 0, 0]
                native.get().conv_i8(x.data, m.weight, out, m.bias, None, m.weightScale, geo, [0, 0, 0], False,
                                     float(x.scale), 0.0)
                return out
            xf = _as_float(x)
            return m.forward(xf.reshape(xf.shape[0], -1) if xf.dim() > 2 else xf)
        return run

    def _pool_runner(self, n):
        m = n.element
        avg = isinstance(m, SpatialAveragePooling)

        def run(x):
            if not isinstance(x, I8Act):
                return m.forward(_as_float(x))
            N, C, H, W = x.shape
            if avg:
                kh, kw, sh, sw, ph, pw = m._geom(torch.empty((0, 0, H, W)))
                count_pad = m.countIncludePad
            else:
                kh, kw, sh, sw = m.kH, m.kW, m.dH, m.dW
                ph, pw = m._pads(H, W)
                count_pad = False
            OH = out_size(H, kh, sh, ph, 1, m.ceilMode)
            OW = out_size(W, kw, sw, pw, 1, m.ceilMode)
            dst, _ = self._dest(n, N, OH, OW, C, x.data.device)
            Cp = x.data.shape[3]
            native.get().pool_i8(x.data, dst, [N, H, W, Cp, OH, OW, kh, kw, sh, sw, ph, pw, dst.stride(2)], avg,
                                 bool(count_pad))
            return I8Act(dst, C, x.scale)
        return run

    def _pass_runner(self, n):
        m = n.element
        flatten = _is_flatten(m)

        def run(x):
            if isinstance(x, I8Act):
                if flatten and not (x.data.shape[1] == 1 and x.data.shape[2] == 1):
                    return m.forward(_as_float(x))
                return x
            return m.forward(x)
        return run

    def _float_runner(self, n):
        m = n.element

        def run(x):
            return m.forward(_as_float(x))
        return run


class _I8Concat:
    """An int8 concat: one [N][H][W][Cp_total] buffer; int8 producers (convs, pools) write their slices in place,
    other inputs are quantized / copied into theirs when the JoinTable node runs."""

    def __init__(self, plan, node):
        self.plan, self.node = plan, node
        self.buf = None

    def slice_for(self, producer, N, H, W, C, dev):
        """Channel slice of the concat buffer for concat input ``producer`` (allocating the buffer on first use),
        or None when the slice offset is not statically known / 16-aligned (the JoinTable then copies)."""
        prevs = self.node.prevs
        off = 0
        for p in prevs:
            if p is producer:
                break
            w = _static_width(p)
            if w is None:
                return None
            off += w
        if off % 16 != 0:
            return None
        if self.buf is None:
            total = 0
            for p in prevs:
                w = _static_width(p) if p is not producer else C
                if w is None:
                    return None
                total += w
            Cp = _ceil16(total)
            self.buf = _i8_buffer((N, H, W, Cp), total, dev)
            self.total = total
        b = self.buf
        if b.shape[0] != N or b.shape[1] != H or b.shape[2] != W:
            return None
        return b[..., off:off + C]

    def run_join(self, x):
        from ..utils.table import Table

        ts = x.toSeq() if isinstance(x, Table) else list(x)
        scale = self.plan.scale[self.node.id]
        buf, self.buf = self.buf, None
        N = ts[0].shape[0]
        H, W = ts[0].shape[2], ts[0].shape[3]
        total = sum(t.shape[1] for t in ts)
        if buf is None or buf.shape[3] != _ceil16(total):
            Cp = _ceil16(total)
            buf = _i8_buffer((N, H, W, Cp), total, _device_of(ts))
        off = 0
        for t in ts:
            C = t.shape[1]
            sl = buf[..., off:off + C]
            if isinstance(t, I8Act):
                if t.data.data_ptr() != sl.data_ptr():
                    if abs(t.scale - scale) <= 1e-12 * max(scale, 1e-30):
                        if sl.is_cuda:
                            native.get().copy_rows_i8(t.data, sl, N * H * W, C, t.data.stride(2), sl.stride(2))
                        else:
                            sl.copy_(t.data[..., :C])
                    else:        # a differently scaled int8 input: go through bf16 once
                        _quantize_into(t.dequantize(), sl, buf.shape[3], scale)
            else:
                _quantize_into(t, sl, buf.shape[3], scale)
            off += C
        return I8Act(buf, total, scale)


def _i8_buffer(shape, C, dev):
    """int8 NHWC buffer whose last dim is padded past C: the padding channels must read as zero (native byte fill,
    no aten kernel); unpadded buffers are left uninitialised."""
    buf = torch.empty(shape, dtype=torch.int8, device=dev)
    if shape[-1] != C and buf.is_cuda:
        native.get().fill_bytes(buf, 0)
    elif shape[-1] != C:
        buf.zero_()
    return buf


def _quantize_into(t, sl, ld, scale):
    t = t.to(BF16, memory_format=CL) if t.dtype != BF16 or not t.is_contiguous(memory_format=CL) else t
    N, C, H, W = t.shape
    if C % 8 == 0 and sl.storage_offset() % 8 == 0:
        native.get().quantize_rows_bf16(t, sl, N * H * W, C, ld, float(scale))
    else:
        sl.copy_(torch.clamp(torch.round(t.permute(0, 2, 3, 1).float() / scale), -127, 127).to(torch.int8))


def _static_width(p, depth=0):
    """Channel count of node p's output when it follows from the graph alone (conv widths, pass-through layers,
    pooling, concats of known widths), else None."""
    m = p.element
    if depth > 64:
        return None
    if isinstance(m, QuantizedSpatialConvolution):
        return m.nOutputPlane
    if (_pass_ok(m) or _pool_ok(m)) and len(p.prevs) == 1:
        return _static_width(p.prevs[0], depth + 1)
    if isinstance(m, JoinTable) and p.prevs:
        ws = [_static_width(q, depth + 1) for q in p.prevs]
        return None if any(w is None for w in ws) else sum(ws)
    return None


def _device_of(ts):
    for t in ts:
        if isinstance(t, I8Act):
            return t.data.device
        if isinstance(t, torch.Tensor):
            return t.device
    return torch.device("cuda")



def plan_int8(graph, calibration):
    """Attach an int8 execution plan to a quantized Graph on the GPU (see module docstring); returns the graph.
    ``calibration``: a representative input batch (on the graph's device)."""
    if not isinstance(graph, Graph):
        raise TypeError("plan_int8 needs an nn.Graph (quantize() lowers Graph models through the IR)")
    Int8GraphPlan(graph, calibration)
    return graph


def unplan_int8(graph):
    for n in graph.order:
        n.fuse_run = None
    graph._int8_plan = None
    return graph


__all__ = ["I8Act", "Int8GraphPlan", "plan_int8", "unplan_int8"]
