"""Training / inference fusion planning for the GPU engine.

Reference analogue: the MKL-DNN engine's compile-time fusion (S/nn/mkldnn/Fusion.scala:32-332 — conv+bn,
conv+relu, bn+relu, conv+sum; S/nn/mkldnn/Sequential.scala:194-305), which the reference only applies to
inference graphs (DnnGraph.scala:396-409). Here fusion also applies to training, and it is an execution
plan only: the module tree, its parameters and its serialized form are untouched; fused modules just skip
work the producer already did.

  conv -> BN          conv epilogue emits per-channel (sum, sumsq): BN skips its statistics pass
  BN -> ReLU          ReLU applied in the BN apply pass; backward mask from the BN output
  conv/Linear -> ReLU ReLU in the GEMM epilogue
  BN -> ReLU -> conv  (default; BIGDL_DGRAD_BN=0 disables) backward: the conv's data-gradient epilogue reduces the BN's
                      backward statistics (sum dy, sum dy * (x - mean) under the ReLU mask): BN skips its
                      reduction pass
  ResNet block        Sequential[ConcatTable[branch(... BN), shortcut], CAddTable, ReLU]: the shortcut runs
                      first, its output is added inside the branch's last BN apply pass together with the
                      ReLU; backward emits the residual-branch gradient from the same pass.
"""
import os

import torch

from ..utils.table import Table
from .activation import ReLU
from .containers import ConcatTable, Sequential, add_activity
from .conv import SpatialConvolution
from .linear import Linear
from .normalization import BatchNormalization
from .table_ops import CAddTable


_TRAIN_NODE_ATTRS = ("res_src", "pass_index", "fold_fanout", "fold_bn")


def _reset(m):
    from .graph import Graph

    for x in [m] + list(m.flattened_layers()):
        if isinstance(x, Graph) and getattr(x, "_order0", None) is not None:
            x.order = x._order0
            x._order0 = None
        if isinstance(x, Graph):
            for n in x.order:
                for a in _TRAIN_NODE_ATTRS:
                    n.__dict__.pop(a, None)
        if isinstance(x, BatchNormalization):
            x._graph_dres = False
    for x in m.flattened_layers():
        for attr, val in (("emit_stats", False), ("fuse_relu", False), ("passthrough", False),
                          ("_dgrad_bn_ok", False), ("_defer_ok", False)):
            if hasattr(x, attr):
                setattr(x, attr, val)
        if isinstance(x, Sequential):
            x._residual_plan = None


def _dgrad_bn_enabled():
    """On by default since the statistics epilogue pairs its two waves' sums in LDS and spreads the atomics over
    128 slots: ResNet-50 b256 30.6 -> 30.2 ms/step (profiles/r2_dgrad_bn_ab.txt). With 32 slots and one atomic
    per wave it lost (+2.7 ms GEMM vs -2.4 ms reduction pass, profiles/r1_dgrad_bn_ab.txt)."""
    return os.environ.get("BIGDL_DGRAD_BN", "1") == "1"


def fuse_for_training(model):
    from .graph import DynamicGraph, Graph

    _reset(model)
    for m in model.flattened_layers():
        if isinstance(m, Sequential):
            _fuse_sequential(m)
        elif isinstance(m, Graph) and not isinstance(m, DynamicGraph) and not getattr(m, "_inference_fused", False):
            _fuse_graph_training(m)
    return model


def _fuse_graph_training(g):
    """Training fusion of an nn.Graph (ResNet.graph, Inception, Caffe / TF / ONNX imports): the pairwise plans of
    _fuse_sequential decided on the graph's edges instead of list neighbours — a producer is fused with its
    consumer only when that consumer is the producer's ONLY user and the producer is not a graph output
    (reference: the DnnGraph compile fuses any container, S/nn/mkldnn/DnnGraph.scala:310-409, Fusion.scala:60-217):
      conv -> BN            the conv epilogue emits the BN statistics
      BN -> ReLU            ReLU in the BN apply pass (and its mask in the BN backward); the ReLU passes through
      conv/Linear -> ReLU   ReLU in the GEMM epilogue
      BN -> ReLU -> conv    the conv's data-gradient epilogue reduces the BN's backward statistics (the conv is the
                            only user of the ReLU output, so its dgrad is that BN's complete output gradient)
    The ResNet block's residual plan (shortcut add inside the last BN pass) stays Sequential-only."""
    users = _graph_users(g)
    outs = {n.id for n in g.output_nodes}
    _plan_graph_residuals(g, users, outs)

    def only_user(n):
        us = users.get(n.id, [])
        ok = (len(us) == 1 and n.id not in outs and len(us[0].prevs) == 1 and us[0].prev_index[0] is None
              and not (n.element.hasName() and n.element.getName() in g._stop_grad))
        return us[0] if ok else None

    for n in g.order:
        m, u = n.element, only_user(n)
        if u is None:
            continue
        c = u.element
        if isinstance(m, SpatialConvolution) and isinstance(c, BatchNormalization) and m.nGroup == 1:
            m.emit_stats = True
        elif isinstance(m, BatchNormalization) and isinstance(c, ReLU):
            m.fuse_relu = True
            c.passthrough = True
        elif isinstance(m, (SpatialConvolution, Linear)) and isinstance(c, ReLU):
            m.fuse_relu = True
            c.passthrough = True
    _plan_fanout_folds(g, users)
    for n in g.order:
        m, u = n.element, only_user(n)
        if isinstance(m, BatchNormalization) and u is not None and isinstance(u.element, ReLU):
            v = only_user(u)
            if v is not None:
                _plan_deferred_bn(m, u.element, v.element)
    if not _dgrad_bn_enabled():
        return
    for n in g.order:
        m, u = n.element, only_user(n)
        if not (isinstance(m, BatchNormalization) and m.fuse_relu and u is not None and isinstance(u.element, ReLU)
                and u.element.passthrough):
            continue
        v = only_user(u)
        if v is not None and isinstance(v.element, SpatialConvolution) and v.element.nGroup == 1:
            v.element._dgrad_bn_ok = True


def _stopped(g, n):
    return n.element.hasName() and n.element.getName() in g._stop_grad


def _plan_graph_residuals(g, users, outs):
    """BN -> CAddTable(BN, shortcut) -> ReLU: the BN adds the shortcut and applies the ReLU in its apply pass and
    returns the shortcut's (masked) gradient from its backward pass; the add passes its BN input on and the ReLU
    passes through — the Graph form of the Sequential residual plan (reference ResNet.graph, models/resnet)."""
    for a in list(g.order):
        if not isinstance(a.element, CAddTable) or len(a.prevs) != 2 or any(k is not None for k in a.prev_index):
            continue
        ua = users.get(a.id, [])
        if (len(ua) != 1 or a.id in outs or _stopped(g, a) or not isinstance(ua[0].element, ReLU)
                or len(ua[0].prevs) != 1 or ua[0].prev_index[0] is not None):
            continue
        for ib in (0, 1):
            b, sc = a.prevs[ib], a.prevs[1 - ib]
            bn = b.element
            if (b is sc or not isinstance(bn, BatchNormalization) or users.get(b.id) != [a] or b.id in outs
                    or _stopped(g, b) or bn.fuse_relu or bn.nOutput % 8 != 0 or getattr(b, "res_src", None)):
                continue
            order = g.order
            if order.index(sc) > order.index(b):
                # the shortcut must exist when the BN runs: move the BN right after it (its only consumer is
                # the add, which follows both)
                if getattr(g, "_order0", None) is None:
                    g._order0 = list(order)
                order.remove(b)
                order.insert(order.index(sc) + 1, b)
            bn.fuse_relu = True
            bn._graph_dres = True
            b.res_src = sc
            a.pass_index = ib + 1
            ua[0].element.passthrough = True
            break


def _plan_fanout_folds(g, users):
    """A tensor read by several nodes: the consumer processed LAST in backward (first in forward order) is a conv
    whose data-gradient epilogue adds the other consumers' summed gradient (the residual_backward fold of the
    Sequential plan, for any fan-out)."""
    pos = {n.id: i for i, n in enumerate(g.order)}
    contrib = {}
    for n in g.order:
        rs = getattr(n, "res_src", None)
        if rs is not None:
            contrib.setdefault(rs.id, []).append(n)
    for p in g.order:
        us = [u for u in users.get(p.id, []) if getattr(u, "pass_index", None) is None]
        srcs = us + contrib.get(p.id, [])
        if len(srcs) < 2:
            continue
        c = min(srcs, key=lambda u: pos[u.id])
        cv = c.element
        if (c not in us or len(c.prevs) != 1 or c.prev_index[0] is not None or _stopped(g, c)
                or not isinstance(cv, SpatialConvolution) or cv.nGroup != 1 or not cv.propagateBack
                or cv.format != "NCHW" or cv.nInputPlane % 8 != 0):
            continue
        c.fold_fanout = True
        c.fold_bn = _dgrad_bn_enabled()


def unfuse(model):
    _reset(model)
    return model


def _last_leaf(m):
    while isinstance(m, Sequential) and m.modules and m._residual_plan is None:
        m = m.modules[-1]
    return m


def _fuse_sequential(seq):
    mods = seq.modules
    # residual block pattern first
    if (len(mods) == 3 and isinstance(mods[0], ConcatTable) and len(mods[0].modules) == 2
            and isinstance(mods[1], CAddTable) and isinstance(mods[2], ReLU)):
        branch, short = mods[0].modules
        if isinstance(branch, Sequential) and branch.modules and isinstance(branch.modules[-1], BatchNormalization):
            bn = branch.modules[-1]
            if bn.nOutput % 8 == 0:
                bn.fuse_relu = True
                seq._residual_plan = (branch, short, bn)
    for a, b in zip(mods[:-1], mods[1:]):
        if isinstance(a, SpatialConvolution) and isinstance(b, BatchNormalization) and a.nGroup == 1:
            a.emit_stats = True
        elif isinstance(a, BatchNormalization) and isinstance(b, ReLU):
            a.fuse_relu = True
            b.passthrough = True
    # BN -> ReLU -> conv: the conv is the only consumer of the BN output, so its data-gradient GEMM
    # produces the BN's complete output gradient and can reduce the BN backward statistics in its epilogue
    for a, b, c in zip(mods[:-2], mods[1:-1], mods[2:]):
        if (_dgrad_bn_enabled() and isinstance(a, BatchNormalization) and a.fuse_relu and isinstance(b, ReLU) and b.passthrough
                and isinstance(c, SpatialConvolution) and c.nGroup == 1):
            c._dgrad_bn_ok = True
        elif isinstance(a, (SpatialConvolution, Linear)) and isinstance(b, ReLU):
            a.fuse_relu = True
            b.passthrough = True
    for a, b, c in zip(mods[:-2], mods[1:-1], mods[2:]):
        _plan_deferred_bn(a, b, c)


# Which consumers take a deferred BN + ReLU output (BIGDL_BN_DEFER): 1 (default) = the 3x3/2 max pool only (it
# applies it on load at no cost; the ResNet stem BN loses its 411 MB apply pass); 2 = also 3x3 / stride-1 convs (halo
# forward + halo weight gradient apply it on load); 0 = none. Level 2 is correct (tests/test_bn_defer_gpu.py) but
# slower on ResNet-50: the on-load transform costs the latency-bound halo kernels more than the HBM-rate apply pass
# it removes (+0.13 ms fwd, +0.42 ms weight gradients vs -0.38 ms of apply passes: profiles/r6_iteration_log.txt)
DEFER_LEVEL = [int(os.environ.get("BIGDL_BN_DEFER", "1") or 0)]


def _defer_consumer(c):
    """Modules that take a deferred BN + ReLU output (ops/bn.py deferred) and apply it on load in every pass that
    reads it: the 3x3/2 max pool, and (level 2) 3x3 / stride-1 convolutions (halo forward and halo weight gradient;
    other shapes get it materialised by the binding). A 1x1 consumer is never deferred: its weight gradient would have
    to materialise the BN output on the side stream, which moves the apply pass instead of removing it."""
    from .pooling import SpatialMaxPooling

    if isinstance(c, SpatialConvolution):        # (subclasses that keep the base forward / weight gradient)
        if DEFER_LEVEL[0] < 2:
            return False
        return (c.nGroup == 1 and c.format == "NCHW" and type(c).updateOutput is SpatialConvolution.updateOutput
                and type(c)._wgrad_gpu is SpatialConvolution._wgrad_gpu and c.kernelW == 3 and c.kernelH == 3
                and c.strideW == 1 and c.strideH == 1 and c.dilationW == 1 and c.dilationH == 1)
    return DEFER_LEVEL[0] >= 1 and type(c) is SpatialMaxPooling and c.format == "NCHW"


def _plan_deferred_bn(a, b, c):
    """BN(+ReLU fused) -> ReLU(pass-through) -> conv / max pool, where the consumer is the ReLU output's only reader:
    the BN skips its apply pass and hands on a deferred output (csrc/kernels.h ConvArgs::pre). Reference analogue:
    the MKL-DNN fused BN + ReLU feeding the next primitive's input (S/nn/mkldnn/Fusion.scala:60-217)."""
    if (isinstance(a, BatchNormalization) and a.fuse_relu and not getattr(a, "_graph_dres", False)
            and isinstance(b, ReLU) and b.passthrough and _defer_consumer(c)):
        a._defer_ok = True


def residual_forward(seq, x):
    branch, short, bn = seq._residual_plan
    concat, add, relu = seq.modules
    res = short.forward(x)
    h = x
    for m in branch.modules[:-1]:
        h = m.forward(h)
    if tuple(res.shape) != tuple(h.shape[:1]) + (bn.nOutput,) + tuple(h.shape[2:]):
        raise ValueError(f"residual block: shortcut output {tuple(res.shape)} does not match the branch output")
    out = bn.updateOutput(h, residual=res)
    bn.output = out
    branch.output = out
    concat.output = Table(out, res)
    add.output = out
    relu.output = out
    seq._res_h = h
    return out


# on by default since the streaming 1x1 kernel loads its mask bytes without a branch (ResNet-50 22.91 -> 22.76 ms,
# profiles/r5_iteration_log.txt; before that the byte loads cost the epilogue what bn_bwd_apply saved);
# BIGDL_MASKED_ADDEND=0 materialises the residual gradient instead
MASKED_ADDEND = [os.environ.get("BIGDL_MASKED_ADDEND", "1") != "0"]


# BIGDL_SHORTCUT_BN_RED=0: the projection shortcut BN's backward reduction runs as its own pass
SHORTCUT_BN_RED = [os.environ.get("BIGDL_SHORTCUT_BN_RED", "1") != "0"]


def _native_det():
    from ..ops import native

    return native.deterministic()


def residual_backward(seq, x, gradOutput):
    branch, short, bn = seq._residual_plan
    mods = branch.modules
    first = mods[0]
    can_fold = (isinstance(first, SpatialConvolution) and first.propagateBack and first.nGroup == 1
                and first.format == "NCHW" and first.nInputPlane % 8 == 0)
    # identity shortcut: its gradient dres = dz * (y > 0) is never materialised; the block's output gradient and the
    # BN's sign mask go to the first dgrad GEMM, whose epilogue adds dz where the mask bit is set (one bf16 write
    # pass less per block: csrc/kernels.h ConvArgs::addzm)
    masked = None
    zm = getattr(bn, "_zm", None)
    if (MASKED_ADDEND[0] and can_fold and zm is not None and type(short).__name__ == "Identity" and first.strideH == 1
            and first.strideW == 1 and torch.is_tensor(gradOutput) and gradOutput.is_cuda
            and tuple(gradOutput.shape) == tuple(x.shape) and x.dtype == torch.bfloat16):
        dh, _ = bn.backward_fused(seq._res_h, gradOutput, need_dres=False)
        gz = gradOutput
        if gz.dtype != torch.bfloat16 or not gz.is_contiguous(memory_format=torch.channels_last):
            gz = gz.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        masked = (gz, zm)
        gs = None
    else:
        # projection shortcut ending in a training BN without ReLU: dres is that BN's output gradient, so its
        # backward reduction rides along in the pass that writes dres (csrc/batchnorm.hip bn_bwd_apply_kernel R2)
        sec, sbn = None, None
        if SHORTCUT_BN_RED[0] and isinstance(short, Sequential) and short.modules:
            sbn = short.modules[-1]
            xs = getattr(sbn, "_xin", None)
            xb = getattr(bn, "_xin", None)
            if (isinstance(sbn, BatchNormalization) and sbn.train and not sbn.fuse_relu and xs is not None
                    and xb is not None and xs.is_cuda and xs.shape == xb.shape and xs.stride() == xb.stride()
                    and xs.dtype == torch.bfloat16 and xs.shape[1] % 8 == 0 and not _native_det()):
                from ..ops import bn as bnops

                sec = (xs, sbn.saveMean, bnops.new_stats(xs.shape[1], xs.device))
        dh, dres = bn.backward_fused(seq._res_h, gradOutput, need_dres=True, sec=sec)
        if sec is not None:
            dres._bn_red = (sbn, sec[2])
        # shortcut first, so its gradient can be summed inside the epilogue of the branch's first dgrad GEMM
        gs = short.backward(x, dres)
    bn.gradInput = dh
    fold = masked is not None or (can_fold and gs is not None and gs.dtype == x.dtype and gs.shape == x.shape)
    g = dh
    for i in range(len(mods) - 2, -1, -1):
        inp = mods[i - 1].output if i > 0 else x
        if i == 0 and fold:
            first._dgrad_addend = masked if masked is not None else gs
            # with the shortcut gradient folded in, the dgrad output is the complete gradient of the block
            # input: if that is the previous block's output, its last BN's reduction can run in the epilogue
            first._dgrad_bn_once = _dgrad_bn_enabled()
        g = mods[i].backward(inp, g)
    return g if fold else add_activity(g, gs)


# ---------------------------------------------------------------------------------------------------------------
# Graph-form inference fusion (nn.Graph on the GPU engine: models imported from Caffe / TF / ONNX and every model
# lowered through the IR by ConversionUtils.convert(model, "dnn")). Reference: the MKL-DNN graph compile
# (S/nn/mkldnn/DnnGraph.scala:396-409 fusion at compile, Fusion.scala:60-217 conv+relu / conv+sum,
# JoinTable.scala:54 concat into the consumer's memory). Flags that depend on run-time shapes are decided in
# per-node hooks that nn.Graph.updateOutput calls right before the node runs (``node.fuse_pre``).
# ---------------------------------------------------------------------------------------------------------------
def _graph_users(g):
    users = {}
    for n in g.order:
        for p in n.prevs:
            users.setdefault(p.id, []).append(n)
    return users


def _conv_fusable(n):
    m = n.element
    return (type(m).__name__ in ("SpatialConvolution", "SpatialShareConvolution", "SpatialDilatedConvolution")
            and isinstance(m, SpatialConvolution) and m.nGroup == 1 and m.format == "NCHW")


def _conv_out_shape(conv, x):
    from ..ops.conv import out_size

    N, _, H, W = x.shape
    ph, pw = conv._pads(H, W)
    return (N, conv.nOutputPlane, out_size(H, conv.kernelH, conv.strideH, ph, conv.dilationH),
            out_size(W, conv.kernelW, conv.strideW, pw, conv.dilationW))


def _topo_with_deps(g, extra):
    """Topological order of ``g`` where node ``k`` also waits for every node in ``extra[k.id]`` (iterative DFS)."""
    order, state = [], {}
    for root in list(g.output_nodes) + list(g.inputs_nodes):
        stack = [(root, False)]
        while stack:
            n, done = stack.pop()
            if done:
                if state.get(n.id) != 2:
                    state[n.id] = 2
                    order.append(n)
                continue
            st = state.get(n.id)
            if st == 2:
                continue
            if st == 1:
                raise ValueError("inference fusion created a cycle")
            state[n.id] = 1
            stack.append((n, True))
            for p in reversed(list(n.prevs) + extra.get(n.id, [])):
                if state.get(p.id) != 2:
                    if state.get(p.id) == 1:
                        raise ValueError("inference fusion created a cycle")
                    stack.append((p, False))
    return order


class _ResidualLink:
    """conv -> CAddTable(conv, other) [-> ReLU]: the add (and ReLU) run in the conv's epilogue when ``other`` is
    a dense bf16 NHWC tensor of the conv's output shape; otherwise every node runs unfused."""

    def __init__(self, conv, other_id, add, idx, relu):
        self.conv, self.other_id, self.add, self.idx, self.relu = conv, other_id, add, idx, relu
        self.used = False

    def pre_conv(self, outs, x):
        import torch

        a = outs[self.other_id]
        self.used = (isinstance(a, torch.Tensor) and x.is_cuda and a.dtype == torch.bfloat16 and a.dim() == 4
                     and a.is_contiguous(memory_format=torch.channels_last)
                     and tuple(a.shape) == _conv_out_shape(self.conv, x))
        self.conv._fuse_addend = a if self.used else None
        self.conv.fuse_relu = self.used and self.relu is not None

    def pre_add(self, outs, x):
        self.add.passthrough = self.used
        self.add._pass_index = self.idx

    def pre_relu(self, outs, x):
        self.relu.passthrough = self.used


class _ConcatLink:
    """JoinTable over channels whose conv producers write their channel slice of one NHWC buffer. Widths of the
    non-producer inputs are read at run time (they are scheduled before the first producer)."""

    def __init__(self, join, prevs, producer_convs):
        self.join, self.prevs, self.conv_of = join, prevs, producer_convs   # conv_of: prev id -> conv module
        self.buf = None

    def _width(self, p, outs):
        c = self.conv_of.get(p.id)
        return c.nOutputPlane if c is not None else outs[p.id].shape[1]

    def pre_conv(self, pid, outs, x):
        import torch

        conv = self.conv_of[pid]
        if not x.is_cuda:
            return
        N, K, OH, OW = _conv_out_shape(conv, x)
        off = 0
        for p in self.prevs:
            if p.id == pid:
                break
            off += self._width(p, outs)
        if self.buf is None:
            ctot = sum(self._width(p, outs) for p in self.prevs)
            self.buf = torch.empty((N, ctot, OH, OW), dtype=torch.bfloat16, device=x.device,
                                   memory_format=torch.channels_last)
        b = self.buf
        if off % 8 == 0 and b.shape[0] == N and b.shape[2] == OH and b.shape[3] == OW:
            conv._fuse_out = b[:, off:off + K]

    def pre_join(self, outs, x):
        self.join._fuse_buf, self.buf = self.buf, None


def _chain(hooks):
    def run(outs, x):
        for h in hooks:
            h(outs, x)
    return run


def fuse_graph_for_inference(g):
    """Compile-time inference fusion of an nn.Graph for the GPU engine:

      ReLU      a ReLU whose only producer is a conv / Linear / BN that feeds nothing else runs in its epilogue
      residual  CAddTable(conv, other) [-> ReLU]: the conv (single consumer) adds ``other`` in its epilogue and
                applies the ReLU; the add and the ReLU pass through. ``other`` is scheduled before the conv.
      concat    JoinTable over channels: convs (through a fused ReLU) that feed only the JoinTable write their
                channel slice of the concat buffer; the JoinTable copies only its other inputs, which are
                scheduled before the first producer conv so the buffer's width is known.
    Inference only: the graph's backward is not valid after this pass (``unfuse_graph`` resets it).
    """
    from ..quantized.modules import QuantizedSpatialConvolution
    from .table_ops import JoinTable
    from .shape_ops import _bdim
    import torch

    unfuse_graph(g)
    users = _graph_users(g)
    single = lambda n: len(users.get(n.id, [])) == 1  # noqa: E731
    # ReLU into producer epilogues
    for n in g.order:
        if isinstance(n.element, ReLU) and len(n.prevs) == 1:
            p = n.prevs[0]
            if isinstance(p.element, (SpatialConvolution, Linear, BatchNormalization, QuantizedSpatialConvolution)) \
                    and hasattr(p.element, "fuse_relu") and single(p):
                p.element.fuse_relu = True
                n.element.passthrough = True
    hooks, extra = {}, {}
    res_convs = set()
    # residual adds into the conv epilogue
    for n in g.order:
        m = n.element
        if not (isinstance(m, CAddTable) and len(n.prevs) == 2 and all(k is None for k in n.prev_index)):
            continue
        for ci in (0, 1):
            c, o = n.prevs[ci], n.prevs[1 - ci]
            if c is o or not _conv_fusable(c) or not single(c) or c.element.fuse_relu:
                continue
            us = users.get(n.id, [])
            relu_n = us[0] if (len(us) == 1 and isinstance(us[0].element, ReLU) and len(us[0].prevs) == 1) else None
            link = _ResidualLink(c.element, o.id, m, ci + 1, relu_n.element if relu_n is not None else None)
            hooks.setdefault(c.id, []).append(link.pre_conv)
            hooks.setdefault(n.id, []).append(link.pre_add)
            if relu_n is not None:
                hooks.setdefault(relu_n.id, []).append(link.pre_relu)
            extra.setdefault(c.id, []).append(o)
            res_convs.add(c.id)
            break
    # concat written in place by its producer convs
    for n in g.order:
        m = n.element
        if not (isinstance(m, JoinTable) and len(n.prevs) >= 2 and all(k is None for k in n.prev_index)):
            continue
        if _bdim(m.dimension, torch.empty((0, 0, 0, 0)), m.nInputDims if m.nInputDims > 0 else None) != 1:
            continue
        if len({p.id for p in n.prevs}) != len(n.prevs):
            continue
        conv_of, conv_node, dyn = {}, {}, []
        for p in n.prevs:
            c = p
            if isinstance(p.element, ReLU) and p.element.passthrough and len(p.prevs) == 1 and single(p):
                c = p.prevs[0]
            if (_conv_fusable(c) and single(c) and c.id not in res_convs and single(p)
                    and c.element.nOutputPlane % 8 == 0):
                conv_of[p.id] = c.element
                conv_node[p.id] = c
            else:
                dyn.append(p)
        if not conv_of:
            continue
        link = _ConcatLink(m, list(n.prevs), conv_of)
        for pid, c in conv_node.items():
            hooks.setdefault(c.id, []).append(lambda outs, x, _p=pid, _l=link: _l.pre_conv(_p, outs, x))
            extra.setdefault(c.id, []).extend(dyn)
        hooks.setdefault(n.id, []).append(link.pre_join)
    for n in g.order:
        hs = hooks.get(n.id)
        n.fuse_pre = _chain(hs) if hs else None
    if extra:
        g.order = _topo_with_deps(g, extra)
        g.modules = [n.element for n in g.order]
    g._inference_fused = True
    return g


def unfuse_graph(g):
    """Undo fuse_graph_for_inference / relu planning on an nn.Graph (flags, hooks)."""
    for n in g.order:
        n.fuse_pre = None
        m = n.element
        for attr, val in (("fuse_relu", False), ("passthrough", False), ("_fuse_out", None),
                          ("_fuse_addend", None), ("_fuse_buf", None)):
            if hasattr(m, attr):
                setattr(m, attr, val)
    g._inference_fused = False
    return g
