"""Training / inference fusion planning for the GPU engine.

Reference analogue: the MKL-DNN engine's compile-time fusion (S/nn/mkldnn/Fusion.scala:32-332 — conv+bn,
conv+relu, bn+relu, conv+sum; S/nn/mkldnn/Sequential.scala:194-305), which the reference only applies to
inference graphs (DnnGraph.scala:396-409). Here fusion also applies to training, and it is an execution
plan only: the module tree, its parameters and its serialized form are untouched; fused modules just skip
work the producer already did.

  conv -> BN          conv epilogue emits per-channel (sum, sumsq): BN skips its statistics pass
  BN -> ReLU          ReLU applied in the BN apply pass; backward mask from the BN output
  conv/Linear -> ReLU ReLU in the GEMM epilogue
  BN -> ReLU -> conv  (opt-in, BIGDL_DGRAD_BN=1) backward: the conv's data-gradient epilogue reduces the BN's
                      backward statistics (sum dy, sum dy * (x - mean) under the ReLU mask): BN skips its
                      reduction pass
  ResNet block        Sequential[ConcatTable[branch(... BN), shortcut], CAddTable, ReLU]: the shortcut runs
                      first, its output is added inside the branch's last BN apply pass together with the
                      ReLU; backward emits the residual-branch gradient from the same pass.
"""
import os

from ..utils.table import Table
from .activation import ReLU
from .containers import ConcatTable, Sequential, add_activity
from .conv import SpatialConvolution
from .linear import Linear
from .normalization import BatchNormalization
from .table_ops import CAddTable


def _reset(m):
    for x in m.flattened_layers():
        for attr, val in (("emit_stats", False), ("fuse_relu", False), ("passthrough", False),
                          ("_dgrad_bn_ok", False)):
            if hasattr(x, attr):
                setattr(x, attr, val)
        if isinstance(x, Sequential):
            x._residual_plan = None


def _dgrad_bn_enabled():
    """Off by default: measured on ResNet-50 b256 (profiles/r1_dgrad_bn_ab.txt) the extra x / z reads in the
    dgrad epilogue cost the GEMM +2.7 ms/step while the skipped reduction pass saved 2.4 ms — the epilogue
    runs at 2 workgroups per CU with nothing to overlap its reads, the separate pass streams at full bandwidth."""
    return os.environ.get("BIGDL_DGRAD_BN", "0") == "1"


def fuse_for_training(model):
    _reset(model)
    for m in model.flattened_layers():
        if isinstance(m, Sequential):
            _fuse_sequential(m)
    return model


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


def residual_backward(seq, x, gradOutput):
    branch, short, bn = seq._residual_plan
    dh, dres = bn.backward_fused(seq._res_h, gradOutput, need_dres=True)
    bn.gradInput = dh
    # shortcut first, so its gradient can be summed inside the epilogue of the branch's first dgrad GEMM
    gs = short.backward(x, dres)
    mods = branch.modules
    first = mods[0]
    fold = (isinstance(first, SpatialConvolution) and first.propagateBack and first.nGroup == 1
            and first.format == "NCHW" and first.nInputPlane % 8 == 0 and gs is not None
            and gs.dtype == x.dtype and gs.shape == x.shape)
    g = dh
    for i in range(len(mods) - 2, -1, -1):
        inp = mods[i - 1].output if i > 0 else x
        if i == 0 and fold:
            first._dgrad_addend = gs
            # with the shortcut gradient folded in, the dgrad output is the complete gradient of the block
            # input: if that is the previous block's output, its last BN's reduction can run in the epilogue
            first._dgrad_bn_once = _dgrad_bn_enabled()
        g = mods[i].backward(inp, g)
    return g if fold else add_activity(g, gs)
