"""Model -> int8 model conversion.

Reference: S/nn/quantized/Quantizer.scala:28-133 (registry of quantizable classes; Container / Graph / Cell
walkers), Quantization.scala:168-180 (``quantize(model)`` clones first, then substitutes), Quantizable.scala,
AbstractModule.scala:920 (``model.quantize()``).

Beyond the reference's substitution, two inference rewrites are applied inside plain Sequential containers
(the int8 analogue of S/nn/mkldnn/Fusion.scala's conv+bn / conv+relu fusion):
  * ``fold_bn``: an evaluation-mode BatchNormalization that directly follows a convolution / Linear is
    folded into the float weights before they are quantized and removed from the container;
  * a ReLU that directly follows a quantized conv runs in the int8 kernel's epilogue.
"""
import torch

from ..nn.activation import ReLU
from ..nn.containers import Container, Sequential
from ..nn.conv import SpatialConvolution, SpatialDilatedConvolution, SpatialShareConvolution
from ..nn.graph import Graph
from ..nn.linear import Linear
from ..nn.normalization import BatchNormalization
from ..nn.recurrent import Cell
from .modules import QuantizedLinear, QuantizedSpatialConvolution, QuantizedSpatialDilatedConvolution


def _q_linear(m):
    q = QuantizedLinear(m.inputSize, m.outputSize, m.withBias)
    q.set_float_weights(m.weight.detach().float().cpu(), None if m.bias is None else m.bias.detach().float().cpu())
    return q.setName(m.getName())


def _q_conv(m):
    w = m.weight.detach().float().cpu()
    b = None if m.bias is None else m.bias.detach().float().cpu()
    if type(m) is SpatialDilatedConvolution:
        q = QuantizedSpatialDilatedConvolution(m.nInputPlane, m.nOutputPlane, m.kernelW, m.kernelH, m.strideW,
                                               m.strideH, m.padW, m.padH, m.dilationW, m.dilationH, format=m.format)
    else:
        q = QuantizedSpatialConvolution(m.nInputPlane, m.nOutputPlane, m.kernelW, m.kernelH, m.strideW, m.strideH,
                                        m.padW, m.padH, m.nGroup, format=m.format, dilationW=m.dilationW,
                                        dilationH=m.dilationH)
    q.fuse_relu = False
    return q.set_float_weights(w, b).setName(m.getName())


# registry keyed by exact class (reference registers exact class names, Quantizer.scala:68-75)
REGISTRY = {Linear: _q_linear, SpatialConvolution: _q_conv, SpatialShareConvolution: _q_conv,
            SpatialDilatedConvolution: _q_conv}


def register(cls, fn):
    """Register a quantizer for another module class (reference Quantizer.registerModule)."""
    if cls in REGISTRY:
        raise ValueError(f"Module: {cls.__name__} has been registered.")
    REGISTRY[cls] = fn


def _fold_bn_into(prev, bn):
    """Fold an eval-mode BN into the preceding conv / Linear float weights (in place)."""
    inv = torch.rsqrt(bn.runningVar.float().cpu() + bn.eps)
    gamma = bn.weight.detach().float().cpu() if bn.affine else torch.ones_like(inv)
    beta = bn.bias.detach().float().cpu() if bn.affine else torch.zeros_like(inv)
    s = gamma * inv
    w = prev.weight.detach().float().cpu()
    b = prev.bias.detach().float().cpu() if prev.bias is not None else torch.zeros(w.shape[0])
    dev = prev.weight.device
    with torch.no_grad():
        prev.weight.data = (w * s.reshape((-1,) + (1,) * (w.dim() - 1))).to(dev)
        newb = (b - bn.runningMean.float().cpu()) * s + beta
        if prev.bias is None:
            prev.bias = newb.to(dev)
        else:
            prev.bias.data = newb.to(dev)
    prev._w16 = {}


def _foldable(a, b):
    return (type(a) in (SpatialConvolution, SpatialShareConvolution, SpatialDilatedConvolution, Linear)
            and isinstance(b, BatchNormalization)
            and getattr(a, "nGroup", 1) == 1 and a.weight.shape[0] == b.nOutput and b.runningMean is not None)


def quantize_module(m, fold_bn=True):
    """Substitute quantizable layers inside ``m`` (in place where possible); returns the new module."""
    fn = REGISTRY.get(type(m))
    if fn is not None:
        q = fn(m)
        if getattr(m, "_calib_amax", None) is not None:
            q.inputAmax = m._calib_amax
        return q
    if isinstance(m, Graph):
        for n in m.order:
            new = quantize_module(n.element, fold_bn)
            if new is not n.element:
                n.element = new
        m.modules = [n.element for n in m.order]
        return m
    if isinstance(m, Cell):
        for name in ("cell", "preTopology"):
            sub = getattr(m, name, None)
            if sub is not None and sub is not m:
                setattr(m, name, quantize_module(sub, fold_bn))
        return m
    if isinstance(m, Container):
        mods = m.modules
        if fold_bn and type(m) is Sequential:
            i = 0
            while i < len(mods) - 1:
                if _foldable(mods[i], mods[i + 1]):
                    _fold_bn_into(mods[i], mods[i + 1])
                    del mods[i + 1]
                i += 1
        for i in range(len(mods)):
            mods[i] = quantize_module(mods[i], fold_bn)
        if type(m) is Sequential:
            for a, b in zip(mods[:-1], mods[1:]):
                if isinstance(a, QuantizedSpatialConvolution) and type(b) is ReLU:
                    a.fuse_relu = True
                    b.passthrough = True
            m._residual_plan = None
        return m
    return m


def calibrate(model, sample):
    """Record the abs-max of every quantizable layer's input over ``sample`` (reference MklInt8Convertible
    .calcScales with input mask 0: one per-tensor range per layer). The quantized layers then quantize their
    input with that fixed range instead of a per-sample abs-max pass."""
    layers = [m for m in model.flattened_layers() if type(m) in REGISTRY]
    saved = {}
    for m in layers:
        orig = m.updateOutput

        def hook(inp, _m=m, _orig=orig):
            a = float(inp.detach().abs().max()) if isinstance(inp, torch.Tensor) else None
            if a is not None:
                _m._calib_amax = max(a, getattr(_m, "_calib_amax", 0.0) or 0.0)
            return _orig(inp)
        saved[id(m)] = orig
        m.updateOutput = hook
    try:
        model.evaluate()
        with torch.no_grad():
            model.forward(sample)
    finally:
        for m in layers:
            del m.updateOutput
    return model


def quantize(model, fold_bn=True, calibration=None, plan=True):
    """Clone ``model`` and return its int8 inference version (reference Quantization.quantize).

    A Graph (e.g. a model imported from Caffe / TF) is first lowered through the engine-neutral IR so BatchNorm
    (and Caffe Scale) folds into the preceding convolution there too. ``calibration`` (a sample input batch)
    switches the activations to calibrated static ranges (see ``calibrate``); for a Graph on the GPU it also
    attaches the static int8 execution plan (``plan``; quantized/int8_graph.py)."""
    from ..utils.intermediate import BlasToIR, IRToDnn

    dev = getattr(model, "_device", None)
    cloned = model.cloneModule()
    if isinstance(cloned, Graph) and fold_bn:
        cloned = IRToDnn.fuse(BlasToIR.convert(cloned)).build("blas", train=False)
        if dev is not None:
            cloned.to(dev)            # rebuilt IR layers start on the CPU; kept general layers are on dev
    if calibration is not None:
        calibrate(cloned, calibration.to(dev if dev is not None else torch.device("cpu")))
    q = quantize_module(cloned, fold_bn)
    q.evaluate()
    if dev is not None and dev.type == "cuda":
        q.to(dev)
    if isinstance(q, Graph):
        IRToDnn.relu_plan(q)
        if plan and calibration is not None and dev is not None and dev.type == "cuda":
            # static int8 execution plan: int8 activations between layers, requantizing epilogues, in-place
            # concats, int8 pooling (quantized/int8_graph.py)
            from .int8_graph import plan_int8

            plan_int8(q, calibration.to(dev))
    return q
