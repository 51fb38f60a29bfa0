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
from ..nn.conv import SpatialConvolution, SpatialDilatedConvolution
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
REGISTRY = {Linear: _q_linear, SpatialConvolution: _q_conv, SpatialDilatedConvolution: _q_conv}


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
    return (type(a) in (SpatialConvolution, SpatialDilatedConvolution, Linear) and isinstance(b, BatchNormalization)
            and getattr(a, "nGroup", 1) == 1 and a.weight.shape[0] == b.nOutput and b.runningMean is not None)


def quantize_module(m, fold_bn=True):
    """Substitute quantizable layers inside ``m`` (in place where possible); returns the new module."""
    fn = REGISTRY.get(type(m))
    if fn is not None:
        return fn(m)
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


def quantize(model, fold_bn=True):
    """Clone ``model`` and return its int8 inference version (reference Quantization.quantize)."""
    dev = getattr(model, "_device", None)
    cloned = model.cloneModule()
    q = quantize_module(cloned, fold_bn)
    q.evaluate()
    if dev is not None and dev.type == "cuda":
        q.to(dev)
    return q
