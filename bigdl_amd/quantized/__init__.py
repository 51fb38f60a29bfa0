"""Int8 inference (reference S/nn/quantized/*): ``model.quantize()`` / ``quantize(model)``."""
from .modules import (QuantizedLinear, QuantizedModule, QuantizedSpatialConvolution,
                      QuantizedSpatialDilatedConvolution, quantization_loss, quantize_per_sample_ref, quantize_rows)
from .quantizer import REGISTRY, quantize, quantize_module, register

__all__ = ["QuantizedModule", "QuantizedLinear", "QuantizedSpatialConvolution", "QuantizedSpatialDilatedConvolution",
           "quantize", "quantize_module", "register", "REGISTRY", "quantize_rows", "quantize_per_sample_ref",
           "quantization_loss"]
