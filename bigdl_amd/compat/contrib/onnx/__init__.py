"""Reference ``bigdl.contrib.onnx`` (P/contrib/onnx/onnx_loader.py, converter_utils.py) over the engine's ONNX
importer (``bigdl_amd.interop.onnx``, which decodes ModelProto itself: the ``onnx`` package is not needed).
``load_model_proto`` takes serialized bytes or any object with ``SerializeToString()`` (an ``onnx.ModelProto``)."""
import math

from ...nn.layer import Layer


def calc_output_shape(input, kernel, padding=0, stride=1, dilation=1, ceil_mode=False):
    """Pooling / convolution output extent (reference converter_utils.calc_output_shape)."""
    rounding = math.ceil if ceil_mode else math.floor
    return int(rounding((input + 2 * padding - dilation * (kernel - 1) - 1) / float(stride) + 1))


class OnnxLoader:
    def load_model(self, file_path):
        from ....interop.onnx import load_onnx

        return Layer.of(load_onnx(file_path))

    def load_model_proto(self, model_proto):
        from ....interop.onnx import load_onnx_bytes

        data = model_proto.SerializeToString() if hasattr(model_proto, "SerializeToString") else model_proto
        return Layer.of(load_onnx_bytes(data))


def load(model_path):
    return OnnxLoader().load_model(model_path)


def load_model_proto(model_proto):
    return OnnxLoader().load_model_proto(model_proto)


__all__ = ["OnnxLoader", "load", "load_model_proto", "calc_output_shape"]
