"""Reference ``bigdl.nn.keras.layer`` (P/nn/keras/layer.py): Keras-1.2.2-style layers with the reference's
snake_case keywords (``output_dim``, ``W_regularizer``, ``border_mode``, ``input_dim`` / ``input_shape``, ...)
over the engine's ``bigdl_amd.keras`` layers."""
import inspect

from .... import keras as _k
from ....keras.engine import KerasLayer as _EngineKerasLayer
from ....keras.engine import KerasModel as _EngineKerasModel
from ..._convert import convert_kwargs
from ..layer import Layer

_WRAPPERS = {}


class KerasLayer(Layer):
    """A reference Keras layer: ``value`` is the engine layer; ``input_dim=n`` means ``input_shape=(n,)``."""

    def __init__(self, *args, **kwargs):
        if "input_dim" in kwargs:
            kwargs["input_shape"] = (kwargs.pop("input_dim"),)
        if "jvalue" in kwargs:
            super().__init__(jvalue=kwargs["jvalue"])
            return
        super().__init__(jvalue=self._impl(*args, **convert_kwargs(self._impl, kwargs)))

    def get_input_shape(self):
        return self.value.getInputShape()

    def get_output_shape(self):
        return self.value.getOutputShape()


def _make(name, impl):
    cls = type(name, (KerasLayer,), {"_impl": impl, "__doc__": f"Reference ``bigdl.nn.keras.layer.{name}`` over "
                                                               f"the engine's ``bigdl_amd.keras.{name}``."})
    cls.__module__ = __name__
    return cls


for _name, _obj in inspect.getmembers(_k, inspect.isclass):
    if (issubclass(_obj, _EngineKerasLayer) and not issubclass(_obj, _EngineKerasModel)
            and not _name.startswith("_") and _name not in ("KerasLayer", "Input")):
        _WRAPPERS[_name] = _make(_name, _obj)
        globals()[_name] = _WRAPPERS[_name]

__all__ = ["KerasLayer"] + sorted(_WRAPPERS)
