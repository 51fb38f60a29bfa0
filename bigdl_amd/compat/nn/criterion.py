"""``bigdl.nn.criterion`` for bigdl_amd (reference P/nn/criterion.py): every engine criterion under its reference
name with snake_case keywords and the ndarray ``forward(input, target) -> loss`` / ``backward -> gradInput`` API."""
import numpy as np

from ... import nn as _nn
from ...nn.abstractnn import AbstractCriterion
from .._convert import convert_kwargs, to_numpy, to_torch


class Criterion:
    _impl = None

    def __init__(self, *args, **kwargs):
        if "jvalue" in kwargs:
            self.value = kwargs["jvalue"]
        else:
            args = [getattr(a, "value", a) for a in args]
            args = [to_torch(a) if isinstance(a, np.ndarray) else a for a in args]
            kw = {k: getattr(v, "value", v) for k, v in kwargs.items()}
            self.value = self._impl(*args, **convert_kwargs(self._impl, kw))
        self.bigdl_type = "float"

    @classmethod
    def of(cls, crit):
        obj = object.__new__(_WRAPPERS.get(type(crit).__name__, Criterion))
        obj.value = crit
        obj.bigdl_type = "float"
        return obj

    def forward(self, input, target):
        return float(self.value.forward(to_torch(input), to_torch(target)))

    def backward(self, input, target):
        return to_numpy(self.value.backward(to_torch(input), to_torch(target)))

    def __str__(self):
        return str(self.value)


_WRAPPERS = {}
for _name in dir(_nn):
    _obj = getattr(_nn, _name)
    if isinstance(_obj, type) and issubclass(_obj, AbstractCriterion) and _name not in (
            "AbstractCriterion", "AutogradCriterion") and not _name.startswith("_"):
        _WRAPPERS[_name] = type(_name, (Criterion,), {"_impl": _obj})
        _WRAPPERS[_name].__module__ = __name__
        globals()[_name] = _WRAPPERS[_name]

__all__ = ["Criterion"] + sorted(_WRAPPERS)
