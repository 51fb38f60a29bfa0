"""Reference ``bigdl.nn.initialization_method`` (P/nn/initialization_method.py) over ``bigdl_amd.nn.init_methods``:
the same class names and constructor signatures (``bigdl_type`` accepted and ignored; note the reference's
``RandomUniform(upper, lower)`` argument order). Instances are the engine's initialisation methods, so they go
straight into ``Layer.set_init_method`` / ``setInitMethod``."""
from ...nn import init_methods as _im

InitializationMethod = _im.InitializationMethod


class Zeros(_im.Zeros):
    def __init__(self, bigdl_type="float"):
        super().__init__()


class Ones(_im.Ones):
    def __init__(self, bigdl_type="float"):
        super().__init__()


class RandomUniform(_im.RandomUniform):
    """U(lower, upper); without bounds U(-1/sqrt(fanIn), 1/sqrt(fanIn))."""

    def __init__(self, upper=None, lower=None, bigdl_type="float"):
        super().__init__(lower, upper)


class RandomNormal(_im.RandomNormal):
    def __init__(self, mean, stdv, bigdl_type="float"):
        super().__init__(mean, stdv)


class ConstInitMethod(_im.ConstInitMethod):
    def __init__(self, value, bigdl_type="float"):
        super().__init__(value)


class Xavier(_im.Xavier):
    def __init__(self, bigdl_type="float"):
        super().__init__()


class MsraFiller(_im.MsraFiller):
    def __init__(self, varianceNormAverage=True, bigdl_type="float"):
        super().__init__(varianceNormAverage)


class BilinearFiller(_im.BilinearFiller):
    def __init__(self, bigdl_type="float"):
        super().__init__()


__all__ = ["InitializationMethod", "Zeros", "Ones", "RandomUniform", "RandomNormal", "ConstInitMethod", "Xavier",
           "MsraFiller", "BilinearFiller"]
