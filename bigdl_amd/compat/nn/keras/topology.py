"""Reference ``bigdl.nn.keras.topology`` (P/nn/keras/topology.py): Keras-style ``Sequential`` / ``Model`` with
``compile`` / ``fit`` / ``evaluate`` / ``predict`` taking the reference's keywords (``batch_size``,
``nb_epoch``, ``validation_data``) and ndarrays, over ``bigdl_amd.keras.engine``."""
import numpy as np

from .... import keras as _k
from ..._convert import to_numpy, to_torch
from .layer import KerasLayer


def _unwrap(v):
    return v.value if hasattr(v, "value") and not isinstance(v, (np.ndarray, str)) else v


class KerasModel(KerasLayer):
    def compile(self, optimizer, loss, metrics=None):
        self.value.compile(_unwrap(optimizer), _unwrap(loss), metrics)
        return self

    def fit(self, x, y=None, batch_size=32, nb_epoch=10, validation_data=None, distributed=False):
        val = None if validation_data is None else tuple(to_torch(np.asarray(v)) for v in validation_data)
        self.value.fit(to_torch(np.asarray(x)), None if y is None else to_torch(np.asarray(y)), batchSize=batch_size,
                       nbEpoch=nb_epoch, validationData=val, distributed=distributed)
        return self

    def evaluate(self, x, y=None, batch_size=32):
        return self.value.evaluate(to_torch(np.asarray(x)), None if y is None else to_torch(np.asarray(y)),
                                   batchSize=batch_size)

    def predict(self, x, batch_size=32, distributed=False):
        return to_numpy(self.value.predict(to_torch(np.asarray(x)), batchSize=batch_size))


class Sequential(KerasModel):
    def __init__(self, jvalue=None, bigdl_type="float"):
        self.value = jvalue if jvalue is not None else _k.Sequential()
        self.bigdl_type = bigdl_type

    def add(self, model):
        self.value.add(_unwrap(model))
        return self


class Model(KerasModel):
    def __init__(self, input, output, jvalue=None, bigdl_type="float"):
        self.value = jvalue if jvalue is not None else _k.Model(_unwrap(input), _unwrap(output))
        self.bigdl_type = bigdl_type


def Input(shape=None, name=None, bigdl_type="float"):
    """Reference keras ``Input``: a graph node for functional ``Model``s."""
    return _k.Input(shape) if name is None else _k.Input(shape, name=name)


__all__ = ["KerasModel", "Sequential", "Model", "Input"]
