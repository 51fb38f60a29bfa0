"""``bigdl.nn.layer`` for bigdl_amd (reference P/nn/layer.py:117-848 ``Layer`` / ``Container`` / ``Model`` and the
per-layer constructors that follow).

Every engine module class is exposed under its reference name with the reference Python calling convention:
positional arguments in the Scala order, snake_case keywords (``n_input_plane``, ``with_bias``, ``init_weight``
as an ndarray, ``bigdl_type`` accepted and ignored), and the ndarray-in / ndarray-out ``Layer`` API
(``forward``, ``backward``, ``get_weights``, ``predict``, ``evaluate``, ``save``, ``Model.loadModel`` ...).
The wrapped engine module is ``layer.value``; graphs are built with ``layer(node)`` and ``Model(inputs,
outputs)`` exactly as in the reference.
"""
import numpy as np
import torch

from ... import nn as _nn
from ...nn.abstractnn import AbstractCriterion, AbstractModule
from .._convert import convert_kwargs, to_numpy, to_torch
from ..util.common import EvaluatedResult, RDD, Sample, samples_to_engine, to_list


class Layer:
    """Reference Layer: a handle on an engine module with the ndarray API."""

    _impl = None

    def __init__(self, *args, **kwargs):
        if "jvalue" in kwargs or (args and isinstance(args[0], AbstractModule) and self._impl is None):
            self.value = kwargs.get("jvalue", args[0] if args else None)
        else:
            args = [to_torch(a) if isinstance(a, np.ndarray) else a for a in args]
            self.value = self._impl(*args, **convert_kwargs(self._impl, kwargs))
        self.bigdl_type = "float"

    # -------------------------------------------------------------- identity / construction
    @classmethod
    def of(cls, module):
        if isinstance(module, Layer):
            return module
        wrap = _WRAPPERS.get(type(module).__name__)
        obj = object.__new__(wrap if wrap is not None else Layer)
        obj.value = module
        obj.bigdl_type = "float"
        return obj

    from_jvalue = of

    def __call__(self, x=None):
        nodes = to_list(x) if x is not None else []
        return self.value.inputs(*nodes)

    def __str__(self):
        return str(self.value)

    __repr__ = __str__

    def set_name(self, name):
        self.value.setName(name)
        return self

    def name(self):
        return self.value.getName()

    def set_seed(self, seed=123):
        from ...utils.random_generator import RNG

        RNG.setSeed(seed)
        return self

    def get_dtype(self):
        return "float32"

    # -------------------------------------------------------------- compute
    def forward(self, input):
        out = self.value.forward(to_torch(_as_array(input)))
        return to_numpy(out)

    def backward(self, input, grad_output):
        g = self.value.backward(to_torch(_as_array(input)), to_torch(_as_array(grad_output)))
        return to_numpy(g)

    def zero_grad_parameters(self):
        self.value.zeroGradParameters()

    def update_parameters(self, learning_rate):
        p = self.value.parameters()
        if p:
            with torch.no_grad():
                for w, g in zip(*p):
                    w.add_(g, alpha=-learning_rate)

    def reset(self):
        self.value.reset()
        return self

    def parameters(self):
        """{layer name: {"weight", "bias", "gradWeight", "gradBias": ndarray}} (reference :219)."""
        out = {}
        for m in _leaves(self.value):
            d = {}
            for w, g in getattr(m, "_params", ()):
                t, gt = getattr(m, w, None), getattr(m, g, None)
                if t is not None:
                    d[w] = to_numpy(t)
                    if gt is not None:
                        d["grad" + w[0].upper() + w[1:]] = to_numpy(gt)
            if d:
                out[m.getName()] = d
        return out

    def get_weights(self):
        p = self.value.parameters()
        return [to_numpy(w) for w in p[0]] if p else None

    def set_weights(self, weights):
        p = self.value.parameters()
        ws = p[0] if p else []
        if len(weights) != len(ws):
            raise ValueError(f"set_weights: expected {len(ws)} arrays, got {len(weights)}")
        with torch.no_grad():
            for w, a in zip(ws, weights):
                if tuple(w.shape) != tuple(np.shape(a)):
                    raise ValueError(f"set_weights: shape {np.shape(a)} does not match {tuple(w.shape)}")
                w.copy_(torch.as_tensor(np.asarray(a), dtype=w.dtype))
        w16 = getattr(self.value, "_w16", None)
        if w16:
            self.value.refresh_bf16_shadow() if hasattr(self.value, "refresh_bf16_shadow") else None

    def is_with_weights(self):
        p = self.value.parameters()
        return bool(p and p[0])

    # -------------------------------------------------------------- modes
    def training(self, is_training=True):
        if is_training:
            self.value.training()
        else:
            self.value.evaluate()
        return self

    def is_training(self):
        return self.value.isTraining()

    def evaluate(self, *args):
        """No argument: switch to inference mode. ``(dataset, batch_size, val_methods)``: distributed
        evaluation returning EvaluatedResults (reference :238)."""
        if not args:
            self.value.evaluate()
            return self
        data, batch_size, methods = args
        from ...optim.evaluator import Evaluator

        ds = samples_to_engine(data) if isinstance(data, (RDD, list)) else data
        methods = [m.value if hasattr(m, "value") else m for m in to_list(methods)]
        res = Evaluator(self.value).test(ds, methods, batch_size)
        return [EvaluatedResult(r.result()[0], r.result()[1], m.format()) for r, m in res]

    def freeze(self, names=None):
        self.value.freeze(*(to_list(names) if names else []))
        return self

    def unfreeze(self, names=None):
        self.value.unFreeze(*(to_list(names) if names else []))
        return self

    def setWRegularizer(self, wRegularizer):
        self.value.wRegularizer = getattr(wRegularizer, "value", wRegularizer)

    def setBRegularizer(self, bRegularizer):
        self.value.bRegularizer = getattr(bRegularizer, "value", bRegularizer)

    def set_running_mean(self, running_mean):
        self.value.runningMean.copy_(torch.as_tensor(np.asarray(running_mean)))
        return self

    def set_running_std(self, running_std):
        self.value.runningVar.copy_(torch.as_tensor(np.asarray(running_std)))
        return self

    def quantize(self):
        return Layer.of(self.value.quantize())

    # -------------------------------------------------------------- prediction
    def predict_local(self, X, batch_size=-1):
        from ...optim.predictor import Predictor

        return to_numpy(Predictor(self.value, batch_size).predict(to_torch(np.asarray(X, dtype=np.float32))))

    def predict_class_local(self, X):
        return self.predict_local(X).argmax(-1) + 1

    def predict(self, features, batch_size=-1):
        if isinstance(features, RDD):
            return self.predict_distributed(features, batch_size)
        return self.predict_local(features, batch_size)

    def predict_class(self, features):
        if isinstance(features, RDD):
            return self.predict_class_distributed(features)
        return self.predict_class_local(features)

    def predict_distributed(self, data_rdd, batch_size=-1):
        from ...optim.predictor import Predictor

        samples = samples_to_engine(data_rdd)
        out = Predictor(self.value, batch_size).predict(samples)
        return RDD(list(to_numpy(out)))

    def predict_class_distributed(self, data_rdd):
        res = self.predict_distributed(data_rdd)
        return RDD([int(np.argmax(r)) + 1 for r in res])

    def predict_image(self, image_frame, output_layer=None, share_buffer=False, batch_per_partition=4,
                      predict_key="predict"):
        from ...optim.predictor import Predictor

        return Predictor(self.value).predictImage(image_frame, output_layer, share_buffer, batch_per_partition,
                                                  predict_key)

    # -------------------------------------------------------------- persistence
    def save(self, path, over_write=False):
        self.value.saveModule(path, overWrite=over_write)
        return self

    def saveModel(self, modelPath, weightPath=None, over_write=False):
        self.value.saveModule(modelPath, weightPath, overWrite=over_write)
        return self

    def save_caffe(self, prototxt_path, model_path, use_v2=True, overwrite=False):
        self.value.saveCaffe(prototxt_path, model_path, use_v2, overwrite)
        return self

    def save_tensorflow(self, inputs, path, byte_order="little_endian", data_format="nhwc"):
        self.value.saveTF(inputs, path, byte_order, data_format.upper())
        return self


def _as_array(x):
    if isinstance(x, Sample):
        return x.feature.to_ndarray()
    return x


def _leaves(m):
    mods = getattr(m, "modules", None)
    if mods:
        out = []
        for c in mods:
            out += _leaves(c)
        return out
    return [m]


class Container(Layer):
    def add(self, model):
        self.value.add(model.value if isinstance(model, Layer) else model)
        return self

    def layers(self):
        return [Layer.of(m) for m in self.value.modules]

    def flattened_layers(self, include_container=False):
        return [Layer.of(m) for m in self.value.flattened_layers()] if hasattr(self.value, "flattened_layers") \
            else [Layer.of(m) for m in _leaves(self.value)]


class Model(Container):
    """Graph container: ``Model(inputs, outputs)`` over nodes from ``Input()`` / ``layer(node)`` (reference :605),
    plus the model loaders."""

    def __init__(self, inputs, outputs, jvalue=None, bigdl_type="float", byte_order="little_endian",
                 model_type="bigdl"):
        if jvalue is not None:
            self.value = jvalue
        else:
            self.value = _nn.Graph(to_list(inputs), to_list(outputs))
        self.bigdl_type = bigdl_type

    @staticmethod
    def load(path, bigdl_type="float"):
        from ...nn.module import Module

        return Layer.of(Module.loadModule(path))

    @staticmethod
    def loadModel(modelPath, weightPath=None, bigdl_type="float"):
        from ...nn.module import Module

        return Layer.of(Module.loadModule(modelPath, weightPath))

    @staticmethod
    def load_torch(path, bigdl_type="float"):
        from ...nn.module import Module

        return Layer.of(Module.loadTorch(path))

    @staticmethod
    def load_keras(json_path=None, hdf5_path=None, by_name=False):
        from ...keras.converter import load_keras

        return Layer.of(load_keras(json_path=json_path, hdf5_path=hdf5_path))

    @staticmethod
    def load_caffe(model, defPath, modelPath, match_all=True, bigdl_type="float"):
        from ...nn.module import Module

        return Layer.of(Module.loadCaffe(model.value if isinstance(model, Layer) else model, defPath, modelPath,
                                         match_all))

    @staticmethod
    def load_caffe_model(defPath, modelPath, bigdl_type="float"):
        from ...nn.module import Module

        return Layer.of(Module.loadCaffeModel(defPath, modelPath))

    @staticmethod
    def load_tensorflow(path, inputs, outputs, byte_order="little_endian", bin_file=None,
                        generated_backward=True, bigdl_type="float"):
        from ...nn.module import Module

        return Layer.of(Module.loadTF(path, inputs, outputs, byte_order, bin_file, generated_backward))

    @staticmethod
    def load_onnx(path):
        from ...nn.module import Module

        return Layer.of(Module.loadONNX(path))


def Input(name=None):
    return _nn.Input(name)


def Node(layer):
    from ...nn.graph import Node as _N

    return _N(layer.value if isinstance(layer, Layer) else layer)


# ------------------------------------------------------------------------------ generated layer classes
_WRAPPERS = {}
_SKIP = {"AbstractModule", "AbstractCriterion", "AutogradModule", "AutogradCriterion", "Container", "Graph",
         "Node", "Input", "Module", "Table", "T"}


def _make(name, impl):
    from ...nn.containers import Container as _EC

    base = Container if issubclass(impl, _EC) else Layer
    cls = type(name, (base,), {"_impl": impl, "__doc__": f"Reference ``bigdl.nn.layer.{name}`` over the engine's "
                                                          f"``bigdl_amd.nn.{name}``."})
    cls.__module__ = __name__
    return cls


for _name in dir(_nn):
    _obj = getattr(_nn, _name)
    if (isinstance(_obj, type) and issubclass(_obj, AbstractModule) and not issubclass(_obj, AbstractCriterion)
            and _name not in _SKIP and not _name.startswith("_")):
        _WRAPPERS[_name] = _make(_name, _obj)
        globals()[_name] = _WRAPPERS[_name]

__all__ = ["Layer", "Container", "Model", "Input", "Node"] + sorted(_WRAPPERS)
