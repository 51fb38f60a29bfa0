"""Keras-1.2.2-style model building on top of bigdl_amd.nn: shape inference at construction time, Sequential /
functional Model, compile / fit / evaluate / predict.

Reference: S/nn/keras/KerasLayer.scala:31-260 (KerasLayer wraps a built "labor" module; KerasIdentityWrapper /
KerasLayerWrapper for torch layers), Topology.scala:40-330 (KerasModel.compile/fit/evaluate/predict, Model,
Sequential), KerasUtils.scala:28-200 (init / activation / loss / optimizer / metric name tables),
Input.scala (Input node).

Shapes are python lists whose first entry is the batch dimension (None). A layer is built as soon as its input
shape is known: ``Sequential.add`` builds with the previous layer's output shape, ``layer.inputs(node)`` builds
with the node's output shape. Output shapes come from ``computeOutputShape`` where the layer defines it, else
from a dry run of the built labor on a ones tensor of batch 2 (reference KerasLayerWrapper does the same).
"""
import math

import torch

from .. import nn
from ..nn.abstractnn import AbstractModule
from ..nn.containers import Container
from ..utils.shape import MultiShape, Shape, SingleShape
from ..utils.table import Table


# ------------------------------------------------------------------------------------------- shapes
def _as_list(shape):
    if shape is None:
        return None
    if isinstance(shape, SingleShape):
        return list(shape.dims)
    if isinstance(shape, MultiShape):
        return [_as_list(s) for s in shape.shapes]
    if isinstance(shape, (list, tuple)) and shape and isinstance(shape[0], (list, tuple, Shape)):
        return [_as_list(s) for s in shape]
    return [None if d in (None, -1) else int(d) for d in shape]


def _is_multi(shape):
    return bool(shape) and isinstance(shape[0], list)


def add_batch(shape):
    if shape is None:
        return None
    if _is_multi(shape):
        return [add_batch(s) for s in shape]
    return [None] + list(shape)


def remove_batch(shape):
    if shape is None:
        return None
    if _is_multi(shape):
        return [remove_batch(s) for s in shape]
    return list(shape[1:])


def _dummy(shape, batch=2):
    if _is_multi(shape):
        t = Table()
        for i, s in enumerate(shape):
            t[i + 1] = _dummy(s, batch)
        return t
    return torch.ones([batch] + [1 if d is None else d for d in shape[1:]])


def _shape_of(out):
    if isinstance(out, torch.Tensor):
        return [None] + list(out.shape[1:])
    if isinstance(out, Table):
        return [_shape_of(out[i + 1]) for i in range(out.length())]
    raise TypeError(f"cannot infer the shape of {type(out)}")


# ------------------------------------------------------------------------------------- name tables
def get_init_method(init):
    if init is None or not isinstance(init, str):
        return init
    m = {"glorot_uniform": nn.Xavier(), "one": nn.Ones(), "zero": nn.Zeros(),
         "uniform": nn.RandomUniform(-0.05, 0.05), "normal": nn.RandomNormal(0.0, 0.05)}
    key = init.lower()
    if key not in m:
        raise ValueError(f"Unsupported initialization method: {key}")
    return m[key]


def get_torch_activation(name):
    if name is None:
        return None
    m = {"tanh": nn.Tanh, "sigmoid": nn.Sigmoid, "relu": nn.ReLU, "softmax": nn.SoftMax, "softplus": nn.SoftPlus,
         "softsign": nn.SoftSign, "hard_sigmoid": nn.HardSigmoid, "linear": nn.Identity}
    key = name.lower()
    if key not in m:
        raise ValueError(f"Invalid activation: {key}. Only simple activations can be constructed using string")
    return m[key]()


def get_keras_activation(act):
    """String / KerasLayer / torch module -> KerasLayer (or None)."""
    if act is None or isinstance(act, KerasLayer):
        return act
    if isinstance(act, str):
        if act.lower() == "softmax":
            from .layers import SoftMax
            return SoftMax()
        return KerasIdentityWrapper(get_torch_activation(act))
    return KerasIdentityWrapper(act)


def to_criterion(loss):
    if not isinstance(loss, str):
        return loss
    m = {"binary_crossentropy": lambda: nn.BCECriterion(), "categorical_crossentropy": lambda: nn.CategoricalCrossEntropy(),
         "mse": lambda: nn.MSECriterion(), "mean_squared_error": lambda: nn.MSECriterion(),
         "mae": lambda: nn.AbsCriterion(), "mean_absolute_error": lambda: nn.AbsCriterion(),
         "hinge": lambda: nn.MarginCriterion(), "mape": lambda: nn.MeanAbsolutePercentageCriterion(),
         "mean_absolute_percentage_error": lambda: nn.MeanAbsolutePercentageCriterion(),
         "msle": lambda: nn.MeanSquaredLogarithmicCriterion(),
         "mean_squared_logarithmic_error": lambda: nn.MeanSquaredLogarithmicCriterion(),
         "squared_hinge": lambda: nn.MarginCriterion(squared=True),
         "sparse_categorical_crossentropy": lambda: nn.ClassNLLCriterion(logProbAsInput=False),
         "kld": lambda: nn.KullbackLeiblerDivergenceCriterion(),
         "kullback_leibler_divergence": lambda: nn.KullbackLeiblerDivergenceCriterion(),
         "cosine_proximity": lambda: nn.CosineProximityCriterion(), "poisson": lambda: nn.PoissonCriterion()}
    key = loss.lower()
    if key not in m:
        raise ValueError(f"Invalid loss: {key}")
    return m[key]()


def to_optim_method(name):
    if not isinstance(name, str):
        return name
    from .. import optim
    m = {"sgd": lambda: optim.SGD(learningRate=0.01), "rmsprop": lambda: optim.RMSprop(learningRate=0.001, decayRate=0.9),
         "adamax": lambda: optim.Adamax(Epsilon=1e-8), "adagrad": lambda: optim.Adagrad(learningRate=0.01),
         "adadelta": lambda: optim.Adadelta(decayRate=0.95, Epsilon=1e-8), "adam": lambda: optim.Adam()}
    return m[name.lower()]()


def to_metrics(metrics):
    if metrics is None:
        return None
    from ..optim import Top1Accuracy
    out = []
    for m in metrics:
        if isinstance(m, str):
            if m.lower() != "accuracy":
                raise ValueError(f"Unsupported metrics: {m}")
            out.append(Top1Accuracy())
        else:
            out.append(m)
    return out


# --------------------------------------------------------------------------------------- KerasLayer
class KerasLayer(Container):
    """A Keras layer: declares its (batch-less) ``inputShape`` optionally, builds a bigdl_amd.nn ``labor``
    module once the input shape is known, and delegates execution to it."""

    def __init__(self, inputShape=None):
        super().__init__()
        s = _as_list(inputShape)
        self.kerasInputShape = add_batch(s) if s is not None else None
        self.kerasOutputShape = None

    # -------- labor
    @property
    def labor(self):
        if not self.modules:
            raise RuntimeError("This Layer hasn't been built")
        return self.modules[0]

    @labor.setter
    def labor(self, m):
        self.modules = [m]

    def _set_children(self, children):
        self.modules = list(children)

    def isBuilt(self):
        return bool(self.modules)

    def isKerasStyle(self):
        return True

    def getInputShape(self):
        return self.kerasInputShape

    def getOutputShape(self):
        if self.kerasOutputShape is None:
            raise RuntimeError(f"{self.getName()}: the layer has not been built")
        return self.kerasOutputShape

    # -------- build
    def doBuild(self, inputShape):
        raise NotImplementedError

    def computeOutputShape(self, inputShape):
        was = self.labor.train
        self.labor.evaluate()
        with torch.no_grad():
            out = self.labor.forward(_dummy(inputShape))
        if was:
            self.labor.training()
        return _shape_of(out)

    def build(self, inputShape):
        inputShape = _as_list(inputShape)
        if self.kerasInputShape is not None and remove_batch(self.kerasInputShape) != remove_batch(inputShape):
            raise ValueError(f"InputShape from constructor {remove_batch(self.kerasInputShape)} should be the same "
                             f"with the calculated inputShape: {remove_batch(inputShape)}")
        self.labor = self.doBuild(inputShape)
        self.kerasInputShape = inputShape
        self.kerasOutputShape = self.computeOutputShape(inputShape)
        return self.kerasOutputShape

    # -------- graph building
    def inputs(self, *nodes):
        if len(nodes) == 1 and isinstance(nodes[0], (list, tuple)):
            nodes = tuple(nodes[0])
        if nodes:
            shapes = [n.element.getOutputShape() for n in nodes]
            self.build(shapes[0] if len(shapes) == 1 else shapes)
        return super().inputs(*nodes)

    def __call__(self, *nodes):
        return self.inputs(*nodes)

    # -------- execution
    def updateOutput(self, input):
        return self.labor.forward(input)

    def updateGradInput(self, input, gradOutput):
        return self.labor.updateGradInput(input, gradOutput)

    def accGradParameters(self, input, gradOutput):
        self.labor.accGradParameters(input, gradOutput)

    def backward(self, input, gradOutput):
        self.gradInput = self.labor.backward(input, gradOutput)
        return self.gradInput

    def __repr__(self):
        return f"{type(self).__name__}[{self.labor!r}]" if self.modules else f"{type(self).__name__}[unbuilt]"


class KerasIdentityWrapper(KerasLayer):
    """Wraps a torch-style layer whose output shape equals its input shape (activations)."""

    def __init__(self, layer):
        super().__init__()
        if getattr(layer, "isKerasStyle", lambda: False)():
            raise ValueError(f"We only accept torch layer here, but got: {layer}")
        self.modules = [layer]

    def build(self, inputShape):
        self.kerasInputShape = _as_list(inputShape)
        self.kerasOutputShape = self.kerasInputShape
        return self.kerasOutputShape


class KerasLayerWrapper(KerasLayer):
    """Wraps any torch-style layer; the output shape is found by a dry run."""

    def __init__(self, torchLayer, inputShape=None):
        super().__init__(inputShape)
        self.torchLayer = torchLayer

    def doBuild(self, inputShape):
        return self.torchLayer


class LastDimSoftMax(nn.AutogradModule):
    """Softmax over the last axis (Keras semantics for 2-D and 3-D inputs)."""

    def fn(self, x):
        return torch.softmax(x.float(), dim=-1).to(x.dtype)


def activation_module(act, input_shape=None):
    """Keras activation spec -> executable module (string, torch module, or Keras layer)."""
    if act is None:
        return None
    if isinstance(act, str):
        return LastDimSoftMax() if act.lower() == "softmax" else get_torch_activation(act)
    if isinstance(act, KerasIdentityWrapper):
        return act.labor
    if isinstance(act, KerasLayer):
        if not act.isBuilt() or act.kerasOutputShape is None:
            act.build(input_shape)
        return act
    return act


def fuse(torch_layer, activation, input_shape):
    """Torch layer followed by an optional Keras activation (reference KerasLayer.fuse)."""
    if activation is None:
        return torch_layer
    out_shape = None
    if isinstance(activation, KerasLayer) and not isinstance(activation, KerasIdentityWrapper):
        w = KerasLayerWrapper(torch_layer)
        out_shape = w.build(input_shape)
        w.modules = []
    return nn.Sequential().add(torch_layer).add(activation_module(activation, out_shape))


class InputLayer(KerasLayer):
    def __init__(self, inputShape):
        super().__init__(inputShape)
        self.modules = [nn.Identity()]
        self.kerasOutputShape = self.kerasInputShape

    def build(self, inputShape):
        return self.kerasOutputShape


def Input(inputShape=None, name=None):
    """Keras input node (reference keras/Input.scala)."""
    layer = InputLayer(inputShape)
    if name:
        layer.setName(name)
    node = nn.Node(layer)
    node._is_input = True
    return node


# --------------------------------------------------------------------------------------- models
class KerasModel(KerasLayer):
    def __init__(self):
        super().__init__()
        self._optim_method = None
        self.criterion = None
        self.vMethods = None

    def getSubModules(self):
        return list(self.labor.modules)

    def compile(self, optimizer, loss, metrics=None):
        self._optim_method = to_optim_method(optimizer)
        self.criterion = to_criterion(loss)
        self.vMethods = to_metrics(metrics)
        return self

    @staticmethod
    def _to_dataset(x, y=None, distributed=False):
        from ..dataset.core import AbstractDataSet, DataSet
        if x is None or isinstance(x, AbstractDataSet):
            return x
        if isinstance(x, (list, tuple)) and x and not isinstance(x[0], torch.Tensor):
            return DataSet.rdd(list(x)) if distributed else DataSet.array(list(x))
        x = torch.as_tensor(x)
        y = None if y is None else torch.as_tensor(y)
        return DataSet.from_tensors(x, y, distributed=distributed)

    def fit(self, x, y=None, batchSize=32, nbEpoch=10, validationData=None, distributed=False):
        from ..optim import Optimizer, Trigger
        if self._optim_method is None or self.criterion is None:
            raise RuntimeError("compile must be called before fit")
        train = self._to_dataset(x, y, distributed)
        opt = Optimizer(model=self, dataset=train, criterion=self.criterion, batchSize=batchSize)
        if validationData is not None:
            if self.vMethods is None:
                raise RuntimeError("Validation metrics haven't been set yet")
            vx, vy = validationData if isinstance(validationData, tuple) else (validationData, None)
            opt.setValidation(Trigger.everyEpoch(), self._to_dataset(vx, vy, distributed), self.vMethods, batchSize)
        opt.setOptimMethod(self._optim_method).setEndWhen(Trigger.maxEpoch(nbEpoch))
        opt.optimize()
        return self

    def evaluate(self, x=None, y=None, batchSize=32):
        if x is None:                 # module-mode switch (AbstractModule.evaluate())
            return super().evaluate()
        from ..optim.evaluator import evaluate_dataset
        if self.vMethods is None:
            raise RuntimeError("Evaluation metrics haven't been set yet")
        res = evaluate_dataset(self, self._to_dataset(x, y), self.vMethods, batchSize)
        return list(zip(res, self.vMethods))

    def predict(self, x, batchSize=32, shareBuffer=False):
        if isinstance(x, torch.Tensor):
            self.evaluate()
            outs = []
            with torch.no_grad():
                for i in range(0, x.shape[0], batchSize):
                    outs.append(self.forward(x[i:i + batchSize]).clone())
            return torch.cat(outs)
        return super().predict(self._to_dataset(x), batchSize, shareBuffer)


class Sequential(KerasModel):
    """Keras Sequential: ``add`` builds each layer against the running output shape."""

    def __init__(self):
        super().__init__()
        self.modules = [nn.Sequential()]
        self.frozen = False

    def add(self, module):
        if self.frozen:
            raise RuntimeError("This Sequential has been frozen, as it has been added into other container")
        if isinstance(module, Sequential):
            module.frozen = True
        if not getattr(module, "isKerasStyle", lambda: False)():
            raise ValueError(f"Sequential only accepts Keras-style layers, got {module}; wrap torch layers in "
                             f"KerasLayerWrapper")
        if not self.labor.modules:
            if module.getInputShape() is None:
                raise RuntimeError("The first layer should explicitly declare inputshape")
            out = module.build(module.getInputShape())
            self.kerasInputShape = module.getInputShape()
        else:
            out = module.build(self.kerasOutputShape)
        self.kerasOutputShape = out
        self.labor.add(module)
        return self

    def build(self, inputShape):
        if self.kerasInputShape is not None and remove_batch(self.kerasInputShape) != remove_batch(_as_list(inputShape)):
            raise ValueError("input shape mismatch")
        return self.kerasOutputShape

    def computeOutputShape(self, inputShape):
        return self.kerasOutputShape


class Model(KerasModel):
    """Functional Keras model over Keras nodes (reference Topology.scala Model)."""

    def __init__(self, input=None, output=None):
        super().__init__()
        if input is None:            # placeholder used by the deserializer
            return
        ins = list(input) if isinstance(input, (list, tuple)) else [input]
        outs = list(output) if isinstance(output, (list, tuple)) else [output]
        self.modules = [nn.Graph(ins, outs)]
        self.kerasInputShape = [n.element.getOutputShape() for n in ins]
        self.kerasOutputShape = [n.element.getOutputShape() for n in outs]
        if len(ins) == 1:
            self.kerasInputShape = self.kerasInputShape[0]
        if len(outs) == 1:
            self.kerasOutputShape = self.kerasOutputShape[0]
        self._init_args = ((), {})

    def build(self, inputShape):
        return self.kerasOutputShape

    def computeOutputShape(self, inputShape):
        return self.kerasOutputShape
