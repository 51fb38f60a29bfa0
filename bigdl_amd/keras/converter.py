"""Keras 1.2.2 model-definition (JSON) and weight conversion into bigdl_amd.keras models.

Reference: P/keras/converter.py:32-1759 (DefinitionLoader: Sequential / functional Model JSON -> layers;
WeightsConverter: per-layer Keras weight layout -> BigDL parameters; WeightLoader.load_weights_*),
P/keras/backend.py (KerasModelWrapper.fit/evaluate/predict through BigDL).

Weights are given as ``{layer_name: [numpy arrays in Keras order]}`` (what ``layer.get_weights()`` returns),
or read from a Keras HDF5 weight file by ``bigdl_amd.utils.hdf5`` when the file uses the plain layout Keras
writes (contiguous float datasets).
"""
import json

import numpy as np
import torch

from .. import nn
from . import layers as KL
from .engine import Input, KerasLayer, Model, Sequential


def _shape(cfg):
    s = cfg.get("batch_input_shape")
    if s is not None:
        return [d for d in s[1:]]
    if cfg.get("input_dim") is not None:
        if cfg.get("input_length") is not None:
            return [cfg["input_length"], cfg["input_dim"]]
        return [cfg["input_dim"]]
    return None


def _act(a):
    return None if a in (None, "linear") else a


def _reg(r):
    if not r:
        return None
    from ..optim.regularizer import L1L2Regularizer
    return L1L2Regularizer(float(r.get("l1", 0.0)), float(r.get("l2", 0.0)))


def create_layer(class_name, cfg):
    """Keras layer config -> bigdl_amd.keras layer (reference LayerConverter.create_*)."""
    ish = _shape(cfg)
    c = class_name
    dimo = cfg.get("dim_ordering", "th")
    if c == "Dense":
        return KL.Dense(cfg["output_dim"], cfg.get("init", "glorot_uniform"), _act(cfg.get("activation")),
                        _reg(cfg.get("W_regularizer")), _reg(cfg.get("b_regularizer")), cfg.get("bias", True), ish)
    if c == "Activation":
        return KL.Activation(cfg["activation"], ish)
    if c == "Dropout":
        return KL.Dropout(cfg["p"], ish)
    if c == "Flatten":
        return KL.Flatten(ish)
    if c == "Reshape":
        return KL.Reshape(cfg["target_shape"], ish)
    if c == "Permute":
        return KL.Permute(cfg["dims"], ish)
    if c == "RepeatVector":
        return KL.RepeatVector(cfg["n"], ish)
    if c == "Convolution1D":
        return KL.Convolution1D(cfg["nb_filter"], cfg["filter_length"], cfg.get("init", "glorot_uniform"),
                                _act(cfg.get("activation")), cfg.get("border_mode", "valid"),
                                cfg.get("subsample_length", 1), _reg(cfg.get("W_regularizer")),
                                _reg(cfg.get("b_regularizer")), cfg.get("bias", True), ish)
    if c == "Convolution2D":
        return KL.Convolution2D(cfg["nb_filter"], cfg["nb_row"], cfg["nb_col"], cfg.get("init", "glorot_uniform"),
                                _act(cfg.get("activation")), cfg.get("border_mode", "valid"),
                                cfg.get("subsample", (1, 1)), dimo, _reg(cfg.get("W_regularizer")),
                                _reg(cfg.get("b_regularizer")), cfg.get("bias", True), ish)
    if c == "Convolution3D":
        return KL.Convolution3D(cfg["nb_filter"], cfg["kernel_dim1"], cfg["kernel_dim2"], cfg["kernel_dim3"],
                                cfg.get("init", "glorot_uniform"), _act(cfg.get("activation")),
                                cfg.get("border_mode", "valid"), cfg.get("subsample", (1, 1, 1)), dimo,
                                _reg(cfg.get("W_regularizer")), _reg(cfg.get("b_regularizer")), cfg.get("bias", True),
                                ish)
    if c == "AtrousConvolution2D":
        return KL.AtrousConvolution2D(cfg["nb_filter"], cfg["nb_row"], cfg["nb_col"], cfg.get("init", "glorot_uniform"),
                                      _act(cfg.get("activation")), cfg.get("subsample", (1, 1)),
                                      cfg.get("atrous_rate", (1, 1)), dimo, inputShape=ish)
    if c == "Deconvolution2D":
        return KL.Deconvolution2D(cfg["nb_filter"], cfg["nb_row"], cfg["nb_col"], cfg.get("init", "glorot_uniform"),
                                  _act(cfg.get("activation")), cfg.get("subsample", (1, 1)), dimo,
                                  bias=cfg.get("bias", True), inputShape=ish)
    if c in ("MaxPooling1D", "AveragePooling1D"):
        cls = KL.MaxPooling1D if c.startswith("Max") else KL.AveragePooling1D
        return cls(cfg.get("pool_length", 2), cfg.get("stride") or -1, cfg.get("border_mode", "valid"), ish)
    if c in ("MaxPooling2D", "AveragePooling2D"):
        cls = KL.MaxPooling2D if c.startswith("Max") else KL.AveragePooling2D
        return cls(cfg.get("pool_size", (2, 2)), cfg.get("strides"), cfg.get("border_mode", "valid"), dimo, ish)
    if c in ("MaxPooling3D", "AveragePooling3D"):
        cls = KL.MaxPooling3D if c.startswith("Max") else KL.AveragePooling3D
        return cls(cfg.get("pool_size", (2, 2, 2)), cfg.get("strides"), dimo, ish)
    if c in ("GlobalMaxPooling1D", "GlobalAveragePooling1D"):
        return getattr(KL, c)(ish)
    if c in ("GlobalMaxPooling2D", "GlobalAveragePooling2D", "GlobalMaxPooling3D", "GlobalAveragePooling3D"):
        return getattr(KL, c)(dimo, ish)
    if c == "BatchNormalization":
        return KL.BatchNormalization(cfg.get("epsilon", 1e-3), cfg.get("momentum", 0.99), dimOrdering=dimo,
                                     inputShape=ish)
    if c == "Embedding":
        return KL.Embedding(cfg["input_dim"], cfg["output_dim"], cfg.get("init", "uniform"),
                            inputShape=[cfg["input_length"]] if cfg.get("input_length") else ish)
    if c in ("SimpleRNN", "LSTM", "GRU"):
        kw = dict(returnSequences=cfg.get("return_sequences", False), goBackwards=cfg.get("go_backwards", False),
                  inputShape=ish)
        if c == "SimpleRNN":
            return KL.SimpleRNN(cfg["output_dim"], cfg.get("activation", "tanh"), **kw)
        return getattr(KL, c)(cfg["output_dim"], cfg.get("activation", "tanh"),
                              cfg.get("inner_activation", "hard_sigmoid"), **kw)
    if c == "Bidirectional":
        inner = cfg["layer"]
        rec = create_layer(inner["class_name"], dict(inner["config"], batch_input_shape=None))
        return KL.Bidirectional(rec, cfg.get("merge_mode", "concat"), ish)
    if c == "TimeDistributed":
        inner = cfg["layer"]
        return KL.TimeDistributed(create_layer(inner["class_name"], dict(inner["config"], batch_input_shape=None)),
                                  ish)
    if c == "ZeroPadding1D":
        p = cfg.get("padding", 1)
        return KL.ZeroPadding1D(p if isinstance(p, (list, tuple)) else (p, p), ish)
    if c == "ZeroPadding2D":
        return KL.ZeroPadding2D(cfg.get("padding", (1, 1)), dimo, ish)
    if c == "ZeroPadding3D":
        return KL.ZeroPadding3D(cfg.get("padding", (1, 1, 1)), dimo, ish)
    if c == "UpSampling1D":
        return KL.UpSampling1D(cfg.get("length", 2), ish)
    if c == "UpSampling2D":
        return KL.UpSampling2D(cfg.get("size", (2, 2)), dimo, ish)
    if c == "UpSampling3D":
        return KL.UpSampling3D(cfg.get("size", (2, 2, 2)), dimo, ish)
    if c == "Cropping1D":
        return KL.Cropping1D(cfg.get("cropping", (1, 1)), ish)
    if c == "Cropping2D":
        cr = cfg.get("cropping", ((0, 0), (0, 0)))
        return KL.Cropping2D(cr[0], cr[1], dimo, ish)
    if c == "Cropping3D":
        cr = cfg.get("cropping", ((1, 1), (1, 1), (1, 1)))
        return KL.Cropping3D(cr[0], cr[1], cr[2], dimo, ish)
    if c == "ELU":
        return KL.ELU(cfg.get("alpha", 1.0), ish)
    if c == "LeakyReLU":
        return KL.LeakyReLU(cfg.get("alpha", 0.3), ish)
    if c == "ThresholdedReLU":
        return KL.ThresholdedReLU(cfg.get("theta", 1.0), ish)
    if c == "Highway":
        return KL.Highway(_act(cfg.get("activation")), bias=cfg.get("bias", True), inputShape=ish)
    if c == "MaxoutDense":
        return KL.MaxoutDense(cfg["output_dim"], cfg.get("nb_feature", 4), bias=cfg.get("bias", True), inputShape=ish)
    if c in ("SpatialDropout1D",):
        return KL.SpatialDropout1D(cfg.get("p", 0.5), ish)
    if c in ("SpatialDropout2D", "SpatialDropout3D"):
        return getattr(KL, c)(cfg.get("p", 0.5), dimo, ish)
    if c == "GaussianNoise":
        return KL.GaussianNoise(cfg["sigma"], ish)
    if c == "GaussianDropout":
        return KL.GaussianDropout(cfg["p"], ish)
    if c == "Masking":
        return KL.Masking(cfg.get("mask_value", 0.0), ish)
    if c == "Merge":
        return KL.Merge(mode=cfg.get("mode", "sum"), concatAxis=cfg.get("concat_axis", -1))
    raise NotImplementedError(f"Keras layer {class_name} is not supported")


class DefinitionLoader:
    """Keras JSON model definition -> bigdl_amd.keras Sequential / Model."""

    @staticmethod
    def from_json_str(s):
        return DefinitionLoader.from_config(json.loads(s))

    @staticmethod
    def from_json_path(path):
        with open(path) as f:
            return DefinitionLoader.from_json_str(f.read())

    @staticmethod
    def from_config(d):
        if d["class_name"] == "Sequential":
            cfg = d["config"]
            layers = cfg if isinstance(cfg, list) else cfg.get("layers", [])
            m = Sequential()
            for l in layers:
                layer = create_layer(l["class_name"], l["config"])
                layer.setName(l["config"].get("name"))
                m.add(layer)
            return m
        if d["class_name"] == "Model":
            return DefinitionLoader._functional(d["config"])
        raise NotImplementedError(f"Keras model class {d['class_name']} is not supported")

    @staticmethod
    def _functional(cfg):
        nodes = {}
        for l in cfg["layers"]:
            name, cn, lc = l["name"], l["class_name"], l["config"]
            if cn == "InputLayer":
                nodes[name] = Input(inputShape=lc["batch_input_shape"][1:], name=name)
                continue
            inbound = l["inbound_nodes"][0] if l["inbound_nodes"] else []
            prev = [nodes[i[0]] for i in inbound]
            layer = create_layer(cn, dict(lc, batch_input_shape=None)).setName(name)
            nodes[name] = layer.inputs(*prev)
        ins = [nodes[i[0]] for i in cfg["input_layers"]]
        outs = [nodes[o[0]] for o in cfg["output_layers"]]
        return Model(ins if len(ins) > 1 else ins[0], outs if len(outs) > 1 else outs[0])


# -------------------------------------------------------------------------------------------- weights
def _find(module, cls_names):
    """First torch-style (bigdl_amd.nn) module below ``module`` whose class name is in ``cls_names``."""
    stack = [module]
    while stack:
        m = stack.pop(0)
        if type(m).__name__ in cls_names and not isinstance(m, KerasLayer):
            return m
        stack.extend(getattr(m, "modules", []) or [])
        if hasattr(m, "preTopology") and m.preTopology is not None:
            stack.append(m.preTopology)
    return None


def _set(t, v):
    t.data.copy_(torch.as_tensor(np.asarray(v), dtype=t.dtype).reshape(t.shape))


def _lstm_like(cell, ws, order_keras, order_ours, n_gates):
    """Keras 1 recurrent weights [W_g, U_g, b_g] per gate (gate order ``order_keras``) -> our stacked layout."""
    H = ws[1].shape[0]
    W = {g: ws[3 * i] for i, g in enumerate(order_keras)}
    U = {g: ws[3 * i + 1] for i, g in enumerate(order_keras)}
    b = {g: ws[3 * i + 2] for i, g in enumerate(order_keras)}
    pre = cell.preTopology
    Wcat = np.concatenate([W[g].T for g in order_ours], 0)
    bcat = np.concatenate([b[g] for g in order_ours], 0)
    _set(pre.weight, Wcat)
    if pre.bias is not None:
        _set(pre.bias, bcat)
    return H, U


def load_layer_weights(layer, ws):
    """Copy Keras-ordered weights ``ws`` into a built bigdl_amd.keras layer (reference WeightsConverter)."""
    c = type(layer).__name__
    ws = [np.asarray(w) for w in ws]
    if not ws:
        return
    if c == "Dense":
        lin = _find(layer, ("Linear",))
        _set(lin.weight, ws[0].T)
        if len(ws) > 1 and lin.bias is not None:
            _set(lin.bias, ws[1])
    elif c in ("Convolution2D", "AtrousConvolution2D"):
        conv = _find(layer, ("SpatialConvolution", "SpatialDilatedConvolution"))
        w = ws[0] if layer.dimOrdering.lower() == "th" else ws[0].transpose(3, 2, 0, 1)
        _set(conv.weight, w)
        if len(ws) > 1 and conv.bias is not None:
            _set(conv.bias, ws[1])
    elif c == "Convolution1D":
        conv = _find(layer, ("SpatialConvolution",))
        # Keras 1 Convolution1D W: (filter_length, 1, input_dim, nb_filter) -> OIHW (nb_filter, input_dim, k, 1)
        w = ws[0].reshape(ws[0].shape[0], ws[0].shape[-2], ws[0].shape[-1]).transpose(2, 1, 0)[..., None]
        _set(conv.weight, w)
        if len(ws) > 1 and conv.bias is not None:
            _set(conv.bias, ws[1])
    elif c == "BatchNormalization":
        bn = _find(layer, ("SpatialBatchNormalization", "BatchNormalization"))
        _set(bn.weight, ws[0])
        _set(bn.bias, ws[1])
        if len(ws) > 3:
            bn.runningMean.copy_(torch.as_tensor(ws[2]))
            bn.runningVar.copy_(torch.as_tensor(ws[3]))
    elif c == "Embedding":
        lt = _find(layer, ("LookupTable",))
        _set(lt.weight, ws[0])
    elif c == "LSTM":
        cell = _find(layer, ("LSTM",))
        H, U = _lstm_like(cell, ws, ["i", "c", "f", "o"], ["i", "c", "f", "o"], 4)
        _set(cell.h2g.weight, np.concatenate([U[g].T for g in ["i", "c", "f", "o"]], 0))
    elif c == "GRU":
        cell = _find(layer, ("GRU",))
        H, U = _lstm_like(cell, ws, ["z", "r", "h"], ["r", "z", "h"], 3)
        _set(cell.h2g.weight, np.concatenate([U["r"].T, U["z"].T], 0))
        _set(cell.h2n.weight, U["h"].T)
    elif c == "SimpleRNN":
        cell = _find(layer, ("RnnCell",))
        _set(cell.preTopology.weight, ws[0].T)
        _set(cell.h2h.weight, ws[1].T)
        if cell.preTopology.bias is not None:
            _set(cell.preTopology.bias, ws[2])
    else:
        params = layer.parameters()[0] if layer.parameters() else []
        if len(params) != len(ws):
            raise NotImplementedError(f"weight conversion for Keras layer {c} is not supported")
        for p, w in zip(params, ws):
            _set(p, w)


class WeightLoader:
    @staticmethod
    def load_weights_from_dict(model, weights):
        """``weights``: {layer_name: [arrays]} in Keras order."""
        layers = _keras_layers(model)
        for name, ws in weights.items():
            if name in layers:
                load_layer_weights(layers[name], ws)
        return model

    @staticmethod
    def load_weights_from_hdf5(model, path):
        from ..utils.hdf5 import read_keras_weights
        return WeightLoader.load_weights_from_dict(model, read_keras_weights(path))

    @staticmethod
    def load_weights_from_json_hdf5(def_json, weights_hdf5):
        m = DefinitionLoader.from_json_path(def_json)
        return WeightLoader.load_weights_from_hdf5(m, weights_hdf5)


def _keras_layers(model):
    out = {}
    stack = [model]
    while stack:
        m = stack.pop()
        if isinstance(m, KerasLayer) and m.hasName():
            out[m.getName()] = m
        stack.extend(getattr(m, "modules", []) or [])
    return out


def load_keras(json_path=None, hdf5_path=None, json_str=None, weights=None):
    """Keras 1.2.2 model -> bigdl_amd model (reference bigdl.keras.converter / Model.load_keras)."""
    m = DefinitionLoader.from_json_str(json_str) if json_str is not None else DefinitionLoader.from_json_path(json_path)
    if weights is not None:
        WeightLoader.load_weights_from_dict(m, weights)
    elif hdf5_path is not None:
        WeightLoader.load_weights_from_hdf5(m, hdf5_path)
    return m


__all__ = ["DefinitionLoader", "WeightLoader", "create_layer", "load_layer_weights", "load_keras"]
