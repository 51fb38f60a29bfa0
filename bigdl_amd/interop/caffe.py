"""Caffe interop: prototxt + caffemodel -> BigDL Graph (and weights into an existing model), and the reverse.

Reference: S/utils/caffe/CaffeLoader.scala:57-577 (``load`` copies blobs into a given model by layer name,
``matchAll``; ``loadCaffe`` builds a Graph from the net definition, returns (model, criterion) with loss layers
turned into a ParallelCriterion; customized converters per layer type :37-55), Converter.scala /
LayerConverter.scala / V1LayerConverter.scala (per-type conversion, V1 and V2 layer formats),
CaffePersister.scala:47 (model -> prototxt + caffemodel).

No generated protobuf code: the caffe.proto messages the loader needs are described by the table below and
decoded / encoded by ``protoschema`` (text format and binary wire format share one representation).
"""
import math
import os

import torch

from .. import nn
from ..utils.table import Table
from .protoschema import Schema

# ---------------------------------------------------------------------------------------------- schema
_FILLER = {1: ("type", "string", None), 2: ("value", "float", None), 3: ("min", "float", None),
           4: ("max", "float", None), 5: ("mean", "float", None), 6: ("std", "float", None),
           7: ("sparse", "int", None), 8: ("variance_norm", "enum", "VarianceNorm")}
_SHAPE = {1: ("dim", "int64", None)}
_BLOB = {1: ("num", "int", None), 2: ("channels", "int", None), 3: ("height", "int", None), 4: ("width", "int", None),
         5: ("data", "float", None), 6: ("diff", "float", None), 7: ("shape", "msg", "BlobShape"),
         8: ("double_data", "double", None), 9: ("double_diff", "double", None)}
_CONV = {1: ("num_output", "uint", None), 2: ("bias_term", "bool", None), 3: ("pad", "uint", None),
         4: ("kernel_size", "uint", None), 5: ("group", "uint", None), 6: ("stride", "uint", None),
         7: ("weight_filler", "msg", "FillerParameter"), 8: ("bias_filler", "msg", "FillerParameter"),
         9: ("pad_h", "uint", None), 10: ("pad_w", "uint", None), 11: ("kernel_h", "uint", None),
         12: ("kernel_w", "uint", None), 13: ("stride_h", "uint", None), 14: ("stride_w", "uint", None),
         15: ("engine", "enum", "Engine"), 16: ("axis", "int", None), 17: ("force_nd_im2col", "bool", None),
         18: ("dilation", "uint", None)}
_IP = {1: ("num_output", "uint", None), 2: ("bias_term", "bool", None), 3: ("weight_filler", "msg", "FillerParameter"),
       4: ("bias_filler", "msg", "FillerParameter"), 5: ("axis", "int", None), 6: ("transpose", "bool", None)}
_POOL = {1: ("pool", "enum", "PoolMethod"), 2: ("kernel_size", "uint", None), 3: ("stride", "uint", None),
         4: ("pad", "uint", None), 5: ("kernel_h", "uint", None), 6: ("kernel_w", "uint", None),
         7: ("stride_h", "uint", None), 8: ("stride_w", "uint", None), 9: ("pad_h", "uint", None),
         10: ("pad_w", "uint", None), 11: ("engine", "enum", "Engine"), 12: ("global_pooling", "bool", None),
         13: ("round_mode", "enum", "RoundMode")}
_LRN = {1: ("local_size", "uint", None), 2: ("alpha", "float", None), 3: ("beta", "float", None),
        4: ("norm_region", "enum", "NormRegion"), 5: ("k", "float", None), 6: ("engine", "enum", "Engine")}
_BN = {1: ("use_global_stats", "bool", None), 2: ("moving_average_fraction", "float", None), 3: ("eps", "float", None)}
_SCALE = {1: ("axis", "int", None), 2: ("num_axes", "int", None), 3: ("filler", "msg", "FillerParameter"),
          4: ("bias_term", "bool", None), 5: ("bias_filler", "msg", "FillerParameter")}
_BIAS = {1: ("axis", "int", None), 2: ("num_axes", "int", None), 3: ("filler", "msg", "FillerParameter")}
_ELTWISE = {1: ("operation", "enum", "EltwiseOp"), 2: ("coeff", "float", None), 3: ("stable_prod_grad", "bool", None)}
_CONCAT = {1: ("concat_dim", "uint", None), 2: ("axis", "int", None)}
_DROPOUT = {1: ("dropout_ratio", "float", None)}
_RELU = {1: ("negative_slope", "float", None), 2: ("engine", "enum", "Engine")}
_PRELU = {1: ("filler", "msg", "FillerParameter"), 2: ("channel_shared", "bool", None)}
_ELU = {1: ("alpha", "float", None)}
_SOFTMAX = {1: ("engine", "enum", "Engine"), 2: ("axis", "int", None)}
_RESHAPE = {1: ("shape", "msg", "BlobShape"), 2: ("axis", "int", None), 3: ("num_axes", "int", None)}
_FLATTEN = {1: ("axis", "int", None), 2: ("end_axis", "int", None)}
_POWER = {1: ("power", "float", None), 2: ("scale", "float", None), 3: ("shift", "float", None)}
_EXPLOG = {1: ("base", "float", None), 2: ("scale", "float", None), 3: ("shift", "float", None)}
_THRESHOLD = {1: ("threshold", "float", None)}
_SLICE = {1: ("slice_dim", "uint", None), 2: ("slice_point", "uint", None), 3: ("axis", "int", None)}
_TILE = {1: ("axis", "int", None), 2: ("tiles", "int", None)}
_INPUT = {1: ("shape", "msg", "BlobShape")}
_PARAMSPEC = {1: ("name", "string", None), 2: ("share_mode", "enum", "DimCheckMode"), 3: ("lr_mult", "float", None),
              4: ("decay_mult", "float", None)}
_STATE = {1: ("phase", "enum", "Phase"), 2: ("level", "int", None), 3: ("stage", "string", None)}
_RULE = {1: ("phase", "enum", "Phase"), 2: ("min_level", "int", None), 3: ("max_level", "int", None),
         4: ("stage", "string", None), 5: ("not_stage", "string", None)}
_LAYER = {1: ("name", "string", None), 2: ("type", "string", None), 3: ("bottom", "string", None),
          4: ("top", "string", None), 5: ("loss_weight", "float", None), 6: ("param", "msg", "ParamSpec"),
          7: ("blobs", "msg", "BlobProto"), 8: ("include", "msg", "NetStateRule"), 9: ("exclude", "msg", "NetStateRule"),
          10: ("phase", "enum", "Phase"), 11: ("propagate_down", "bool", None),
          104: ("concat_param", "msg", "ConcatParameter"), 106: ("convolution_param", "msg", "ConvolutionParameter"),
          108: ("dropout_param", "msg", "DropoutParameter"), 110: ("eltwise_param", "msg", "EltwiseParameter"),
          111: ("exp_param", "msg", "ExpParameter"), 117: ("inner_product_param", "msg", "InnerProductParameter"),
          118: ("lrn_param", "msg", "LRNParameter"), 121: ("pooling_param", "msg", "PoolingParameter"),
          122: ("power_param", "msg", "PowerParameter"), 123: ("relu_param", "msg", "ReLUParameter"),
          125: ("softmax_param", "msg", "SoftmaxParameter"), 126: ("slice_param", "msg", "SliceParameter"),
          128: ("threshold_param", "msg", "ThresholdParameter"), 131: ("prelu_param", "msg", "PReLUParameter"),
          133: ("reshape_param", "msg", "ReshapeParameter"), 134: ("log_param", "msg", "LogParameter"),
          135: ("flatten_param", "msg", "FlattenParameter"), 138: ("tile_param", "msg", "TileParameter"),
          139: ("batch_norm_param", "msg", "BatchNormParameter"), 140: ("elu_param", "msg", "ELUParameter"),
          141: ("bias_param", "msg", "BiasParameter"), 142: ("scale_param", "msg", "ScaleParameter"),
          143: ("input_param", "msg", "InputParameter")}
_V1LAYER = {2: ("bottom", "string", None), 3: ("top", "string", None), 4: ("name", "string", None),
            5: ("type", "enum", "V1LayerType"), 6: ("blobs", "msg", "BlobProto"), 7: ("blobs_lr", "float", None),
            8: ("weight_decay", "float", None), 9: ("concat_param", "msg", "ConcatParameter"),
            10: ("convolution_param", "msg", "ConvolutionParameter"), 12: ("dropout_param", "msg", "DropoutParameter"),
            17: ("inner_product_param", "msg", "InnerProductParameter"), 18: ("lrn_param", "msg", "LRNParameter"),
            19: ("pooling_param", "msg", "PoolingParameter"), 21: ("power_param", "msg", "PowerParameter"),
            24: ("eltwise_param", "msg", "EltwiseParameter"), 25: ("threshold_param", "msg", "ThresholdParameter"),
            30: ("relu_param", "msg", "ReLUParameter"), 31: ("slice_param", "msg", "SliceParameter"),
            32: ("include", "msg", "NetStateRule"), 33: ("exclude", "msg", "NetStateRule"),
            35: ("loss_weight", "float", None), 39: ("softmax_param", "msg", "SoftmaxParameter"),
            41: ("exp_param", "msg", "ExpParameter")}
_NET = {1: ("name", "string", None), 2: ("layers", "msg", "V1LayerParameter"), 3: ("input", "string", None),
        4: ("input_dim", "int", None), 5: ("force_backward", "bool", None), 6: ("state", "msg", "NetState"),
        7: ("debug_info", "bool", None), 8: ("input_shape", "msg", "BlobShape"), 100: ("layer", "msg", "LayerParameter")}

_V1TYPES = {0: "NONE", 35: "ABSVAL", 1: "ACCURACY", 30: "ARGMAX", 2: "BNLL", 3: "CONCAT", 37: "CONTRASTIVE_LOSS",
            4: "CONVOLUTION", 5: "DATA", 39: "DECONVOLUTION", 6: "DROPOUT", 32: "DUMMY_DATA", 7: "EUCLIDEAN_LOSS",
            25: "ELTWISE", 38: "EXP", 8: "FLATTEN", 9: "HDF5_DATA", 10: "HDF5_OUTPUT", 28: "HINGE_LOSS", 11: "IM2COL",
            12: "IMAGE_DATA", 13: "INFOGAIN_LOSS", 14: "INNER_PRODUCT", 15: "LRN", 29: "MEMORY_DATA",
            16: "MULTINOMIAL_LOGISTIC_LOSS", 34: "MVN", 17: "POOLING", 26: "POWER", 18: "RELU", 19: "SIGMOID",
            27: "SIGMOID_CROSS_ENTROPY_LOSS", 36: "SILENCE", 20: "SOFTMAX", 21: "SOFTMAX_LOSS", 22: "SPLIT",
            33: "SLICE", 23: "TANH", 24: "WINDOW_DATA", 31: "THRESHOLD"}

SCHEMA = Schema(
    {"NetParameter": _NET, "LayerParameter": _LAYER, "V1LayerParameter": _V1LAYER, "BlobProto": _BLOB,
     "BlobShape": _SHAPE, "FillerParameter": _FILLER, "ConvolutionParameter": _CONV, "InnerProductParameter": _IP,
     "PoolingParameter": _POOL, "LRNParameter": _LRN, "BatchNormParameter": _BN, "ScaleParameter": _SCALE,
     "BiasParameter": _BIAS, "EltwiseParameter": _ELTWISE, "ConcatParameter": _CONCAT, "DropoutParameter": _DROPOUT,
     "ReLUParameter": _RELU, "PReLUParameter": _PRELU, "ELUParameter": _ELU, "SoftmaxParameter": _SOFTMAX,
     "ReshapeParameter": _RESHAPE, "FlattenParameter": _FLATTEN, "PowerParameter": _POWER, "ExpParameter": _EXPLOG,
     "LogParameter": _EXPLOG, "ThresholdParameter": _THRESHOLD, "SliceParameter": _SLICE, "TileParameter": _TILE,
     "InputParameter": _INPUT, "ParamSpec": _PARAMSPEC, "NetState": _STATE, "NetStateRule": _RULE},
    {"PoolMethod": {0: "MAX", 1: "AVE", 2: "STOCHASTIC"}, "EltwiseOp": {0: "PROD", 1: "SUM", 2: "MAX"},
     "NormRegion": {0: "ACROSS_CHANNELS", 1: "WITHIN_CHANNEL"}, "Phase": {0: "TRAIN", 1: "TEST"},
     "Engine": {0: "DEFAULT", 1: "CAFFE", 2: "CUDNN"}, "RoundMode": {0: "CEIL", 1: "FLOOR"},
     "VarianceNorm": {0: "FAN_IN", 1: "FAN_OUT", 2: "AVERAGE"}, "DimCheckMode": {0: "STRICT", 1: "PERMISSIVE"},
     "V1LayerType": _V1TYPES})

# V1 enum names -> V2 type strings
_V1_TO_V2 = {"CONVOLUTION": "Convolution", "DECONVOLUTION": "Deconvolution", "INNER_PRODUCT": "InnerProduct",
             "POOLING": "Pooling", "RELU": "ReLU", "SIGMOID": "Sigmoid", "TANH": "TanH", "LRN": "LRN",
             "DROPOUT": "Dropout", "SOFTMAX": "Softmax", "SOFTMAX_LOSS": "SoftmaxWithLoss", "CONCAT": "Concat",
             "ELTWISE": "Eltwise", "FLATTEN": "Flatten", "SPLIT": "Split", "SLICE": "Slice", "POWER": "Power",
             "EXP": "Exp", "ABSVAL": "AbsVal", "THRESHOLD": "Threshold", "BNLL": "BNLL", "DATA": "Data",
             "ACCURACY": "Accuracy", "SILENCE": "Silence", "EUCLIDEAN_LOSS": "EuclideanLoss", "MVN": "MVN"}


def _g(d, key, default=None):
    v = d.get(key) if d else None
    return v[-1] if v else default


def _gl(d, key):
    return list(d.get(key, [])) if d else []


# ---------------------------------------------------------------------------------------------- reading
def read_net_text(path):
    with open(path, "r") as f:
        return SCHEMA.parse_text("NetParameter", f.read())


def read_net_binary(path):
    with open(path, "rb") as f:
        return SCHEMA.decode("NetParameter", f.read())


def _layers(net):
    """Normalized list of layer dicts (V2 ``layer`` or V1 ``layers`` converted to V2 type strings)."""
    if net.get("layer"):
        return net["layer"]
    out = []
    for l in net.get("layers", []):
        l = dict(l)
        t = _g(l, "type")
        l["type"] = [_V1_TO_V2.get(t, str(t).title())]
        out.append(l)
    return out


def blob_to_tensor(b):
    data = b.get("data") or b.get("double_data") or []
    t = torch.tensor(data, dtype=torch.float32)
    sh = b.get("shape")
    if sh:
        dims = [int(x) for x in sh[-1].get("dim", [])]
    else:
        dims = [int(_g(b, k, 1)) for k in ("num", "channels", "height", "width")]
    if dims and math.prod(dims) == t.numel():
        return t.reshape(dims)
    return t


def tensor_to_blob(t):
    t = t.detach().float().cpu().contiguous()
    return {"shape": [{"dim": list(t.shape)}], "data": t.reshape(-1).tolist()}


# ---------------------------------------------------------------------------------------------- converters
def _conv_geom(p):
    def pick(single, h, w, default):
        if _g(p, h) is not None:
            return int(_g(p, h)), int(_g(p, w, _g(p, h)))
        v = _gl(p, single)
        if not v:
            return default, default
        return (int(v[0]), int(v[1] if len(v) > 1 else v[0]))

    kh, kw = pick("kernel_size", "kernel_h", "kernel_w", 1)
    sh, sw = pick("stride", "stride_h", "stride_w", 1)
    ph, pw = pick("pad", "pad_h", "pad_w", 0)
    dil = _gl(p, "dilation")
    d = int(dil[0]) if dil else 1
    return kh, kw, sh, sw, ph, pw, d


def _convert_layer(layer, ctx):
    """Returns a module (or None to skip) for a V2-format layer dict. ``ctx`` carries inferred channel counts."""
    t = _g(layer, "type")
    name = _g(layer, "name")
    blobs = [blob_to_tensor(b) for b in layer.get("blobs", [])]
    cin = ctx.get("channels")
    if t in ("Convolution", "Deconvolution"):
        p = _g(layer, "convolution_param", {})
        nout = int(_g(p, "num_output"))
        group = int(_g(p, "group", 1))
        bias = _g(p, "bias_term", True)
        kh, kw, sh, sw, ph, pw, d = _conv_geom(p)
        if blobs:
            cin = blobs[0].shape[1] * group if t == "Convolution" else blobs[0].shape[0]
        if t == "Convolution":
            if d > 1:
                m = nn.SpatialDilatedConvolution(cin, nout, kw, kh, sw, sh, pw, ph, d, d)
            else:
                m = nn.SpatialConvolution(cin, nout, kw, kh, sw, sh, pw, ph, group, withBias=bias)
        else:
            m = nn.SpatialFullConvolution(cin, nout, kw, kh, sw, sh, pw, ph, 0, 0, group, noBias=not bias)
        ctx["channels"] = nout
        return m
    if t == "InnerProduct":
        p = _g(layer, "inner_product_param", {})
        nout = int(_g(p, "num_output"))
        bias = _g(p, "bias_term", True)
        nin = blobs[0].shape[-1] if blobs else ctx.get("flat", cin)
        lin = nn.Linear(int(nin), nout, withBias=bias).setName(name)
        ctx["channels"] = nout
        ctx["flat"] = nout
        return nn.Sequential().add(nn.InferReshape([0, -1])).add(lin).setName(name + "_seq"), lin
    if t == "Pooling":
        p = _g(layer, "pooling_param", {})
        kh, kw, sh, sw, ph, pw, _ = _conv_geom(p)
        method = _g(p, "pool", "MAX")
        glob = _g(p, "global_pooling", False)
        ceil = _g(p, "round_mode", "CEIL") == "CEIL"
        if glob:
            if method == "AVE":
                return nn.SpatialAveragePooling(1, 1, globalPooling=True)
            return _GlobalMax()
        if method == "AVE":
            m = nn.SpatialAveragePooling(kw, kh, sw, sh, pw, ph)
        else:
            m = nn.SpatialMaxPooling(kw, kh, sw, sh, pw, ph)
        return m.ceil() if ceil else m.floor()
    if t == "ReLU":
        p = _g(layer, "relu_param", {})
        slope = _g(p, "negative_slope", 0.0)
        return nn.LeakyReLU(slope) if slope else nn.ReLU(True)
    if t == "PReLU":
        return nn.PReLU(int(blobs[0].numel()) if blobs else 0)
    if t in ("Recurrent", "RNN"):
        # Converter.scala:200-202: a bare Recurrent container (the cell is not described by the Caffe layer); its
        # weights land through load_caffe_into once a cell is added
        return nn.Recurrent()
    if t == "ELU":
        return nn.ELU(_g(_g(layer, "elu_param", {}), "alpha", 1.0))
    if t == "Sigmoid":
        return nn.Sigmoid()
    if t == "TanH":
        return nn.Tanh()
    if t == "AbsVal":
        return nn.Abs()
    if t == "BNLL":
        return nn.SoftPlus()
    if t == "LRN":
        p = _g(layer, "lrn_param", {})
        size, alpha, beta, k = int(_g(p, "local_size", 5)), _g(p, "alpha", 1.0), _g(p, "beta", 0.75), _g(p, "k", 1.0)
        if _g(p, "norm_region", "ACROSS_CHANNELS") == "WITHIN_CHANNEL":
            return nn.SpatialWithinChannelLRN(size, alpha, beta)
        return nn.SpatialCrossMapLRN(size, alpha, beta, k)
    if t == "Dropout":
        return nn.Dropout(_g(_g(layer, "dropout_param", {}), "dropout_ratio", 0.5))
    if t == "Softmax":
        return nn.SoftMax()
    if t == "BatchNorm":
        p = _g(layer, "batch_norm_param", {})
        n = int(blobs[0].numel()) if blobs else cin
        return nn.SpatialBatchNormalization(n, _g(p, "eps", 1e-5), affine=False)
    if t == "Scale":
        p = _g(layer, "scale_param", {})
        n = int(blobs[0].numel()) if blobs else cin
        if _g(p, "bias_term", False):
            return nn.Scale([1, n, 1, 1])
        return nn.CMul([1, n, 1, 1])
    if t == "Bias":
        n = int(blobs[0].numel()) if blobs else cin
        return nn.CAdd([1, n, 1, 1])
    if t == "Concat":
        p = _g(layer, "concat_param", {})
        axis = int(_g(p, "axis", _g(p, "concat_dim", 1)))
        return nn.JoinTable(axis + 1, 0)
    if t == "Eltwise":
        p = _g(layer, "eltwise_param", {})
        op = _g(p, "operation", "SUM")
        coeff = _gl(p, "coeff")
        if op == "PROD":
            return nn.CMulTable()
        if op == "MAX":
            return nn.CMaxTable()
        if coeff and any(abs(c - 1) > 1e-9 for c in coeff):
            if len(coeff) == 2 and coeff[0] == 1 and coeff[1] == -1:
                return nn.CSubTable()
            pt = nn.ParallelTable()
            for c in coeff:
                pt.add(nn.MulConstant(c))
            return nn.Sequential().add(pt).add(nn.CAddTable())
        return nn.CAddTable()
    if t == "Flatten":
        return nn.InferReshape([0, -1])
    if t == "Reshape":
        p = _g(layer, "reshape_param", {})
        dims = [int(x) for x in _g(p, "shape", {}).get("dim", [])]
        return nn.InferReshape(dims)
    if t == "Power":
        p = _g(layer, "power_param", {})
        return nn.Power(_g(p, "power", 1.0), _g(p, "scale", 1.0), _g(p, "shift", 0.0))
    if t == "Exp":
        return nn.Exp()
    if t == "Log":
        return nn.Log()
    if t == "Threshold":
        return nn.BinaryThreshold(_g(_g(layer, "threshold_param", {}), "threshold", 0.0))
    if t == "Slice":
        p = _g(layer, "slice_param", {})
        axis = int(_g(p, "axis", _g(p, "slice_dim", 1)))
        return nn.SplitTable(axis + 1) if not _gl(p, "slice_point") else _SliceAt(axis, _gl(p, "slice_point"))
    if t == "Tile":
        p = _g(layer, "tile_param", {})
        return nn.Replicate(int(_g(p, "tiles")), int(_g(p, "axis", 1)) + 1)
    if t in ("Split",):
        return nn.Identity()
    return None


class _GlobalMax(nn.AutogradModule):
    def fn(self, x):
        return x.amax(dim=(2, 3), keepdim=True)


class _SliceAt(nn.AbstractModule):
    """Caffe Slice with explicit slice points along ``axis`` (0-based) -> Table of pieces."""

    def __init__(self, axis, points):
        super().__init__()
        self.axis, self.points = axis, [int(p) for p in points]

    def updateOutput(self, input):
        edges = [0] + self.points + [input.shape[self.axis]]
        return Table(*[input.narrow(self.axis, a, b - a) for a, b in zip(edges[:-1], edges[1:])])

    def updateGradInput(self, input, gradOutput):
        return torch.cat(gradOutput.toSeq(), self.axis)


_LOSS = {"SoftmaxWithLoss": lambda: nn.ClassNLLCriterion(), "EuclideanLoss": lambda: nn.MSECriterion(),
         "SigmoidCrossEntropyLoss": lambda: nn.BCECriterion(), "HingeLoss": lambda: nn.MarginCriterion(),
         "MultinomialLogisticLoss": lambda: nn.ClassNLLCriterion(), "InfogainLoss": lambda: nn.ClassNLLCriterion()}
_SKIP = {"Data", "ImageData", "HDF5Data", "DummyData", "MemoryData", "WindowData", "Accuracy", "Silence",
         "HDF5Output"}


def _is_test_excluded(layer):
    for inc in layer.get("include", []):
        if _g(inc, "phase") == "TRAIN":
            return True
    return False


def _copy_blobs(module, blobs, name):
    """Copy Caffe blobs into the module's parameters (BN: mean/var/scale-factor into running stats)."""
    if isinstance(module, nn.Recurrent):       # every parameter of the cell, in parameters() order
        if module.cell is None:                 # a bare imported container has no parameters yet (reference)
            return
        ps = (module.parameters() or ([], []))[0]
        if len(blobs) != len(ps):
            raise ValueError(f"{name}: {len(blobs)} blobs for a Recurrent with {len(ps)} parameters")
        for dst, b in zip(ps, blobs):
            if dst.numel() != b.numel():
                raise ValueError(f"{name}: blob size {tuple(b.shape)} does not match parameter {tuple(dst.shape)}")
            dst.data.copy_(b.reshape(dst.shape))
        return
    if isinstance(module, nn.BatchNormalization) and not module.affine:
        sf = float(blobs[2].reshape(-1)[0]) if len(blobs) > 2 else 1.0
        sf = 1.0 / sf if sf != 0 else 0.0
        module.runningMean.copy_(blobs[0].reshape(-1) * sf)
        module.runningVar.copy_(blobs[1].reshape(-1) * sf)
        return
    ws = [(w, g) for w, g in module._params if getattr(module, w, None) is not None]
    if len(blobs) < len(ws) and len(blobs) != 0:
        ws = ws[:len(blobs)]
    for (w, _), b in zip(ws, blobs):
        dst = getattr(module, w)
        if dst.numel() != b.numel():
            raise ValueError(f"{name}: blob size {tuple(b.shape)} does not match parameter {w} {tuple(dst.shape)}")
        dst.data.copy_(b.reshape(dst.shape))


def load_caffe(defPath, modelPath=None, customizedConverters=None, outputNames=None):
    """Build (Graph, ParallelCriterion) from a Caffe definition and (optionally) weights."""
    net = read_net_text(defPath)
    weights = {}
    if modelPath:
        for l in _layers(read_net_binary(modelPath)):
            if l.get("blobs"):
                weights[_g(l, "name")] = l
    conv = {k.upper(): v for k, v in (customizedConverters or {}).items()}
    tops = {}
    inputs = []
    ctx = {"channels": None}
    for name in net.get("input", []):
        node = nn.Input(name)
        tops[name] = node
        inputs.append(node)
    dims = net.get("input_dim", [])
    if net.get("input_shape"):
        dims = net["input_shape"][0].get("dim", [])
    if len(dims) >= 2:
        ctx["channels"] = int(dims[1])
    criterion = nn.ParallelCriterion()
    consumed = set()
    for layer in _layers(net):
        if _is_test_excluded(layer):
            continue
        t = _g(layer, "type")
        name = _g(layer, "name")
        if name in weights:
            layer = dict(layer)
            layer["blobs"] = weights[name]["blobs"]
        if t == "Input":
            for tp in layer.get("top", []):
                node = nn.Input(tp)
                tops[tp] = node
                inputs.append(node)
            shp = _g(_g(layer, "input_param", {}), "shape", {})
            if shp and len(shp.get("dim", [])) >= 2:
                ctx["channels"] = int(shp["dim"][1])
            continue
        if t in _SKIP:
            if t in ("Data", "ImageData", "DummyData", "MemoryData") and layer.get("top"):
                node = nn.Input(layer["top"][0])
                tops[layer["top"][0]] = node
                inputs.append(node)
            continue
        if t in _LOSS and t.upper() not in conv:
            criterion.add(_LOSS[t]())
            consumed.update(layer.get("bottom", []))
            continue
        if t.upper() in conv:
            produced = conv[t.upper()](layer)
            modules = produced if isinstance(produced, (list, tuple)) else [produced]
            m, param_m = modules[0], None
        else:
            res = _convert_layer(layer, ctx)
            if res is None:
                raise ValueError(f"unsupported Caffe layer type {t!r} ({name}); pass customizedConverters")
            m, param_m = (res if isinstance(res, tuple) else (res, res))
        m.setName(name) if not m.hasName() else None
        if layer.get("blobs") and param_m is not None:
            _copy_blobs(param_m, [blob_to_tensor(b) for b in layer["blobs"]], name)
        bottoms = [tops[b] for b in layer.get("bottom", []) if b in tops]
        consumed.update(layer.get("bottom", []))
        node = m.inputs(*bottoms) if bottoms else m.inputs()
        if not bottoms:
            inputs.append(node)
        outs = layer.get("top", [])
        if len(outs) > 1 and t in ("Slice",):
            for i, tp in enumerate(outs):
                tops[tp] = nn.SelectTable(i + 1).inputs(node)
        else:
            for tp in outs:
                tops[tp] = node
    if outputNames:
        outputs = [tops[n] for n in outputNames]
    else:
        all_tops = []
        for layer in _layers(net):
            for tp in layer.get("top", []):
                if tp in tops and tp not in consumed and tops[tp] not in all_tops and tops[tp] not in inputs:
                    all_tops.append(tops[tp])
        outputs = all_tops or [list(tops.values())[-1]]
    model = nn.Graph(inputs if len(inputs) > 1 else inputs[0], outputs if len(outputs) > 1 else outputs[0])
    return model, criterion


def load_caffe_into(model, defPath, modelPath, matchAll=True, customizedConverters=None):
    """Copy Caffe weights into ``model`` by layer name (CaffeLoader.load)."""
    weights = {}
    for l in _layers(read_net_binary(modelPath)):
        if l.get("blobs"):
            weights[_g(l, "name")] = [blob_to_tensor(b) for b in l["blobs"]]
    byname = {m.getName(): m for m in model.flattened_layers() if m.hasName()}

    def walk(m):
        yield m
        for c in getattr(m, "modules", None) or []:
            yield from walk(c)

    for m in walk(model):     # Recurrent containers carry their cell's weights as one Caffe layer
        if isinstance(m, nn.Recurrent) and m.hasName() and m.getName() in weights:
            byname[m.getName()] = m
    for name, m in byname.items():
        if isinstance(m, nn.Recurrent):
            if name in weights:
                _copy_blobs(m, weights[name], name)
            continue
        if not m._params and not isinstance(m, nn.BatchNormalization):
            continue
        if name not in weights:
            if matchAll and m._params:
                raise ValueError(f"module {name} has no weights in {modelPath}")
            continue
        _copy_blobs(m, weights[name], name)
    return model


# ---------------------------------------------------------------------------------------------- writing
def _layer_def(m, name, bottoms, tops):
    d = {"name": [name], "bottom": list(bottoms), "top": list(tops)}
    blobs = []
    if isinstance(m, nn.SpatialConvolution):
        d["type"] = ["Convolution"]
        d["convolution_param"] = [{"num_output": [m.nOutputPlane], "group": [m.nGroup], "pad_h": [m.padH],
                                   "pad_w": [m.padW], "kernel_h": [m.kernelH], "kernel_w": [m.kernelW],
                                   "stride_h": [m.strideH], "stride_w": [m.strideW],
                                   "bias_term": [m.bias is not None]}]
        blobs = [m.weight] + ([m.bias] if m.bias is not None else [])
    elif isinstance(m, nn.Linear):
        d["type"] = ["InnerProduct"]
        d["inner_product_param"] = [{"num_output": [m.outputSize], "bias_term": [m.bias is not None]}]
        blobs = [m.weight] + ([m.bias] if m.bias is not None else [])
    elif isinstance(m, (nn.SpatialMaxPooling, nn.SpatialAveragePooling)):
        d["type"] = ["Pooling"]
        d["pooling_param"] = [{"pool": ["MAX" if isinstance(m, nn.SpatialMaxPooling) else "AVE"],
                               "kernel_h": [m.kH], "kernel_w": [m.kW], "stride_h": [m.dH], "stride_w": [m.dW],
                               "pad_h": [m.padH], "pad_w": [m.padW],
                               "round_mode": ["CEIL" if getattr(m, "ceilMode", False) else "FLOOR"]}]
    elif isinstance(m, nn.ReLU):
        d["type"] = ["ReLU"]
    elif isinstance(m, nn.Sigmoid):
        d["type"] = ["Sigmoid"]
    elif isinstance(m, nn.Tanh):
        d["type"] = ["TanH"]
    elif isinstance(m, nn.SoftMax):
        d["type"] = ["Softmax"]
    elif isinstance(m, nn.LogSoftMax):            # Softmax + Log (layer pair)
        d["type"] = ["Softmax"]
        log = {"name": [name + "_log"], "bottom": list(tops), "top": list(tops), "type": ["Log"]}
        return [d, log]
    elif isinstance(m, nn.Dropout):
        d["type"] = ["Dropout"]
        d["dropout_param"] = [{"dropout_ratio": [float(m.p)]}]
    elif isinstance(m, nn.SpatialCrossMapLRN):
        d["type"] = ["LRN"]
        d["lrn_param"] = [{"local_size": [m.size], "alpha": [m.alpha], "beta": [m.beta], "k": [m.k]}]
    elif isinstance(m, nn.BatchNormalization):
        d["type"] = ["BatchNorm"]
        d["batch_norm_param"] = [{"eps": [float(m.eps)]}]
        d["blobs"] = [tensor_to_blob(b) for b in (m.runningMean, m.runningVar, torch.ones(1))]
        if getattr(m, "weight", None) is None:
            return d
        # affine part as the Caffe-standard in-place Scale layer (gamma, beta)
        sc = {"name": [name + "_scale"], "bottom": list(tops), "top": list(tops), "type": ["Scale"],
              "scale_param": [{"bias_term": [m.bias is not None]}],
              "blobs": [tensor_to_blob(b) for b in ([m.weight] + ([m.bias] if m.bias is not None else []))]}
        return [d, sc]
    elif isinstance(m, (nn.Scale, nn.CMul)) and m.weight.numel() == max(m.weight.shape):
        # per-channel affine / multiply ([1, C, 1, 1] parameters) as the Caffe Scale layer
        d["type"] = ["Scale"]
        has_b = isinstance(m, nn.Scale)
        d["scale_param"] = [{"bias_term": [has_b]}]
        blobs = [m.weight.reshape(-1)] + ([m.bias.reshape(-1)] if has_b else [])
    elif isinstance(m, nn.CAdd) and m.bias.numel() == max(m.bias.shape):
        d["type"] = ["Bias"]
        blobs = [m.bias.reshape(-1)]
    elif isinstance(m, nn.JoinTable):
        d["type"] = ["Concat"]
        d["concat_param"] = [{"axis": [m.dimension - 1]}]
    elif isinstance(m, nn.CAddTable):
        d["type"] = ["Eltwise"]
        d["eltwise_param"] = [{"operation": ["SUM"]}]
    elif isinstance(m, nn.Recurrent):
        # LayerConverter.scala:530-532: type "Recurrent" with the module's weights as blobs (no recurrent_param)
        d["type"] = ["Recurrent"]
        blobs = list((m.parameters() or ([], []))[0]) if m.cell is not None else []
    elif isinstance(m, (nn.View, nn.Reshape, nn.InferReshape)):
        d["type"] = ["Flatten"]
    else:
        return None
    if blobs:
        d["blobs"] = [tensor_to_blob(b) for b in blobs]
    return d


_CAFFE_PASSTHROUGH = ("Identity", "Contiguous", "SelectTable", "Echo", "Squeeze", "Unsqueeze", "FlattenTable")


def save_caffe(module, prototxtPath, modelPath, overwrite=False, input_shape=None):
    """Persist a Sequential/Graph of convertible layers as prototxt + caffemodel (CaffePersister)."""
    for p in (prototxtPath, modelPath):
        if os.path.exists(p) and not overwrite:
            raise FileExistsError(p)
    layers = []
    # containers (Sequential / ConcatTable / Concat / ...) are flattened into a graph of their leaf layers so
    # branches keep their true bottoms (utils/intermediate BlasToIR)
    g = module if isinstance(module, nn.Graph) else module.toGraph()
    names = {}
    for n in g.order:
        nm = n.element.getName()
        if n in g.inputs_nodes and not n.prevs:
            names[n.id] = "data" if len(g.inputs_nodes) == 1 else nm
            continue
        bottoms = [names[p.id] for p in n.prevs]
        d = _layer_def(n.element, nm, bottoms, [nm])
        if d is None:
            # only layout / identity layers may vanish from the Caffe net; anything that computes must not be
            # dropped silently
            if len(bottoms) != 1 or type(n.element).__name__ not in _CAFFE_PASSTHROUGH:
                raise ValueError(f"save_caffe: cannot express {n.element.getPrintName()} in Caffe")
            names[n.id] = bottoms[0]            # pass-through (Identity, SelectTable of one input, ...)
            continue
        names[n.id] = nm
        layers.extend(d if isinstance(d, list) else [d])
    net_inputs = [names[n.id] for n in g.inputs_nodes]
    net = {"name": [module.getName()], "input": net_inputs, "layer": layers}
    if input_shape:
        net["input_dim"] = list(input_shape)
    text_net = {k: v for k, v in net.items()}
    text_net["layer"] = [{k: v for k, v in l.items() if k != "blobs"} for l in layers]
    with open(prototxtPath, "w") as f:
        f.write(SCHEMA.to_text("NetParameter", text_net) + "\n")
    with open(modelPath, "wb") as f:
        f.write(SCHEMA.encode("NetParameter", net))
    return module
