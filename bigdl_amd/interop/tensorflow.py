"""TensorFlow GraphDef import / export.

Reference: S/utils/tf/TensorflowLoader.scala:55-616 (parse .pb / .pbtxt, cut the sub-graph between the given
inputs and outputs, build a BigDL Graph; shared weights stay shared), TensorflowToBigDL.scala:41-854 (pattern
conversion of MatMul/Conv2D/BiasAdd/BatchNorm subgraphs with constant weights into trainable layers),
utils/tf/loaders/* (per-op loaders), BigDLToTensorflow.scala:33-483 + TensorflowSaver.scala:36-199 (export),
Tensorflow.scala (const / tensor builders), TFRecordIterator / TFRecordWriter (record files; see
visualization.tensorboard for the framing code shared with event files).

Import strategy:
  * the GraphDef is decoded with the schema codec (interop/protoschema.py) — binary or text;
  * nodes reachable from the requested outputs, stopping at the requested inputs, are kept;
  * constant sub-graphs (Const, Identity/read of constants, shape arithmetic on constants) are folded on the host;
  * MatMul(+BiasAdd/Add) and Conv2D/DepthwiseConv2dNative(+BiasAdd) with constant weights become nn.Linear /
    nn.SpatialConvolution (trainable, GPU implicit-GEMM engine); FusedBatchNorm with constants becomes
    SpatialBatchNormalization; activations / pooling map to nn layers; every other op becomes a TFOp
    (nn/tf_ops.py) with its constant inputs baked in. Weights reached through the same Const/Variable node are
    shared between the converted layers.
"""
import struct

import numpy as np
import torch

from .. import nn
from ..nn.tf_ops import MULTI_OUTPUT, OPS, TF_DTYPES, TFOp, run_op
from ..utils.table import Table
from .protoschema import Schema

_DT = {1: "DT_FLOAT", 2: "DT_DOUBLE", 3: "DT_INT32", 4: "DT_UINT8", 5: "DT_INT16", 6: "DT_INT8", 7: "DT_STRING",
       8: "DT_COMPLEX64", 9: "DT_INT64", 10: "DT_BOOL", 11: "DT_QINT8", 12: "DT_QUINT8", 13: "DT_QINT32",
       14: "DT_BFLOAT16", 15: "DT_QINT16", 16: "DT_QUINT16", 17: "DT_UINT16", 18: "DT_COMPLEX128", 19: "DT_HALF",
       20: "DT_RESOURCE", 21: "DT_VARIANT", 22: "DT_UINT32", 23: "DT_UINT64"}
_DT.update({k + 100: v + "_REF" for k, v in list(_DT.items())})

SCHEMA = Schema(
    {
        "GraphDef": {1: ("node", "msg", "NodeDef"), 3: ("version", "int", None), 4: ("versions", "msg", "VersionDef")},
        "VersionDef": {1: ("producer", "int", None), 2: ("min_consumer", "int", None)},
        "NodeDef": {1: ("name", "string", None), 2: ("op", "string", None), 3: ("input", "string", None),
                    4: ("device", "string", None), 5: ("attr", "msg", "AttrEntry")},
        "AttrEntry": {1: ("key", "string", None), 2: ("value", "msg", "AttrValue")},
        "AttrValue": {1: ("list", "msg", "ListValue"), 2: ("s", "bytes", None), 3: ("i", "int64", None),
                      4: ("f", "float", None), 5: ("b", "bool", None), 6: ("type", "enum", "DataType"),
                      7: ("shape", "msg", "TensorShapeProto"), 8: ("tensor", "msg", "TensorProto"),
                      9: ("placeholder", "string", None), 10: ("func", "msg", "NameAttrList")},
        "ListValue": {2: ("s", "bytes", None), 3: ("i", "int64", None), 4: ("f", "float", None),
                      5: ("b", "bool", None), 6: ("type", "enum", "DataType"), 7: ("shape", "msg", "TensorShapeProto"),
                      8: ("tensor", "msg", "TensorProto")},
        "NameAttrList": {1: ("name", "string", None), 2: ("attr", "msg", "AttrEntry")},
        "TensorShapeProto": {2: ("dim", "msg", "Dim"), 3: ("unknown_rank", "bool", None)},
        "Dim": {1: ("size", "int64", None), 2: ("name", "string", None)},
        "TensorProto": {1: ("dtype", "enum", "DataType"), 2: ("tensor_shape", "msg", "TensorShapeProto"),
                        3: ("version_number", "int", None), 4: ("tensor_content", "bytes", None),
                        5: ("float_val", "float", None), 6: ("double_val", "double", None),
                        7: ("int_val", "int", None), 8: ("string_val", "bytes", None),
                        10: ("int64_val", "int64", None), 11: ("bool_val", "bool", None),
                        13: ("half_val", "int", None)},
    },
    {"DataType": _DT},
)

_NP = {"DT_FLOAT": np.float32, "DT_DOUBLE": np.float64, "DT_INT32": np.int32, "DT_UINT8": np.uint8,
       "DT_INT16": np.int16, "DT_INT8": np.int8, "DT_INT64": np.int64, "DT_BOOL": np.bool_, "DT_HALF": np.float16,
       "DT_UINT16": np.uint16, "DT_UINT32": np.uint32, "DT_UINT64": np.uint64}


# ----------------------------------------------------------------------------------------- parsing
def read_graph(path):
    """GraphDef from a binary .pb or a text .pbtxt file -> list of node dicts."""
    with open(path, "rb") as f:
        data = f.read()
    if path.endswith((".pbtxt", ".txt", ".prototxt")):
        g = SCHEMA.parse_text("GraphDef", data.decode("utf-8"))
    else:
        g = SCHEMA.decode("GraphDef", data)
    return g.get("node", [])


def _first(d, k, default=None):
    v = d.get(k)
    return v[0] if v else default


def attrs_of(node):
    """NodeDef attr map -> python values (tensors for TensorProto, lists for ListValue)."""
    out = {}
    for e in node.get("attr", []):
        k, v = _first(e, "key"), _first(e, "value", {})
        if "list" in v:
            lv = v["list"][0]
            if "i" in lv:
                out[k] = [int(x) for x in lv["i"]]
            elif "f" in lv:
                out[k] = list(lv["f"])
            elif "s" in lv:
                out[k] = [x.decode("utf-8", "replace") for x in lv["s"]]
            elif "type" in lv:
                out[k] = list(lv["type"])
            elif "shape" in lv:
                out[k] = [shape_of(s) for s in lv["shape"]]
            else:
                out[k] = []
        elif "tensor" in v:
            out[k] = tensor_of(v["tensor"][0])
        elif "shape" in v:
            out[k] = shape_of(v["shape"][0])
        elif "type" in v:
            out[k] = v["type"][0]
        elif "s" in v:
            out[k] = v["s"][0].decode("utf-8", "replace")
        elif "i" in v:
            out[k] = int(v["i"][0])
        elif "f" in v:
            out[k] = float(v["f"][0])
        elif "b" in v:
            out[k] = bool(v["b"][0])
        else:
            out[k] = None
    return out


def shape_of(s):
    if _first(s, "unknown_rank", False):
        return None
    return [int(_first(d, "size", 0)) for d in s.get("dim", [])]


def tensor_of(t):
    """TensorProto -> torch tensor (strings -> list of bytes)."""
    dt = _first(t, "dtype", "DT_FLOAT")
    shape = shape_of(_first(t, "tensor_shape", {})) or []
    n = int(np.prod(shape)) if shape else 1
    if dt == "DT_STRING":
        return list(t.get("string_val", []))
    npdt = _NP.get(dt.replace("_REF", ""), np.float32)
    content = _first(t, "tensor_content")
    if content:
        arr = np.frombuffer(content, dtype=npdt).copy()
    else:
        key = {"DT_FLOAT": "float_val", "DT_DOUBLE": "double_val", "DT_INT64": "int64_val", "DT_BOOL": "bool_val",
               "DT_HALF": "half_val"}.get(dt, "int_val")
        vals = t.get(key, [])
        if dt == "DT_HALF":
            arr = np.array(vals, dtype=np.uint16).view(np.float16)
        else:
            arr = np.array(vals, dtype=npdt)
        if arr.size == 0:
            arr = np.zeros(1, dtype=npdt)
        if arr.size < n:                                   # TF repeats the last value to fill the shape
            arr = np.concatenate([arr, np.full(n - arr.size, arr[-1], dtype=npdt)])
    arr = arr.reshape(shape) if shape else arr.reshape(())
    if npdt in (np.uint16, np.uint32, np.uint64):
        arr = arr.astype(np.int64)
    return torch.from_numpy(np.ascontiguousarray(arr))


def _split_ref(ref):
    """'^ctrl' -> (None), 'name:1' -> ('name', 1), 'name' -> ('name', 0)."""
    if ref.startswith("^"):
        return None
    if ":" in ref:
        a, b = ref.rsplit(":", 1)
        if b.isdigit():
            return a, int(b)
    return ref, 0


# ------------------------------------------------------------------------------------------ loading
_ACT = {"Relu": nn.ReLU, "Tanh": nn.Tanh, "Sigmoid": nn.Sigmoid, "Relu6": nn.ReLU6, "Elu": nn.ELU,
        "Softplus": nn.SoftPlus, "Softsign": nn.SoftSign}
_PASSTHROUGH = {"Identity", "StopGradient", "Snapshot", "CheckNumerics"}
_DATA_INPUT_OPS = ("Placeholder", "PlaceholderWithDefault", "QueueDequeueV2", "QueueDequeueManyV2",
                   "QueueDequeueUpToV2", "ReaderReadV2")


class _Loader:
    def __init__(self, nodes, inputs, outputs):
        self.nodes = {n["name"][0]: n for n in nodes}
        self.inputs = [(_split_ref(i)) for i in inputs]
        names = [i[0] for i in self.inputs]
        if len(set(names)) != len(names):
            raise ValueError("duplicate input names")
        for n in names:
            if n not in self.nodes:
                raise ValueError(f"input {n} is not in the graph")
        self.outputs = [_split_ref(o) for o in outputs]
        self.consts = {}          # name -> folded value (tensor / list / Table of outputs)
        self.gnodes = {}          # (name, port) -> graph Node
        self.layer_cache = {}     # shared-weight conversions keyed by the weight node
        self.input_nodes = []
        self.context = {}         # variable name -> value (checkpoint bin file, tf_session.checkpoints)
        self.var_bindings = []    # (variable name, module, attribute, layout) of variables that became parameters

    # -- helpers
    def op(self, name):
        return self.nodes[name]["op"][0]

    def data_inputs(self, name):
        return [r for r in (_split_ref(x) for x in self.nodes[name].get("input", [])) if r is not None]

    def const_value(self, ref):
        """Folded constant for (name, port) or None when the value depends on a graph input."""
        name, port = ref
        if name in self.consts:
            v = self.consts[name]
            return v[port] if isinstance(v, list) else v
        if any(name == i[0] for i in self.inputs):
            return None
        node = self.nodes[name]
        op = self.op(name)
        at = attrs_of(node)
        if op == "Const":
            v = at.get("value")
        elif op in ("VariableV2", "Variable"):
            v = self._variable_init(name)
        elif op in ("Placeholder", "PlaceholderWithDefault"):
            v = None
            if op == "PlaceholderWithDefault":
                v = self.const_value(self.data_inputs(name)[0])
        elif op in OPS and op not in ("RandomUniform", "TruncatedNormal", "RandomStandardNormal", "NoOp"):
            ins = [self.const_value(r) for r in self.data_inputs(name)]
            if any(x is None for x in ins):
                v = None
            else:
                try:
                    r = run_op(op, ins, at)
                except Exception:
                    r = None
                v = list(r) if isinstance(r, (list, tuple)) else r
        else:
            v = None
        self.consts[name] = v
        if isinstance(v, list) and v and isinstance(v[0], torch.Tensor):
            return v[port]
        return v

    def _variable_init(self, name):
        """Value of a VariableV2: the session context (checkpoint) when it holds the name, else the constant of
        its Assign(var, const) initializer, if any."""
        if name in self.context:
            return torch.as_tensor(self.context[name]).clone()
        for n, node in self.nodes.items():
            if self.op(n) == "Assign":
                ins = self.data_inputs(n)
                if ins and ins[0][0] == name:
                    return self.const_value(ins[1])
        return None

    # -- conversion
    def _multi(self, name):
        """Ops whose output is a Table of several tensors (every port, 0 included, is selected from it)."""
        if name not in self.nodes:
            return False
        op = self.op(name)
        if op in MULTI_OUTPUT:
            return True
        if op in ("QueueDequeueV2", "QueueDequeueManyV2", "QueueDequeueUpToV2"):
            return len(attrs_of(self.nodes[name]).get("component_types") or []) > 1
        return False

    def node_for(self, ref):
        name, port = ref
        if (name, port) in self.gnodes:
            return self.gnodes[(name, port)]
        if self._multi(name):
            base = self.gnodes.get((name, "*"))
            if base is None:
                base = self._convert(name)
                self.gnodes[(name, "*")] = base
            sel = nn.SelectTable(port + 1).setName(f"{name}:{port}").inputs(base)
            self.gnodes[(name, port)] = sel
            return sel
        if (name, 0) in self.gnodes and port:
            base = self.gnodes[(name, 0)]
            sel = nn.SelectTable(port + 1).setName(f"{name}:{port}").inputs(base)
            self.gnodes[(name, port)] = sel
            return sel
        node = self._convert(name)
        self.gnodes[(name, 0)] = node
        if port:
            return self.node_for(ref)
        return node

    def _convert(self, name):
        feed = None
        for i, (iname, _) in enumerate(self.inputs):
            if name == iname:
                # placeholders and data-pipeline ops (queue dequeues, readers: Session.scala inputOp) ARE the input
                data_op = self.op(name) in _DATA_INPUT_OPS
                feed = nn.Input(name if data_op else name + "/input")
                self.input_nodes.append((i, feed))
                if data_op:
                    return feed
        op = self.op(name)
        at = attrs_of(self.nodes[name])
        ins = self.data_inputs(name)
        if op in _PASSTHROUGH and len(ins) == 1:
            return self.node_for(ins[0])
        folded = self.const_value((name, 0))
        if folded is not None and op != "Placeholder":
            raise ValueError(f"{name} is constant; it cannot be a graph output or input edge")
        layer = self._layer(name, op, at, ins)
        if layer is not None:
            module, data_refs = layer
        else:
            consts, dyn = {}, []
            for i, r in enumerate(ins):
                c = self.const_value(r)
                if c is not None:
                    consts[i] = c
                else:
                    dyn.append(r)
            module = TFOp(op, at, consts, len(ins))
            data_refs = dyn
        module.setName(name)
        if feed is not None:      # an op named as graph input: the placeholder replaces its data inputs
            return module.inputs(feed)
        preds = [self.node_for(r) for r in data_refs]
        return module.inputs(*preds)

    def _weight(self, ref):
        v = self.const_value(ref)
        return v if isinstance(v, torch.Tensor) and v.is_floating_point() else None

    def _var_of(self, ref):
        """Name of the VariableV2 behind a weight reference (through Identity / 'read' nodes), or None."""
        name = ref[0]
        for _ in range(8):
            if name not in self.nodes:
                return None
            op = self.op(name)
            if op in ("VariableV2", "Variable"):
                return name
            if op not in _PASSTHROUGH:
                return None
            ins = self.data_inputs(name)
            if not ins:
                return None
            name = ins[0][0]
        return None

    def _bind(self, ref, module, attr, layout):
        var = self._var_of(ref)
        if var is not None:
            self.var_bindings.append((var, module, attr, layout))

    def _share(self, layer, key):
        """Layers converted from the same weight node share one weight tensor (reference: shared variables)."""
        first = self.layer_cache.get(key)
        if first is None:
            self.layer_cache[key] = layer
        else:
            layer.weight = first.weight
            layer.gradWeight = first.gradWeight

    def _consumers(self, name):
        return [n for n in self.nodes
                if any((_split_ref(x) or (None,))[0] == name for x in self.nodes[n].get("input", []))]

    def _layer(self, name, op, at, ins):
        if op in ("BiasAdd", "BiasAddV1", "Add", "AddV2") and len(ins) == 2:
            # MatMul / Conv2D with constant weights followed by a constant bias: one layer with bias
            b = self._weight(ins[1])
            src = ins[0][0]
            if (b is not None and b.dim() == 1 and ins[0][1] == 0 and src in self.nodes
                    and self.op(src) in ("MatMul", "Conv2D") and len(self._consumers(src)) == 1
                    and not any(src == i[0] for i in self.inputs)):
                inner = self._layer(src, self.op(src), attrs_of(self.nodes[src]), self.data_inputs(src))
                if inner is not None:
                    layer, refs = inner
                    layer.bias = b.clone().float()
                    layer.gradBias = torch.zeros_like(layer.bias)
                    self._bind(ins[1], layer, "bias", "id")
                    if ("bias", "gradBias") not in layer._params:
                        layer._params.append(("bias", "gradBias"))
                    if hasattr(layer, "withBias"):
                        layer.withBias = True
                    return layer, refs
        if op in _ACT:
            return _ACT[op](), ins[:1]
        if op == "MatMul" and len(ins) == 2:
            w = self._weight(ins[1])
            if w is None or at.get("transpose_a", False):
                return None
            W = w.t() if not at.get("transpose_b", False) else w
            lin = nn.Linear(W.shape[1], W.shape[0], withBias=False)
            lin.weight.data.copy_(W)
            self._share(lin, ("mm", ins[1][0], bool(at.get("transpose_b", False))))
            self._bind(ins[1], lin, "weight", "id" if at.get("transpose_b", False) else "t")
            return lin, ins[:1]
        if op in ("Conv2D",) and len(ins) == 2:
            w = self._weight(ins[1])
            if w is None:
                return None
            fmt = at.get("data_format", "NHWC")
            st = at.get("strides", [1, 1, 1, 1])
            dl = at.get("dilations", [1, 1, 1, 1])
            sh, sw = (st[1], st[2]) if fmt == "NHWC" else (st[2], st[3])
            dh, dw = (dl[1], dl[2]) if fmt == "NHWC" else (dl[2], dl[3])
            kh, kw, cin, cout = w.shape
            pad = -1 if at.get("padding", "VALID") == "SAME" else 0
            conv = nn.SpatialConvolution(cin, cout, kw, kh, sw, sh, pad, pad, withBias=False, format=fmt,
                                         dilationW=dw, dilationH=dh)
            conv.weight.data.copy_(w.permute(3, 2, 0, 1))
            self._share(conv, ("conv", ins[1][0]))
            self._bind(ins[1], conv, "weight", "hwio")
            return conv, ins[:1]
        if op in ("BiasAdd", "BiasAddV1") and len(ins) == 2:
            b = self._weight(ins[1])
            if b is None:
                return None
            fmt = at.get("data_format", "NHWC")
            tb = _TFBias(b, fmt)
            self._bind(ins[1], tb, "bias", "id")
            return tb, ins[:1]
        if op in ("MaxPool", "AvgPool"):
            fmt = at.get("data_format", "NHWC")
            k, s = at["ksize"], at["strides"]
            kh, kw = (k[1], k[2]) if fmt == "NHWC" else (k[2], k[3])
            sh, sw = (s[1], s[2]) if fmt == "NHWC" else (s[2], s[3])
            if at.get("padding", "VALID") == "SAME":
                return None                         # asymmetric TF SAME pooling: TFOp handles it exactly
            if op == "MaxPool":
                return nn.SpatialMaxPooling(kw, kh, sw, sh, 0, 0, format=fmt), ins[:1]
            return nn.SpatialAveragePooling(kw, kh, sw, sh, 0, 0, format=fmt), ins[:1]
        if op in ("FusedBatchNorm", "FusedBatchNormV2", "FusedBatchNormV3") and not at.get("is_training", True):
            vals = [self._weight(r) for r in ins[1:5]]
            if any(v is None for v in vals):
                return None
            fmt = at.get("data_format", "NHWC")
            c = vals[0].numel()
            bn = nn.SpatialBatchNormalization(c, float(at.get("epsilon", 1e-3)), dataFormat=fmt)
            bn.weight.data.copy_(vals[0])
            bn.bias.data.copy_(vals[1])
            bn.runningMean.copy_(vals[2])
            bn.runningVar.copy_(vals[3])
            bn.evaluate()
            return bn, ins[:1]
        return None

    def build(self):
        outs = [self.node_for(o) for o in self.outputs]
        inputs = [n for _, n in sorted(self.input_nodes)]
        if len(inputs) != len(self.inputs):
            missing = set(i[0] for i in self.inputs) - set(n.element.getName() for n in inputs)
            raise ValueError(f"inputs {sorted(missing)} are not connected to the requested outputs")
        return nn.Graph(inputs, outs)


class _TFBias(nn.AutogradModule):
    """BiasAdd with a (trainable) bias vector, NHWC or NCHW."""

    def __init__(self, bias, fmt="NHWC"):
        super().__init__()
        self.fmt = fmt
        self.register_parameter("bias", "gradBias", bias.clone().float())

    def fn(self, x):
        if self.fmt == "NCHW" and x.dim() >= 3:
            return x + self.bias.reshape((1, -1) + (1,) * (x.dim() - 2)).to(x.dtype)
        return x + self.bias.to(x.dtype)


def load_tf(graphFile, inputs, outputs, byteOrder=None, binFile=None, generatedBackward=True):
    """Load a TensorFlow GraphDef into a bigdl_amd Graph (reference TensorflowLoader.load); ``binFile`` (a name ->
    tensor file written by Session.saveParameters) supplies the variable values."""
    nodes = read_graph(graphFile)
    loader = _Loader(nodes, list(inputs), list(outputs))
    if binFile:
        from .tf_session import load_bin

        loader.context = load_bin(binFile)
    return loader.build()


def parse_graph(graphFile):
    """(list of node dicts) — reference TensorflowLoader.parse."""
    return read_graph(graphFile)


# ---------------------------------------------------------------------------------------- exporting
def _attr(key, **kw):
    return {"key": [key], "value": [kw]}


def _tensor_proto(t):
    t = torch.as_tensor(t).detach().cpu().contiguous()
    dt = {torch.float32: "DT_FLOAT", torch.float64: "DT_DOUBLE", torch.int32: "DT_INT32",
          torch.int64: "DT_INT64", torch.bool: "DT_BOOL"}[t.dtype]
    return {"dtype": [dt], "tensor_shape": [{"dim": [{"size": [s]} for s in t.shape]}],
            "tensor_content": [t.numpy().tobytes()]}


class _Saver:
    def __init__(self, fmt):
        self.nodes = []
        self.fmt = fmt
        self.count = 0

    def uniq(self, base):
        self.count += 1
        return f"{base}_{self.count}"

    def const(self, t, name):
        self.nodes.append({"name": [name], "op": ["Const"], "attr": [
            _attr("dtype", type=[_tensor_proto(t)["dtype"][0]]), _attr("value", tensor=[_tensor_proto(t)])]})
        return name

    def node(self, op, name, inputs, **attrs):
        d = {"name": [name], "op": [op], "input": list(inputs), "attr": []}
        for k, v in attrs.items():
            d["attr"].append(_attr(k, **v))
        if "T" not in attrs and op not in ("Placeholder", "Const"):
            d["attr"].append(_attr("T", type=["DT_FLOAT"]))
        self.nodes.append(d)
        return name

    def module(self, m, x):
        """Emit ``m`` applied to tensor name ``x``; returns the output tensor name."""
        name = m.getName() if m.hasName() else self.uniq(type(m).__name__)
        t = type(m).__name__
        if t == "Sequential":
            for c in m.modules:
                x = self.module(c, x)
            return x
        if t == "Linear":
            w = self.const(m.weight.detach().t().contiguous(), name + "/weight")
            y = self.node("MatMul", name + "/matmul", [x, w], transpose_a={"b": [False]}, transpose_b={"b": [False]})
            if m.bias is not None:
                b = self.const(m.bias.detach(), name + "/bias")
                y = self.node("BiasAdd", name, [y, b], data_format={"s": [b"NHWC"]})
            return y
        if t in ("SpatialConvolution", "SpatialShareConvolution"):
            assert m.nGroup == 1, "grouped conv export is not supported"
            w = self.const(m.weight.detach().permute(2, 3, 1, 0).contiguous(), name + "/filter")
            pad = "SAME" if m.padW == -1 else "VALID"
            xin = x
            if pad == "VALID" and (m.padW or m.padH):
                p = self.const(torch.tensor([[0, 0], [m.padH, m.padH], [m.padW, m.padW], [0, 0]], dtype=torch.int32),
                               name + "/paddings")
                xin = self.node("Pad", name + "/pad", [x, p], Tpaddings={"type": ["DT_INT32"]})
            y = self.node("Conv2D", name + "/conv", [xin, w], strides={"list": [{"i": [1, m.strideH, m.strideW, 1]}]},
                          padding={"s": [pad.encode()]}, data_format={"s": [b"NHWC"]},
                          dilations={"list": [{"i": [1, m.dilationH, m.dilationW, 1]}]})
            if m.bias is not None:
                b = self.const(m.bias.detach(), name + "/bias")
                y = self.node("BiasAdd", name, [y, b], data_format={"s": [b"NHWC"]})
            return y
        simple = {"ReLU": "Relu", "Tanh": "Tanh", "Sigmoid": "Sigmoid", "ReLU6": "Relu6", "ELU": "Elu",
                  "SoftPlus": "Softplus", "SoftSign": "Softsign", "Identity": "Identity", "SoftMax": "Softmax",
                  "LogSoftMax": "LogSoftmax", "Abs": "Abs", "Exp": "Exp", "Log": "Log", "Sqrt": "Sqrt",
                  "Square": "Square"}
        if t in simple:
            return self.node(simple[t], name, [x])
        if t in ("SpatialMaxPooling", "SpatialAveragePooling"):
            pad = "SAME" if m.padW == -1 else "VALID"
            return self.node("MaxPool" if t == "SpatialMaxPooling" else "AvgPool", name, [x],
                             ksize={"list": [{"i": [1, m.kH, m.kW, 1]}]},
                             strides={"list": [{"i": [1, m.dH, m.dW, 1]}]}, padding={"s": [pad.encode()]},
                             data_format={"s": [b"NHWC"]})
        if t in ("Reshape", "InferReshape", "View"):
            size = list(getattr(m, "size", getattr(m, "sizes", [])))
            shape = self.const(torch.tensor([-1] + [int(s) for s in size], dtype=torch.int32), name + "/shape")
            return self.node("Reshape", name, [x, shape], Tshape={"type": ["DT_INT32"]})
        if t in ("SpatialBatchNormalization", "BatchNormalization"):
            c = [self.const(v.detach().float(), f"{name}/{k}") for k, v in
                 (("scale", m.weight), ("offset", m.bias), ("mean", m.runningMean), ("variance", m.runningVar))]
            return self.node("FusedBatchNorm", name, [x] + c, epsilon={"f": [float(m.eps)]},
                             is_training={"b": [False]}, data_format={"s": [b"NHWC"]})
        if t == "Dropout":
            return x
        raise NotImplementedError(f"export of {t} to TensorFlow is not supported")


def save_tf(model, inputs, path, byteOrder=None, dataFormat="NHWC"):
    """Export a (Sequential) model to a frozen GraphDef (reference TensorflowSaver.saveGraph). ``inputs`` is a list of
    (name, shape) pairs; image models are exported NHWC. Returns the output tensor name."""
    s = _Saver(dataFormat)
    (iname, ishape), = inputs
    s.node("Placeholder", iname, [], dtype={"type": ["DT_FLOAT"]},
           shape={"shape": [{"dim": [{"size": [d if d is not None else -1]} for d in ishape]}]})
    out = s.module(model, iname)
    g = {"node": s.nodes, "versions": [{"producer": [21]}]}
    data = SCHEMA.encode("GraphDef", g)
    with open(path, "wb") as f:
        f.write(data)
    return out


def freeze_graph_with_variables(graph_file, values, output_node_names, output_graph):
    """Replace every variable node (VariableV2 / Variable / VarHandleOp) named in ``values`` by a Const holding that
    value, drop the nodes the outputs do not depend on (Assign / initialisers / savers) and write a binary GraphDef:
    the freezing step of the reference tf_utils.merge_checkpoint, without TensorFlow."""
    nodes = read_graph(graph_file)
    by_name = {_first(n, "name"): n for n in nodes}
    keep, stack = set(), [o.split(":")[0] for o in output_node_names]
    while stack:
        nm = stack.pop()
        if nm in keep or nm not in by_name:
            continue
        keep.add(nm)
        if _first(by_name[nm], "op") in ("VariableV2", "Variable", "VarHandleOp") and nm in values:
            continue
        for i in by_name[nm].get("input", []):
            stack.append(i.lstrip("^").split(":")[0])
    out = []
    for n in nodes:
        nm = _first(n, "name")
        if nm not in keep:
            continue
        if _first(n, "op") in ("VariableV2", "Variable", "VarHandleOp") and nm in values:
            t = torch.as_tensor(values[nm])
            tp = _tensor_proto(t)
            n = {"name": [nm], "op": ["Const"], "attr": [_attr("dtype", type=[tp["dtype"][0]]),
                                                          _attr("value", tensor=[tp])]}
        out.append(n)
    with open(output_graph, "wb") as f:
        f.write(SCHEMA.encode("GraphDef", {"node": out, "versions": [{"producer": [21]}]}))
    return output_graph


__all__ = ["load_tf", "save_tf", "read_graph", "freeze_graph_with_variables", "parse_graph", "attrs_of", "tensor_of", "SCHEMA", "TensorflowLoader",
           "TensorflowSaver", "TensorflowToBigDL", "BigDLToTensorflow"]


class Session:
    """Train / run an imported TensorFlow graph (reference utils/tf/Session.scala BigDLSessionImpl): placeholder-fed
    training on a DataSet, or queue-fed training / prediction over the graph's own input pipeline
    (interop/tf_session.py)."""

    def __init__(self, graphFile, inputs=None, context=None):
        from .tf_session import BigDLSession

        self._s = BigDLSession(graphFile, inputs, context)
        self.graphFile, self.inputs = graphFile, list(inputs or [])

    def train(self, outputs, dataset=None, optMethod=None, criterion=None, endWhen=None, batchSize=None,
              isDataBatch=False, loss=None):
        return self._s.train(outputs, dataset, optMethod, criterion, endWhen, batchSize, isDataBatch, loss)

    def predict(self, outputs, x=None, isDataBatch=False, batchSize=32):
        if x is None:
            return self._s.predict(outputs, isDataBatch, batchSize)
        model = load_tf(self.graphFile, self.inputs, outputs)
        model.evaluate()
        with torch.no_grad():
            return model.forward(x)

    def saveParameters(self, binFile):
        self._s.saveParameters(binFile)
        return self

    def variables(self):
        return self._s.variables()


class TensorflowLoader:
    """Reference S/utils/tf/TensorflowLoader.scala:55 ``load(graphFile, inputs, outputs, byteOrder, binFile)``,
    :88 ``checkpoints(graphFile, binFile)``."""

    load = staticmethod(load_tf)
    parse = staticmethod(parse_graph)

    @staticmethod
    def checkpoints(graphFile, binFile, byteOrder=None):
        from .tf_session import checkpoints

        s = Session.__new__(Session)
        s._s = checkpoints(graphFile, binFile)
        s.graphFile, s.inputs = graphFile, []
        return s


class TensorflowSaver:
    """Reference S/utils/tf/TensorflowSaver.scala:36 ``saveGraph(model, inputs, path, byteOrder, dataFormat)``."""

    @staticmethod
    def saveGraph(model, inputs, path, byteOrder=None, dataFormat="NHWC"):
        return save_tf(model, inputs, path, byteOrder, dataFormat)


TensorflowToBigDL = TensorflowLoader     # op-by-op conversion lives in the loader (TensorflowToBigDL.scala:41)
BigDLToTensorflow = TensorflowSaver      # module-by-module emission lives in the saver (BigDLToTensorflow.scala:33)
