"""ONNX model import / export.

Reference: P/contrib/onnx/onnx_loader.py:24-110 (walk graph nodes, initializers become constants),
ops_converter.py / ops_mapping.py (Constant, Sum, Concat, Relu, Conv, BatchNormalization, Softmax, Gemm,
Reshape, Unsqueeze, AveragePool, MaxPool, Shape, Gather), S/nn/onnx/{Gemm, Reshape, Shape}.scala.

The onnx python package is not needed: ModelProto is decoded with the schema codec (interop/protoschema.py).
Conv / ConvTranspose / Gemm / MatMul / BatchNormalization with initializer weights become trainable nn layers
(GPU engine); other ops map to nn layers or to OnnxOp, a TF-op-style module with ONNX semantics. The importer
accepts opset 7-13 attribute / input conventions (e.g. Reshape shape as input, Unsqueeze axes as attr or input).
"""
import numpy as np
import torch
import torch.nn.functional as F

from .. import nn
from ..nn.tf_ops import run_op
from ..utils.table import Table
from .protoschema import Schema

_ONNX_DT = {1: "FLOAT", 2: "UINT8", 3: "INT8", 4: "UINT16", 5: "INT16", 6: "INT32", 7: "INT64", 8: "STRING",
            9: "BOOL", 10: "FLOAT16", 11: "DOUBLE", 12: "UINT32", 13: "UINT64", 16: "BFLOAT16"}
_NP = {1: np.float32, 2: np.uint8, 3: np.int8, 4: np.uint16, 5: np.int16, 6: np.int32, 7: np.int64, 9: np.bool_,
       10: np.float16, 11: np.float64, 12: np.uint32, 13: np.uint64}

SCHEMA = Schema(
    {
        "ModelProto": {1: ("ir_version", "int64", None), 2: ("producer_name", "string", None),
                       3: ("producer_version", "string", None), 4: ("domain", "string", None),
                       5: ("model_version", "int64", None), 6: ("doc_string", "string", None),
                       7: ("graph", "msg", "GraphProto"), 8: ("opset_import", "msg", "OperatorSetIdProto")},
        "OperatorSetIdProto": {1: ("domain", "string", None), 2: ("version", "int64", None)},
        "GraphProto": {1: ("node", "msg", "NodeProto"), 2: ("name", "string", None),
                       5: ("initializer", "msg", "TensorProto"), 10: ("doc_string", "string", None),
                       11: ("input", "msg", "ValueInfoProto"), 12: ("output", "msg", "ValueInfoProto"),
                       13: ("value_info", "msg", "ValueInfoProto")},
        "NodeProto": {1: ("input", "string", None), 2: ("output", "string", None), 3: ("name", "string", None),
                      4: ("op_type", "string", None), 5: ("attribute", "msg", "AttributeProto"),
                      6: ("doc_string", "string", None), 7: ("domain", "string", None)},
        "AttributeProto": {1: ("name", "string", None), 2: ("f", "float", None), 3: ("i", "int64", None),
                           4: ("s", "bytes", None), 5: ("t", "msg", "TensorProto"), 6: ("g", "msg", "GraphProto"),
                           7: ("floats", "float", None), 8: ("ints", "int64", None), 9: ("strings", "bytes", None),
                           10: ("tensors", "msg", "TensorProto"), 20: ("type", "int", None)},
        "TensorProto": {1: ("dims", "int64", None), 2: ("data_type", "int", None), 4: ("float_data", "float", None),
                        5: ("int32_data", "int", None), 6: ("string_data", "bytes", None),
                        7: ("int64_data", "int64", None), 8: ("name", "string", None), 9: ("raw_data", "bytes", None),
                        10: ("double_data", "double", None), 11: ("uint64_data", "uint64", None)},
        "ValueInfoProto": {1: ("name", "string", None), 2: ("type", "msg", "TypeProto")},
        "TypeProto": {1: ("tensor_type", "msg", "TypeTensor")},
        "TypeTensor": {1: ("elem_type", "int", None), 2: ("shape", "msg", "ShapeProto")},
        "ShapeProto": {1: ("dim", "msg", "Dimension")},
        "Dimension": {1: ("dim_value", "int64", None), 2: ("dim_param", "string", None)},
    },
    {},
)


def _first(d, k, default=None):
    v = d.get(k)
    return v[0] if v else default


def tensor_of(t):
    dt = _first(t, "data_type", 1)
    dims = [int(d) for d in t.get("dims", [])]
    npdt = _NP.get(dt, np.float32)
    raw = _first(t, "raw_data")
    if raw:
        arr = np.frombuffer(raw, dtype=npdt).copy()
    else:
        key = {1: "float_data", 11: "double_data", 7: "int64_data", 13: "uint64_data", 12: "uint64_data"}.get(
            dt, "int32_data")
        arr = np.array(t.get(key, []), dtype=npdt if key != "int32_data" else np.int64).astype(npdt)
    arr = arr.reshape(dims) if dims else arr.reshape(())
    if npdt in (np.uint16, np.uint32, np.uint64):
        arr = arr.astype(np.int64)
    return torch.from_numpy(np.ascontiguousarray(arr))


def attrs_of(node):
    out = {}
    for a in node.get("attribute", []):
        name = _first(a, "name")
        if "ints" in a:
            out[name] = [int(v) for v in a["ints"]]
        elif "floats" in a:
            out[name] = list(a["floats"])
        elif "t" in a:
            out[name] = tensor_of(a["t"][0])
        elif "s" in a:
            out[name] = a["s"][0].decode("utf-8", "replace")
        elif "strings" in a:
            out[name] = [s.decode("utf-8", "replace") for s in a["strings"]]
        elif "i" in a:
            out[name] = int(a["i"][0])
        elif "f" in a:
            out[name] = float(a["f"][0])
        else:
            out[name] = None
    return out


# ----------------------------------------------------------------------------------------- op table
def _onnx_reshape(x, at):
    t, shape = x[0], [int(v) for v in x[1].reshape(-1).tolist()]
    shape = [t.shape[i] if s == 0 else s for i, s in enumerate(shape)]
    return t.reshape(shape)


def _axes(at, x, idx=1):
    if "axes" in at:
        return list(at["axes"])
    if len(x) > idx and x[idx] is not None:
        return [int(v) for v in x[idx].reshape(-1).tolist()]
    return None


def _unsqueeze(x, at):
    t = x[0]
    for a in sorted(_axes(at, x)):
        t = t.unsqueeze(a if a >= 0 else a + t.dim() + 1)
    return t


def _squeeze(x, at):
    ax = _axes(at, x)
    t = x[0]
    if ax is None:
        return t.squeeze()
    for a in sorted([a + t.dim() if a < 0 else a for a in ax], reverse=True):
        t = t.squeeze(a)
    return t


def _reduce(fn):
    def run(x, at):
        ax = _axes(at, x)
        keep = bool(at.get("keepdims", 1))
        t = x[0]
        ax = list(range(t.dim())) if ax is None else [a + t.dim() if a < 0 else a for a in ax]
        return fn(t, ax, keep)
    return run


def _flatten(x, at):
    a = int(at.get("axis", 1))
    t = x[0]
    a = a + t.dim() if a < 0 else a
    return t.reshape(int(np.prod(t.shape[:a])) if a else 1, -1)


def _gather(x, at):
    t, idx = x[0], x[1].long()
    a = int(at.get("axis", 0))
    a = a + t.dim() if a < 0 else a
    idx = torch.where(idx < 0, idx + t.shape[a], idx)
    return t.index_select(a, idx.reshape(-1)).reshape(t.shape[:a] + idx.shape + t.shape[a + 1:])


def _concat(x, at):
    return torch.cat(list(x), dim=int(at.get("axis", 0)))


def _slice(x, at):
    t = x[0]
    if len(x) >= 3:
        starts, ends = x[1].reshape(-1).tolist(), x[2].reshape(-1).tolist()
        axes = x[3].reshape(-1).tolist() if len(x) > 3 and x[3] is not None else list(range(len(starts)))
        steps = x[4].reshape(-1).tolist() if len(x) > 4 and x[4] is not None else [1] * len(starts)
    else:
        starts, ends = at["starts"], at["ends"]
        axes = at.get("axes", list(range(len(starts))))
        steps = [1] * len(starts)
    idx = [slice(None)] * t.dim()
    for s, e, a, st in zip(starts, ends, axes, steps):
        n = t.shape[a]
        s = max(min(s + n if s < 0 else s, n), 0)
        e = max(min(e + n if e < 0 else e, n), 0)
        idx[a] = slice(int(s), int(e), int(st))
    return t[tuple(idx)]


def _clip(x, at):
    lo = x[1] if len(x) > 1 and x[1] is not None else at.get("min", float("-inf"))
    hi = x[2] if len(x) > 2 and x[2] is not None else at.get("max", float("inf"))
    lo = float(lo) if not isinstance(lo, torch.Tensor) else float(lo.reshape(-1)[0])
    hi = float(hi) if not isinstance(hi, torch.Tensor) else float(hi.reshape(-1)[0])
    return x[0].clamp(lo, hi)


def _softmax(log):
    def run(x, at):
        a = int(at.get("axis", -1 if at.get("_opset", 13) >= 13 else 1))
        t = x[0]
        if at.get("_opset", 13) < 13 and t.dim() > 2:        # legacy: coerce to 2-D at axis
            a = a + t.dim() if a < 0 else a
            flat = t.reshape(int(np.prod(t.shape[:a])), -1)
            y = torch.log_softmax(flat, 1) if log else torch.softmax(flat, 1)
            return y.reshape(t.shape)
        return torch.log_softmax(t, a) if log else torch.softmax(t, a)
    return run


def _pad(x, at):
    pads = [int(v) for v in (x[1].reshape(-1).tolist() if len(x) > 1 and x[1] is not None else at["pads"])]
    value = float(x[2].reshape(-1)[0]) if len(x) > 2 and x[2] is not None else float(at.get("value", 0.0))
    n = len(pads) // 2
    tp = []
    for i in reversed(range(n)):
        tp += [pads[i], pads[i + n]]
    mode = at.get("mode", "constant")
    return F.pad(x[0], tp, mode="constant" if mode == "constant" else ("reflect" if mode == "reflect" else "replicate"),
                 value=value) if mode == "constant" else F.pad(x[0], tp, mode="reflect" if mode == "reflect" else "replicate")


OPS = {
    "Add": lambda x, at: x[0] + x[1], "Sub": lambda x, at: x[0] - x[1], "Mul": lambda x, at: x[0] * x[1],
    "Div": lambda x, at: x[0] / x[1] if x[0].is_floating_point() else torch.div(x[0], x[1], rounding_mode="trunc"),
    "Pow": lambda x, at: torch.pow(x[0], x[1]), "Sum": lambda x, at: sum(x[1:], x[0]),
    "Mean": lambda x, at: sum(x[1:], x[0]) / len(x), "Max": lambda x, at: torch.stack(list(x)).amax(0),
    "Min": lambda x, at: torch.stack(list(x)).amin(0), "Abs": lambda x, at: x[0].abs(),
    "Neg": lambda x, at: -x[0], "Exp": lambda x, at: x[0].exp(), "Log": lambda x, at: x[0].log(),
    "Sqrt": lambda x, at: x[0].sqrt(), "Reciprocal": lambda x, at: x[0].reciprocal(),
    "Ceil": lambda x, at: x[0].ceil(), "Floor": lambda x, at: x[0].floor(), "Tanh": lambda x, at: x[0].tanh(),
    "Sigmoid": lambda x, at: x[0].sigmoid(), "Relu": lambda x, at: x[0].relu(),
    "LeakyRelu": lambda x, at: F.leaky_relu(x[0], float(at.get("alpha", 0.01))),
    "Elu": lambda x, at: F.elu(x[0], float(at.get("alpha", 1.0))), "Selu": lambda x, at: F.selu(x[0]),
    "Softplus": lambda x, at: F.softplus(x[0]), "Softsign": lambda x, at: F.softsign(x[0]),
    "HardSigmoid": lambda x, at: (float(at.get("alpha", 0.2)) * x[0] + float(at.get("beta", 0.5))).clamp(0, 1),
    "Clip": _clip, "Identity": lambda x, at: x[0], "Dropout": lambda x, at: x[0],
    "Softmax": _softmax(False), "LogSoftmax": _softmax(True),
    "Reshape": _onnx_reshape, "Flatten": _flatten, "Unsqueeze": _unsqueeze, "Squeeze": _squeeze,
    "Transpose": lambda x, at: x[0].permute(*(at.get("perm") or list(reversed(range(x[0].dim()))))),
    "Concat": _concat, "Gather": _gather, "Slice": _slice, "Pad": _pad,
    "Shape": lambda x, at: torch.tensor(list(x[0].shape), dtype=torch.int64),
    "Cast": lambda x, at: x[0].to({1: torch.float32, 6: torch.int32, 7: torch.int64, 9: torch.bool,
                                   11: torch.float64}.get(int(at.get("to", 1)), torch.float32)),
    "ReduceMean": _reduce(lambda t, a, k: t.mean(dim=a, keepdim=k)),
    "ReduceSum": _reduce(lambda t, a, k: t.sum(dim=a, keepdim=k)),
    "ReduceMax": _reduce(lambda t, a, k: t.amax(dim=a, keepdim=k)),
    "ReduceMin": _reduce(lambda t, a, k: t.amin(dim=a, keepdim=k)),
    "ReduceProd": _reduce(lambda t, a, k: t.prod(dim=a[0], keepdim=k) if len(a) == 1 else t.prod()),
    "GlobalAveragePool": lambda x, at: x[0].mean(dim=tuple(range(2, x[0].dim())), keepdim=True),
    "GlobalMaxPool": lambda x, at: x[0].amax(dim=tuple(range(2, x[0].dim())), keepdim=True),
    "MatMul": lambda x, at: x[0] @ x[1],
    "Equal": lambda x, at: x[0] == x[1], "Greater": lambda x, at: x[0] > x[1], "Less": lambda x, at: x[0] < x[1],
    "Not": lambda x, at: ~x[0].bool(), "Where": lambda x, at: torch.where(x[0].bool(), x[1], x[2]),
    "ArgMax": lambda x, at: torch.argmax(x[0], dim=int(at.get("axis", 0)), keepdim=bool(at.get("keepdims", 1))),
    "ArgMin": lambda x, at: torch.argmin(x[0], dim=int(at.get("axis", 0)), keepdim=bool(at.get("keepdims", 1))),
    "Expand": lambda x, at: x[0] * torch.ones([int(v) for v in x[1].reshape(-1).tolist()], dtype=x[0].dtype),
    "ConstantOfShape": lambda x, at: torch.full([int(v) for v in x[0].reshape(-1).tolist()],
                                                float(at["value"].reshape(-1)[0]) if "value" in at else 0.0),
    "Split": lambda x, at: list(torch.split(x[0], at["split"] if "split" in at else
                                            (x[0].shape[int(at.get("axis", 0))] // 2), dim=int(at.get("axis", 0)))),
}


class OnnxOp(nn.AutogradModule):
    """One ONNX op with constant inputs baked in (cf. nn.tf_ops.TFOp)."""

    def __init__(self, op, attrs=None, consts=None, n_inputs=None):
        super().__init__()
        if op not in OPS:
            raise NotImplementedError(f"ONNX op {op} is not supported")
        self.op, self.attrs, self.n_inputs = op, dict(attrs or {}), n_inputs
        self.const_pos = sorted((consts or {}).keys())
        self._buffers = []
        for p in self.const_pos:
            setattr(self, f"const{p}", consts[p])
            self._buffers.append(f"const{p}")

    def fn(self, x):
        dyn = [] if x is None else ([x[i + 1] for i in range(x.length())] if isinstance(x, Table) else [x])
        n = self.n_inputs if self.n_inputs is not None else len(dyn) + len(self.const_pos)
        it, ins = iter(dyn), []
        for i in range(n):
            if i in self.const_pos:
                c = getattr(self, f"const{i}")
                ins.append(c.to(dyn[0].device) if dyn and isinstance(c, torch.Tensor) else c)
            else:
                ins.append(next(it))
        r = OPS[self.op](ins, self.attrs)
        if isinstance(r, list):
            t = Table()
            for i, v in enumerate(r):
                t[i + 1] = v
            return t
        return r

    def __repr__(self):
        return f"OnnxOp[{self.op}]"


# ----------------------------------------------------------------------------------------- importer
def _pads2(at, k):
    p = at.get("pads", [0] * (2 * k))
    return p[:k], p[k:]


def load_onnx(path):
    """ONNX file -> bigdl_amd Graph (reference onnx_loader.load)."""
    with open(path, "rb") as f:
        return load_onnx_bytes(f.read())


def load_onnx_bytes(data):
    """Serialized ModelProto bytes -> bigdl_amd Graph (reference onnx_loader.load_model_proto)."""
    model = SCHEMA.decode("ModelProto", bytes(data))
    opset = max([int(_first(o, "version", 13)) for o in model.get("opset_import", [])] or [13])
    g = model["graph"][0]
    inits = {_first(t, "name"): tensor_of(t) for t in g.get("initializer", [])}
    consts = dict(inits)
    producers = {}
    nodes = g.get("node", [])
    for n in nodes:
        for o in n.get("output", []):
            producers[o] = n
    graph_inputs = [_first(v, "name") for v in g.get("input", []) if _first(v, "name") not in inits]
    gnodes = {}
    input_nodes = []

    def const(name):
        if name == "":
            return None
        if name in consts:
            return consts[name]
        n = producers.get(name)
        if n is None:
            return None
        op = _first(n, "op_type")
        at = attrs_of(n)
        at["_opset"] = opset
        if op == "Constant":
            v = at.get("value")
        elif op in OPS:
            ins = [const(i) for i in n.get("input", [])]
            if any(v is None for v, nm in zip(ins, n.get("input", [])) if nm != ""):
                v = None
            else:
                try:
                    r = OPS[op](ins, at)
                    v = r[n["output"].index(name)] if isinstance(r, list) else r
                except Exception:
                    v = None
        else:
            v = None
        if v is not None:
            consts[name] = v
        return v

    def node_for(name):
        if name in gnodes:
            return gnodes[name]
        if name in graph_inputs:
            nd = nn.Input(name)
            input_nodes.append((graph_inputs.index(name), nd))
            gnodes[name] = nd
            return nd
        n = producers[name]
        outs = n.get("output", [])
        if len(outs) > 1 and name != outs[0]:
            base = node_for(outs[0])
            sel = nn.SelectTable(outs.index(name) + 1).inputs(base)
            gnodes[name] = sel
            return sel
        op = _first(n, "op_type")
        at = attrs_of(n)
        at["_opset"] = opset
        ins = list(n.get("input", []))
        module, data = _layer(op, at, ins, const)
        if module is None:
            cst, dyn = {}, []
            for i, nm in enumerate(ins):
                v = const(nm) if nm else None
                if v is not None or nm == "":
                    cst[i] = v
                else:
                    dyn.append(nm)
            module, data = OnnxOp(op, {k: v for k, v in at.items()}, cst, len(ins)), dyn
        module.setName(_first(n, "name") or name)
        nd = module.inputs(*[node_for(d) for d in data])
        gnodes[name] = nd
        return nd

    outs = [node_for(_first(v, "name")) for v in g.get("output", [])]
    ins = [n for _, n in sorted(input_nodes, key=lambda p: p[0])]
    return nn.Graph(ins, outs)


def _layer(op, at, ins, const):
    """Trainable / native-layer conversions. Returns (module, data input names) or (None, None)."""
    if op in ("Conv",) and const(ins[1]) is not None:
        w = const(ins[1]).float()
        b = const(ins[2]).float() if len(ins) > 2 and ins[2] else None
        if w.dim() != 4:
            return None, None
        cout, cin_g, kh, kw = w.shape
        g = int(at.get("group", 1))
        st = at.get("strides", [1, 1])
        dl = at.get("dilations", [1, 1])
        auto = at.get("auto_pad", "NOTSET")
        if auto in ("SAME_UPPER", "SAME_LOWER"):
            ph = pw = -1
        else:
            (pt, pl), (pb, pr) = _pads2(at, 2)
            if pt != pb or pl != pr:
                return None, None
            ph, pw = pt, pl
        conv = nn.SpatialConvolution(cin_g * g, cout, kw, kh, st[1], st[0], pw, ph, nGroup=g, withBias=b is not None,
                                     dilationW=dl[1], dilationH=dl[0])
        conv.weight.data.copy_(w)
        if b is not None:
            conv.bias.data.copy_(b)
        return conv, [ins[0]]
    if op == "Gemm" and const(ins[1]) is not None and not at.get("transA", 0):
        w = const(ins[1]).float()
        W = w if at.get("transB", 0) else w.t()
        alpha, beta = float(at.get("alpha", 1.0)), float(at.get("beta", 1.0))
        c = const(ins[2]) if len(ins) > 2 and ins[2] else None
        lin = nn.Linear(W.shape[1], W.shape[0], withBias=c is not None)
        lin.weight.data.copy_(W * alpha)
        if c is not None:
            lin.bias.data.copy_((c.float() * beta).expand(W.shape[0]))
        return lin, [ins[0]]
    if op == "MatMul" and const(ins[1]) is not None and const(ins[1]).dim() == 2:
        w = const(ins[1]).float()
        lin = nn.Linear(w.shape[0], w.shape[1], withBias=False)
        lin.weight.data.copy_(w.t())
        return lin, [ins[0]]
    if op == "BatchNormalization" and all(const(i) is not None for i in ins[1:5]):
        s, b, m, v = [const(i).float() for i in ins[1:5]]
        bn = nn.SpatialBatchNormalization(s.numel(), float(at.get("epsilon", 1e-5)), 1.0 - float(at.get("momentum", 0.9)))
        bn.weight.data.copy_(s)
        bn.bias.data.copy_(b)
        bn.runningMean.copy_(m)
        bn.runningVar.copy_(v)
        bn.evaluate()
        return bn, [ins[0]]
    if op in ("MaxPool", "AveragePool") and len(at.get("kernel_shape", [])) == 2:
        kh, kw = at["kernel_shape"]
        st = at.get("strides", [1, 1])
        (pt, pl), (pb, pr) = _pads2(at, 2)
        if pt != pb or pl != pr or at.get("auto_pad", "NOTSET") not in ("NOTSET", "VALID"):
            return None, None
        ceil = bool(at.get("ceil_mode", 0))
        if op == "MaxPool":
            m = nn.SpatialMaxPooling(kw, kh, st[1], st[0], pl, pt)
            if ceil:
                m.ceil()
            return m, [ins[0]]
        return nn.SpatialAveragePooling(kw, kh, st[1], st[0], pl, pt, ceilMode=ceil,
                                        countIncludePad=bool(at.get("count_include_pad", 0))), [ins[0]]
    simple = {"Relu": nn.ReLU, "Tanh": nn.Tanh, "Sigmoid": nn.Sigmoid}
    if op in simple:
        return simple[op](), [ins[0]]
    return None, None


# ----------------------------------------------------------------------------------------- exporter
def _tp(name, t):
    t = torch.as_tensor(t).detach().cpu().contiguous()
    code = {torch.float32: 1, torch.int64: 7, torch.int32: 6, torch.float64: 11}[t.dtype]
    return {"name": [name], "dims": list(t.shape), "data_type": [code], "raw_data": [t.numpy().tobytes()]}


def _attr_i(name, v):
    return {"name": [name], "i": [int(v)], "type": [2]}


def _attr_ints(name, v):
    return {"name": [name], "ints": [int(x) for x in v], "type": [7]}


def _attr_f(name, v):
    return {"name": [name], "f": [float(v)], "type": [1]}


def save_onnx(model, input_shape, path, input_name="input", opset=11):
    """Export a Sequential of common layers (NCHW) to an ONNX file. Returns the output name."""
    nodes, inits = [], []
    state = {"n": 0}

    def uniq(b):
        state["n"] += 1
        return f"{b}_{state['n']}"

    def emit(m, x):
        t = type(m).__name__
        name = uniq(t)
        if t == "Sequential":
            for c in m.modules:
                x = emit(c, x)
            return x
        if t in ("SpatialConvolution", "SpatialShareConvolution"):
            wn, out = name + "_W", name + "_out"
            inits.append(_tp(wn, m.weight))
            ins = [x, wn]
            if m.bias is not None:
                inits.append(_tp(name + "_B", m.bias))
                ins.append(name + "_B")
            at = [_attr_ints("kernel_shape", [m.kernelH, m.kernelW]), _attr_ints("strides", [m.strideH, m.strideW]),
                  _attr_ints("dilations", [m.dilationH, m.dilationW]), _attr_i("group", m.nGroup)]
            if m.padW == -1:
                at.append({"name": ["auto_pad"], "s": [b"SAME_UPPER"], "type": [3]})
            else:
                at.append(_attr_ints("pads", [m.padH, m.padW, m.padH, m.padW]))
            nodes.append({"input": ins, "output": [out], "name": [name], "op_type": ["Conv"], "attribute": at})
            return out
        if t == "Linear":
            wn, out = name + "_W", name + "_out"
            inits.append(_tp(wn, m.weight))
            ins = [x, wn]
            if m.bias is not None:
                inits.append(_tp(name + "_B", m.bias))
                ins.append(name + "_B")
            nodes.append({"input": ins, "output": [out], "name": [name], "op_type": ["Gemm"],
                          "attribute": [_attr_i("transB", 1)]})
            return out
        if t in ("SpatialBatchNormalization", "BatchNormalization"):
            names = [f"{name}_{k}" for k in ("scale", "B", "mean", "var")]
            for nm, v in zip(names, (m.weight, m.bias, m.runningMean, m.runningVar)):
                inits.append(_tp(nm, v.float()))
            out = name + "_out"
            nodes.append({"input": [x] + names, "output": [out], "name": [name], "op_type": ["BatchNormalization"],
                          "attribute": [_attr_f("epsilon", m.eps)]})
            return out
        if t in ("SpatialMaxPooling", "SpatialAveragePooling"):
            out = name + "_out"
            op = "MaxPool" if t == "SpatialMaxPooling" else "AveragePool"
            nodes.append({"input": [x], "output": [out], "name": [name], "op_type": [op], "attribute": [
                _attr_ints("kernel_shape", [m.kH, m.kW]), _attr_ints("strides", [m.dH, m.dW]),
                _attr_ints("pads", [m.padH, m.padW, m.padH, m.padW])]})
            return out
        simple = {"ReLU": "Relu", "Tanh": "Tanh", "Sigmoid": "Sigmoid", "SoftMax": "Softmax", "Identity": "Identity",
                  "Dropout": "Identity", "LogSoftMax": "LogSoftmax"}
        if t in simple:
            out = name + "_out"
            at = [_attr_i("axis", 1)] if t in ("SoftMax", "LogSoftMax") else []
            nodes.append({"input": [x], "output": [out], "name": [name], "op_type": [simple[t]], "attribute": at})
            return out
        if t in ("Reshape", "View", "InferReshape"):
            sn, out = name + "_shape", name + "_out"
            inits.append(_tp(sn, torch.tensor([0] + [int(s) for s in m.size], dtype=torch.int64)))
            nodes.append({"input": [x, sn], "output": [out], "name": [name], "op_type": ["Reshape"]})
            return out
        raise NotImplementedError(f"ONNX export of {t} is not supported")

    out = emit(model, input_name)
    shape = {"dim": [{"dim_value": [d]} if d is not None else {"dim_param": ["N"]} for d in input_shape]}
    graph = {"node": nodes, "name": ["bigdl_amd"], "initializer": inits,
             "input": [{"name": [input_name], "type": [{"tensor_type": [{"elem_type": [1], "shape": [shape]}]}]}],
             "output": [{"name": [out], "type": [{"tensor_type": [{"elem_type": [1]}]}]}]}
    mp = {"ir_version": [6], "producer_name": ["bigdl_amd"], "graph": [graph],
          "opset_import": [{"domain": [""], "version": [opset]}]}
    with open(path, "wb") as f:
        f.write(SCHEMA.encode("ModelProto", mp))
    return out


__all__ = ["load_onnx", "load_onnx_bytes", "save_onnx", "OnnxOp", "SCHEMA"]
