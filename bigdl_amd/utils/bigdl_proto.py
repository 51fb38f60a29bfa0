"""BigDL's native protobuf model format (``bigdl.proto``): read and write ``BigDLModule`` files.

Reference: RES/serialization/bigdl.proto:4-182 (BigDLModule / BigDLTensor / TensorStorage / AttrValue),
S/utils/serializer/ModuleSerializable.scala:60-480 (module type = the Scala class name, one attribute per primary
constructor parameter, ``module_tags`` / ``module_numerics``, ``hasParameters`` + ``parameters``),
S/utils/serializer/ModuleLoader.scala:47-140 / :230-327 (``global_storage``: every tensor's storage is written
once, in the root module's attributes, and parameters reference it by id; the optional separate weight file:
magic 3721, storages, MD5 digest), S/utils/serializer/converters/TensorConverter.scala (1-based storage offsets,
sizes / strides), S/nn/Graph.scala:663-730 (``inputNames`` / ``outputNames`` / ``<node>_edges`` and the
``preModules`` of each sub-module), S/nn/BatchNormalization.scala:376-410 (``runningMean`` / ``runningVar``).

Mapping onto the engine: every module records its constructor arguments (``_init_args``), which are bound to the
constructor's parameter names — the engine keeps the Scala parameter names — and written as typed AttrValues;
loading looks the class up by its Scala simple name and calls the constructor with the attributes it accepts.
Python floats are written as DOUBLE (the Scala side's Float-typed parameters are not distinguishable here);
parity with files written by the reference JVM is pinned to the .proto field layout only: the reference ships no
``.model`` fixtures.
"""
import hashlib
import inspect
import os
import struct

import numpy as np
import torch

from ..interop.protoschema import Schema

PKG = "com.intel.analytics.bigdl."
VERSION = "0.10.0"
MAGIC_NO = 3721

_E = {
    "DataType": {0: "INT32", 1: "INT64", 2: "FLOAT", 3: "DOUBLE", 4: "STRING", 5: "BOOL", 6: "CHAR", 7: "SHORT",
                 8: "BYTES", 9: "REGULARIZER", 10: "TENSOR", 11: "VARIABLE_FORMAT", 12: "INITMETHOD", 13: "MODULE",
                 14: "NAME_ATTR_LIST", 15: "ARRAY_VALUE", 16: "DATA_FORMAT", 17: "CUSTOM", 18: "SHAPE"},
    "TensorType": {0: "DENSE", 1: "QUANT"},
    "RegularizerType": {0: "L1L2Regularizer", 1: "L1Regularizer", 2: "L2Regularizer"},
    "InitMethodType": {0: "EMPTY_INITIALIZATION", 1: "RANDOM_UNIFORM", 2: "RANDOM_UNIFORM_PARAM", 3: "RANDOM_NORMAL",
                       4: "ZEROS", 5: "ONES", 6: "CONST", 7: "XAVIER", 8: "BILINEARFILLER"},
    "InputDataFormat": {0: "NCHW", 1: "NHWC"},
    "ShapeType": {0: "SINGLE", 1: "MULTI"},
    "VarFormat": {0: "EMPTY_FORMAT", 1: "DEFAULT", 2: "ONE_D", 3: "IN_OUT", 4: "OUT_IN", 5: "IN_OUT_KW_KH",
                  6: "OUT_IN_KW_KH", 7: "GP_OUT_IN_KW_KH", 8: "GP_IN_OUT_KW_KH", 9: "OUT_IN_KT_KH_KW"},
}

SCHEMA = Schema({
    "BigDLModule": {1: ("name", "string", None), 2: ("subModules", "msg", "BigDLModule"),
                    3: ("weight", "msg", "BigDLTensor"), 4: ("bias", "msg", "BigDLTensor"),
                    5: ("preModules", "string", None), 6: ("nextModules", "string", None),
                    7: ("moduleType", "string", None), 8: ("attr", "msg", "AttrEntry"), 9: ("version", "string", None),
                    10: ("train", "bool", None), 11: ("namePostfix", "string", None), 12: ("id", "int", None),
                    13: ("inputShape", "msg", "Shape"), 14: ("outputShape", "msg", "Shape"),
                    15: ("hasParameters", "bool", None), 16: ("parameters", "msg", "BigDLTensor"),
                    17: ("isMklInt8Enabled", "bool", None), 18: ("inputDimMasks", "int", None),
                    19: ("inputScales", "msg", "AttrValue"), 20: ("outputDimMasks", "int", None),
                    21: ("outputScales", "msg", "AttrValue"), 22: ("weightDimMasks", "int", None),
                    23: ("weightScales", "msg", "AttrValue")},
    "AttrEntry": {1: ("key", "string", None), 2: ("value", "msg", "AttrValue")},
    "InitMethod": {1: ("methodType", "enum", "InitMethodType"), 2: ("data", "double", None)},
    "BigDLTensor": {1: ("datatype", "enum", "DataType"), 2: ("size", "int", None), 3: ("stride", "int", None),
                    4: ("offset", "int", None), 5: ("dimension", "int", None), 6: ("nElements", "int", None),
                    7: ("isScalar", "bool", None), 8: ("storage", "msg", "TensorStorage"), 9: ("id", "int", None),
                    10: ("tensorType", "enum", "TensorType")},
    "TensorStorage": {1: ("datatype", "enum", "DataType"), 2: ("float_data", "float", None),
                      3: ("double_data", "double", None), 4: ("bool_data", "bool", None),
                      5: ("string_data", "string", None), 6: ("int_data", "int", None),
                      7: ("long_data", "int64", None), 8: ("bytes_data", "bytes", None), 9: ("id", "int", None)},
    "Regularizer": {1: ("regularizerType", "enum", "RegularizerType"), 2: ("regularData", "double", None)},
    "ArrayValue": {1: ("size", "int", None), 2: ("datatype", "enum", "DataType"), 3: ("i32", "int", None),
                   4: ("i64", "int64", None), 5: ("flt", "float", None), 6: ("dbl", "double", None),
                   7: ("str", "string", None), 8: ("boolean", "bool", None), 9: ("Regularizer", "msg", "Regularizer"),
                   10: ("tensor", "msg", "BigDLTensor"), 11: ("variableFormat", "enum", "VarFormat"),
                   12: ("initMethod", "msg", "InitMethod"), 13: ("bigDLModule", "msg", "BigDLModule"),
                   14: ("nameAttrList", "msg", "NameAttrList"), 15: ("dataFormat", "enum", "InputDataFormat"),
                   17: ("shape", "msg", "Shape")},
    "AttrValue": {1: ("dataType", "enum", "DataType"), 2: ("subType", "string", None), 3: ("int32Value", "int", None),
                  4: ("int64Value", "int64", None), 5: ("floatValue", "float", None),
                  6: ("doubleValue", "double", None), 7: ("stringValue", "string", None),
                  8: ("boolValue", "bool", None), 9: ("regularizerValue", "msg", "Regularizer"),
                  10: ("tensorValue", "msg", "BigDLTensor"), 11: ("variableFormatValue", "enum", "VarFormat"),
                  12: ("initMethodValue", "msg", "InitMethod"), 13: ("bigDLModuleValue", "msg", "BigDLModule"),
                  14: ("nameAttrListValue", "msg", "NameAttrList"), 15: ("arrayValue", "msg", "ArrayValue"),
                  16: ("dataFormatValue", "enum", "InputDataFormat"), 18: ("shape", "msg", "Shape")},
    "NameAttrList": {1: ("name", "string", None), 2: ("attr", "msg", "AttrEntry")},
    "Shape": {1: ("shapeType", "enum", "ShapeType"), 2: ("ssize", "int", None), 3: ("shapeValue", "int", None),
              4: ("shape", "msg", "Shape")},
}, _E)

_DTYPES = {torch.float32: ("FLOAT", "float_data"), torch.float64: ("DOUBLE", "double_data"),
           torch.int32: ("INT32", "int_data"), torch.int64: ("INT64", "long_data"), torch.bool: ("BOOL", "bool_data"),
           torch.int16: ("SHORT", "int_data")}
_TORCH = {"FLOAT": torch.float32, "DOUBLE": torch.float64, "INT32": torch.int32, "INT64": torch.int64,
          "BOOL": torch.bool, "SHORT": torch.int16, "CHAR": torch.int32}


def _one(d, k, default=None):
    v = d.get(k)
    return v[0] if v else default


def _attr_map(entries):
    return {_one(e, "key"): _one(e, "value", {}) for e in entries or []}


# ============================================================================================ serialize
class _SerCtx:
    def __init__(self, storage="proto"):
        self.next_id = 1
        self.tensor_ids = {}           # id(python tensor) -> tensor id
        self.storages = {}             # tensor id -> full BigDLTensor dict (with storage data)
        self.raw = {}                  # storage id -> (dtype name, flat numpy) for the separate weight file
        self.module_ids = {}
        self.storage = storage
        self.keep = []                 # keeps every serialized object alive so id() stays unique

    def new_id(self):
        i = self.next_id
        self.next_id += 1
        return i


def _tensor_attr(t, ctx):
    ctx.keep.append(t)
    key = id(t)
    if key in ctx.tensor_ids:
        full = ctx.storages[ctx.tensor_ids[key]]
        return _strip_storage(full)
    t = t.detach().to("cpu")
    if t.dtype in (torch.float16, torch.bfloat16):
        t = t.float()
    dt, field = _DTYPES.get(t.dtype, ("FLOAT", "float_data"))
    if t.dtype not in _DTYPES:
        t = t.float()
    tid, sid = ctx.new_id(), ctx.new_id()
    c = t.contiguous()
    flat = c.reshape(-1)
    st = {"datatype": [dt], "id": [sid]}
    if ctx.storage == "proto":
        vals = flat.tolist()
        st[field] = [bool(v) for v in vals] if dt == "BOOL" else vals
    else:
        ctx.raw[sid] = (dt, flat.numpy().copy())
    strides, acc = [], 1
    for s in reversed(list(c.shape)):
        strides.insert(0, acc)
        acc *= s
    full = {"datatype": [dt], "size": list(c.shape), "stride": strides, "offset": [1], "dimension": [c.dim()],
            "nElements": [c.numel()], "isScalar": [c.dim() == 0], "storage": [st], "id": [tid],
            "tensorType": ["DENSE"]}
    ctx.tensor_ids[key] = tid
    ctx.storages[tid] = full
    return _strip_storage(full)


def _strip_storage(full):
    d = dict(full)
    st = full["storage"][0]
    d["storage"] = [{"datatype": st["datatype"], "id": st["id"]}]
    return d


def _attr(v, ctx):
    from ..nn.abstractnn import AbstractCriterion, AbstractModule
    from ..nn.init_methods import InitializationMethod
    from ..optim.regularizer import L1L2Regularizer

    if v is None:
        return {"subType": ["null"]}
    if isinstance(v, bool):
        return {"dataType": ["BOOL"], "boolValue": [v]}
    if isinstance(v, int):
        if -(1 << 31) <= v < (1 << 31):
            return {"dataType": ["INT32"], "int32Value": [v]}
        return {"dataType": ["INT64"], "int64Value": [v]}
    if isinstance(v, float):
        return {"dataType": ["DOUBLE"], "doubleValue": [v]}
    if isinstance(v, str):
        return {"dataType": ["STRING"], "stringValue": [v]}
    if isinstance(v, torch.Tensor):
        return {"dataType": ["TENSOR"], "tensorValue": [_tensor_attr(v, ctx)]}
    if isinstance(v, np.ndarray):
        return _attr(torch.from_numpy(v), ctx)
    if isinstance(v, L1L2Regularizer):
        kind = type(v).__name__ if type(v).__name__ in _E["RegularizerType"].values() else "L1L2Regularizer"
        return {"dataType": ["REGULARIZER"], "regularizerValue": [{"regularizerType": [kind],
                                                                    "regularData": [v.l1, v.l2]}]}
    if isinstance(v, InitializationMethod):
        return {"dataType": ["INITMETHOD"], "initMethodValue": [_init_method(v)]}
    if isinstance(v, AbstractModule):
        return {"dataType": ["MODULE"], "bigDLModuleValue": [serialize_module(v, ctx)]}
    if isinstance(v, AbstractCriterion) or hasattr(v, "_init_args"):
        return {"dataType": ["CUSTOM"], "subType": ["py:" + type(v).__name__],
                "nameAttrListValue": [_bound_args(v, ctx, type(v).__name__)]}
    if isinstance(v, (list, tuple)):
        return {"dataType": ["ARRAY_VALUE"], "arrayValue": [_array(list(v), ctx)]}
    if isinstance(v, dict) or hasattr(v, "items"):
        return {"dataType": ["NAME_ATTR_LIST"], "nameAttrListValue": [
            {"name": ["table"], "attr": [{"key": [str(k)], "value": [_attr(x, ctx)]} for k, x in v.items()]}]}
    raise TypeError(f"bigdl.proto: cannot serialize attribute of type {type(v).__name__}")


def _array(vals, ctx):
    from ..nn.abstractnn import AbstractModule

    a = {"size": [len(vals)]}
    if not vals or all(isinstance(x, bool) for x in vals):
        a.update(datatype=["BOOL"], boolean=list(vals)) if vals else a.update(datatype=["INT32"])
    elif all(isinstance(x, int) and not isinstance(x, bool) for x in vals):
        a.update(datatype=["INT32"], i32=list(vals))
    elif all(isinstance(x, (int, float)) and not isinstance(x, bool) for x in vals):
        a.update(datatype=["DOUBLE"], dbl=[float(x) for x in vals])
    elif all(isinstance(x, str) for x in vals):
        a.update(datatype=["STRING"], str=list(vals))
    elif all(isinstance(x, torch.Tensor) for x in vals):
        a.update(datatype=["TENSOR"], tensor=[_tensor_attr(x, ctx) for x in vals])
    elif all(isinstance(x, AbstractModule) for x in vals):
        a.update(datatype=["MODULE"], bigDLModule=[serialize_module(x, ctx) for x in vals])
    else:   # heterogeneous (nested lists, None, objects): one NameAttrList entry per element
        a.update(datatype=["NAME_ATTR_LIST"], nameAttrList=[
            {"name": ["item"], "attr": [{"key": ["v"], "value": [_attr(x, ctx)]}]} for x in vals])
    return a


def _init_method(m):
    n = type(m).__name__
    if n == "RandomUniform":
        if m.lower is None:
            return {"methodType": ["RANDOM_UNIFORM"]}
        return {"methodType": ["RANDOM_UNIFORM_PARAM"], "data": [float(m.lower), float(m.upper)]}
    if n == "RandomNormal":
        return {"methodType": ["RANDOM_NORMAL"], "data": [float(m.mean), float(m.stdv)]}
    if n == "Zeros":
        return {"methodType": ["ZEROS"]}
    if n == "Ones":
        return {"methodType": ["ONES"]}
    if n == "ConstInitMethod":
        return {"methodType": ["CONST"], "data": [float(m.value)]}
    if n == "Xavier":
        return {"methodType": ["XAVIER"]}
    if n == "BilinearFiller":
        return {"methodType": ["BILINEARFILLER"]}
    return {"methodType": ["EMPTY_INITIALIZATION"]}


def _bound_args(m, ctx, name):
    args, kw = getattr(m, "_init_args", ((), {}))
    try:
        bound = inspect.signature(type(m).__init__).bind(None, *args, **kw).arguments
        bound.pop(next(iter(bound)))      # self
    except TypeError:
        bound = {f"arg{i}": a for i, a in enumerate(args)}
        bound.update(kw)
    entries = []
    for k, v in bound.items():
        if isinstance(v, dict) and inspect.signature(type(m).__init__).parameters[k].kind == \
                inspect.Parameter.VAR_KEYWORD:
            for kk, vv in v.items():
                entries.append({"key": [kk], "value": [_attr(vv, ctx)]})
            continue
        if isinstance(v, tuple) and k in inspect.signature(type(m).__init__).parameters and \
                inspect.signature(type(m).__init__).parameters[k].kind == inspect.Parameter.VAR_POSITIONAL:
            v = list(v)
        entries.append({"key": [k], "value": [_attr(v, ctx)]})
    return {"name": [name], "attr": entries}


def _module_type(m):
    from ..nn.abstractnn import module_key

    key = module_key(type(m))
    if key.startswith("keras."):
        return PKG + "nn.keras." + key[6:]
    if key.startswith("ops."):
        return PKG + "nn.ops." + key[4:]
    if key.startswith("nn."):
        return PKG + key
    return PKG + "nn." + key


def serialize_module(m, ctx, pre=(), nxt=()):
    from ..nn.graph import Graph

    ctx.keep.append(m)
    if id(m) in ctx.module_ids:
        mid = ctx.module_ids[id(m)]
    else:
        mid = ctx.new_id()
        ctx.module_ids[id(m)] = mid
    d = {"moduleType": [_module_type(m)], "version": [VERSION], "train": [bool(m.train)], "id": [mid],
         "namePostfix": [""], "preModules": list(pre), "nextModules": list(nxt)}
    if m.hasName():
        d["name"] = [m.getName()]
    from ..nn.abstractnn import module_key

    entries = [] if isinstance(m, Graph) else _bound_args(m, ctx, "args")["attr"]
    entries += [{"key": ["module_tags"], "value": [_attr(["Float"], ctx)]},
                {"key": ["module_numerics"], "value": [_attr(["Float"], ctx)]},
                # the engine's registry key: disambiguates engine classes that share a Scala simple name
                {"key": ["engine_class"], "value": [_attr(module_key(type(m)), ctx)]}]
    for b in getattr(m, "_buffers", ()):
        t = getattr(m, b, None)
        if t is not None:
            entries.append({"key": [b], "value": [_attr(t, ctx)]})
    for k in ("wRegularizer", "bRegularizer"):
        r = getattr(m, k, None)
        if r is not None and not any(e["key"][0] == k for e in entries):
            entries.append({"key": [k], "value": [_attr(r, ctx)]})
    if isinstance(m, Graph):
        subs = []
        names = {}
        for n in m.order:
            names[n.id] = n.element.getName()
        for n in m.order:
            pres = [names[p.id] for p in n.prevs]
            nexts = [names[x.id] for x in n.nexts]
            subs.append(serialize_module(n.element, ctx, pres, nexts))
            edges = {"name": [names[n.id]], "attr": [
                {"key": [names[p.id]], "value": [_attr(-1 if i is None else int(i), ctx)]}
                for p, i in zip(n.prevs, n.prev_index)]}
            entries.append({"key": [f"{names[n.id]}_edges"],
                            "value": [{"dataType": ["NAME_ATTR_LIST"], "nameAttrListValue": [edges]}]})
        d["subModules"] = subs
        entries.append({"key": ["inputNames"], "value": [_attr([names[n.id] for n in m.inputs_nodes], ctx)]})
        entries.append({"key": ["outputNames"], "value": [_attr([names[n.id] for n in m.output_nodes], ctx)]})
        if type(m).__name__ == "DynamicGraph":
            entries.append({"key": ["generateBackward"],
                            "value": [_attr(bool(getattr(m, "generateBackward", True)), ctx)]})
    elif _has_children(m):
        d["subModules"] = [serialize_module(c, ctx) for c in m.modules]
    else:
        # leaf, or a composite whose constructor builds its own sub-modules (cells, heads, attention blocks):
        # all parameters (recursively, in parameters() order) and every nested buffer
        p = m.parameters()
        if p and p[0]:
            d["hasParameters"] = [True]
            d["parameters"] = [_tensor_attr(w, ctx) for w in p[0]]
        nested = _nested_buffers(m)
        if nested:
            entries.append({"key": ["nested_buffers"], "value": [_attr(nested, ctx)]})
    d["attr"] = entries
    return d


def _has_children(m):
    """True for containers whose children come from ``add`` (Sequential, Concat, Recurrent, ...): a fresh
    instance built from the same constructor arguments has no children."""
    from ..nn.abstractnn import AbstractModule

    if not (hasattr(m, "modules") and isinstance(m.modules, list) and m.modules):
        return False
    args, kw = getattr(m, "_init_args", ((), {}))
    if any(isinstance(a, AbstractModule) for a in list(args) + list(kw.values())):
        return False
    if hasattr(m, "_set_children"):          # fixed child slots whose contents are added later (BiRecurrent)
        return True
    try:
        fresh = type(m)(*args, **kw)
    except Exception:  # noqa: BLE001
        return True
    return not getattr(fresh, "modules", None)


def _nested_buffers(m):
    """Buffers of sub-modules built by the constructor (e.g. BN running stats inside a detection head)."""
    out = []
    for c in _walk(m):
        if c is m:
            continue
        for b in getattr(c, "_buffers", ()):
            t = getattr(c, b, None)
            if isinstance(t, torch.Tensor):
                out.append(t)
    return out


def _walk(m):
    yield m
    for c in getattr(m, "modules", None) or []:
        if hasattr(c, "parameters"):
            yield from _walk(c)


def save_bigdl(module, path, weightPath=None, overWrite=False):
    """Reference ``module.saveModule(path, weightPath, overWrite)`` in bigdl.proto form."""
    for p in (path, weightPath):
        if p and os.path.exists(p) and not overWrite:
            raise FileExistsError(f"{p} exists (set overWrite)")
    ctx = _SerCtx("proto" if weightPath is None else "bigdl")
    root = serialize_module(module, ctx)
    if weightPath is None:
        gs = {"name": ["global_storage"], "attr": [
            {"key": [str(tid)], "value": [{"dataType": ["TENSOR"], "tensorValue": [full]}]}
            for tid, full in ctx.storages.items()]}
        root["attr"].append({"key": ["global_storage"],
                             "value": [{"dataType": ["NAME_ATTR_LIST"], "nameAttrListValue": [gs]}]})
    with open(path, "wb") as f:
        f.write(SCHEMA.encode("BigDLModule", root))
    if weightPath is not None:
        _write_weights(weightPath, ctx.raw)
    return module


# The weight file keys storages by the Scala ``BigDLDataType`` enumeration (serializer/Types.scala:49-52:
# FLOAT, DOUBLE, CHAR, BOOL, STRING, INT, SHORT, LONG, BYTESTRING, BYTE = 0..9), NOT by the protobuf DataType
# numbering used inside TensorStorage messages. Element encodings follow DataReaderWriter.scala (big-endian
# DataOutputStream: writeFloat / writeDouble / writeChar (u16) / writeBoolean (u8) / writeInt / writeShort /
# writeLong / raw bytes).
_DT_ID = {"FLOAT": 0, "DOUBLE": 1, "CHAR": 2, "BOOL": 3, "INT32": 5, "SHORT": 6, "INT64": 7, "BYTE": 9}
_DT_FMT = {0: ">f4", 1: ">f8", 2: ">u2", 3: ">u1", 5: ">i4", 6: ">i2", 7: ">i8", 9: ">i1"}


def _write_weights(path, raw):
    """Reference ModulePersister.saveWeightsToFile: big-endian DataOutputStream, MD5 over everything before it."""
    body = bytearray(struct.pack(">ii", MAGIC_NO, len(raw)))
    for sid, (dt, arr) in raw.items():
        code = _DT_ID[dt]
        body += struct.pack(">iii", sid, code, arr.size)
        body += np.asarray(arr).astype(_DT_FMT[code]).tobytes()
    digest = hashlib.md5(bytes(body)).digest()
    with open(path, "wb") as f:
        f.write(bytes(body) + struct.pack(">i", len(digest)) + digest)


def _read_weights(path):
    with open(path, "rb") as f:
        data = f.read()
    magic, n = struct.unpack_from(">ii", data, 0)
    if magic != MAGIC_NO:
        raise ValueError(f"Magic number mismatch, expected {MAGIC_NO}, actual {magic}")
    pos, out = 8, {}
    for _ in range(n):
        sid, code, size = struct.unpack_from(">iii", data, pos)
        pos += 12
        if code not in _DT_FMT:
            raise ValueError(f"weight file storage {sid}: unsupported BigDLDataType code {code}")
        fmt = np.dtype(_DT_FMT[code])
        out[sid] = np.frombuffer(data, dtype=fmt, count=size, offset=pos).astype(fmt.newbyteorder("="))
        pos += size * fmt.itemsize
    (dlen,) = struct.unpack_from(">i", data, pos)
    stored = data[pos + 4:pos + 4 + dlen]
    if hashlib.md5(data[:pos]).digest() != stored:
        raise ValueError("check sum error, please check weight file")
    return out


# ============================================================================================ deserialize
class _LoadCtx:
    def __init__(self, storages):
        self.storages = storages     # storage id -> numpy flat data
        self.tensors = {}            # tensor id -> torch tensor
        self.modules = {}


def _tensor_from(d, ctx):
    st = _one(d, "storage")
    if st is None:
        return None
    tid = _one(d, "id", 0)
    if tid in ctx.tensors:
        return ctx.tensors[tid]
    sid = _one(st, "id", -1)
    dt = _one(d, "datatype", "FLOAT")
    data = ctx.storages.get(sid)
    if data is None:
        for field in ("float_data", "double_data", "int_data", "long_data", "bool_data"):
            if st.get(field):
                data = np.asarray(st[field])
                break
        if data is None:
            data = np.zeros(0, dtype=np.float32)
        ctx.storages[sid] = data
    flat = torch.as_tensor(np.asarray(data)).to(_TORCH.get(dt, torch.float32))
    sizes, strides = d.get("size", []), d.get("stride", [])
    off = _one(d, "offset", 1) - 1
    if not sizes:
        t = flat[off:off + 1].reshape(()) if _one(d, "isScalar", False) else flat.new_empty(0)
    else:
        t = torch.as_strided(flat, sizes, strides or None, off).clone()
    ctx.tensors[tid] = t
    return t


def _value(a, ctx):
    if not a:
        return None
    dt = _one(a, "dataType")
    if _one(a, "subType") == "null" and dt is None:
        return None
    for f in ("int32Value", "int64Value", "floatValue", "doubleValue", "stringValue", "boolValue"):
        if f in a:
            return a[f][0]
    if "tensorValue" in a:
        return _tensor_from(a["tensorValue"][0], ctx)
    if "regularizerValue" in a:
        from ..optim import regularizer as R

        r = a["regularizerValue"][0]
        kind = _one(r, "regularizerType", "L1L2Regularizer")
        d = r.get("regularData", [0.0, 0.0]) + [0.0, 0.0]
        if kind == "L1Regularizer":
            return R.L1Regularizer(d[0])
        if kind == "L2Regularizer":
            return R.L2Regularizer(d[1] if len(r.get("regularData", [])) > 1 else d[0])
        return R.L1L2Regularizer(d[0], d[1])
    if "initMethodValue" in a:
        return _init_from(a["initMethodValue"][0])
    if "bigDLModuleValue" in a:
        return load_module_dict(a["bigDLModuleValue"][0], ctx)
    if "arrayValue" in a:
        return _array_from(a["arrayValue"][0], ctx)
    if "nameAttrListValue" in a:
        nal = a["nameAttrListValue"][0]
        sub = _one(a, "subType", "")
        entries = _attr_map(nal.get("attr"))
        if sub.startswith("py:"):
            from ..nn.abstractnn import all_module_classes

            import bigdl_amd.nn as nnmod

            cls = getattr(nnmod, sub[3:], None) or all_module_classes().get(sub[3:])
            return _construct(cls, {k: _value(v, ctx) for k, v in entries.items()})
        return {k: _value(v, ctx) for k, v in entries.items()}
    if "dataFormatValue" in a:
        return a["dataFormatValue"][0]
    if "variableFormatValue" in a:
        return a["variableFormatValue"][0]
    if "shape" in a:
        return a["shape"][0].get("shapeValue", [])
    return None


def _array_from(a, ctx):
    dt = _one(a, "datatype", "INT32")
    for f in ("i32", "i64", "flt", "dbl", "str", "boolean"):
        if f in a:
            return list(a[f])
    if "tensor" in a:
        return [_tensor_from(t, ctx) for t in a["tensor"]]
    if "bigDLModule" in a:
        return [load_module_dict(m, ctx) for m in a["bigDLModule"]]
    if "Regularizer" in a:
        return [_value({"regularizerValue": [r]}, ctx) for r in a["Regularizer"]]
    if "initMethod" in a:
        return [_init_from(m) for m in a["initMethod"]]
    if "nameAttrList" in a:
        return [_value(_attr_map(n.get("attr")).get("v"), ctx) for n in a["nameAttrList"]]
    del dt
    return []


def _init_from(d):
    from ..nn import init_methods as I

    kind = _one(d, "methodType", "EMPTY_INITIALIZATION")
    data = d.get("data", [])
    if kind == "RANDOM_UNIFORM":
        return I.RandomUniform()
    if kind == "RANDOM_UNIFORM_PARAM":
        return I.RandomUniform(data[0], data[1])
    if kind == "RANDOM_NORMAL":
        return I.RandomNormal(data[0], data[1])
    if kind == "ZEROS":
        return I.Zeros()
    if kind == "ONES":
        return I.Ones()
    if kind == "CONST":
        return I.ConstInitMethod(data[0])
    if kind == "XAVIER":
        return I.Xavier()
    if kind == "BILINEARFILLER":
        return I.BilinearFiller()
    return None


def _class_for(module_type, engine_key=None):
    from ..nn.abstractnn import all_module_classes

    reg = all_module_classes()
    if engine_key and engine_key in reg:
        return reg[engine_key]
    name = module_type[len(PKG):] if module_type.startswith(PKG) else module_type
    cands = []
    if name.startswith("nn.keras."):
        cands = ["keras." + name[9:]]
    elif name.startswith("nn.ops."):
        cands = ["ops." + name[7:], "nn.ops." + name[7:], name[7:]]
    elif name.startswith("nn.tf."):
        cands = ["nn.tf." + name[6:], name[6:]]
    elif name.startswith("nn.mkldnn.") or name.startswith("nn.quantized."):
        cands = [name, name.split(".")[-1]]     # nn.mkldnn.RNN is its own class; other MKL-DNN layers map by name
    elif name.startswith("nn."):
        cands = [name[3:]]
    cands.append(name.split(".")[-1])
    for c in cands:
        if c in reg:
            return reg[c]
    raise KeyError(f"bigdl.proto: no engine module for {module_type}")


def _construct(cls, attrs):
    sig = inspect.signature(cls.__init__).parameters
    args, kw = [], {}
    for name, p in list(sig.items())[1:]:
        if p.kind == inspect.Parameter.VAR_POSITIONAL:
            if name in attrs and isinstance(attrs[name], list):
                args.extend(attrs[name])
            continue
        if p.kind == inspect.Parameter.VAR_KEYWORD:
            continue
        if name in attrs:
            if p.kind == inspect.Parameter.POSITIONAL_ONLY:
                args.append(attrs[name])
            else:
                kw[name] = attrs[name]
    return cls(*args, **kw)


_META = {"module_tags", "module_numerics", "global_storage", "group_type", "inputNames", "outputNames",
         "generateBackward", "sharedWeight", "sharedBias", "stopGradientLayers", "engine_class", "nested_buffers"}


def load_module_dict(d, ctx):
    from ..nn.graph import Graph, Node

    mid = _one(d, "id", 0)
    if mid and mid in ctx.modules:
        return ctx.modules[mid]
    attrs = _attr_map(d.get("attr"))
    ek = _value(attrs["engine_class"], ctx) if "engine_class" in attrs else None
    cls = _class_for(_one(d, "moduleType", ""), ek)
    if issubclass(cls, Graph):
        subs = [load_module_dict(s, ctx) for s in d.get("subModules", [])]
        nodes = {}
        for s, m in zip(d.get("subModules", []), subs):
            nodes[_one(s, "name", m.getName())] = (Node(m), s)
        for name, (node, s) in nodes.items():
            edges = _attr_map(_one(attrs.get(f"{name}_edges", {}), "nameAttrListValue", {}).get("attr"))
            for pre in s.get("preModules", []):
                idx = _value(edges.get(pre), ctx) if pre in edges else -1
                nodes[pre][0].add_next(node, None if idx in (None, -1) else int(idx))
        ins = [nodes[n][0] for n in _value(attrs.get("inputNames"), ctx) or []]
        outs = [nodes[n][0] for n in _value(attrs.get("outputNames"), ctx) or []]
        for n in ins:
            n._is_input = True
        m = cls(ins, outs)
    else:
        kw = {k: _value(v, ctx) for k, v in attrs.items() if k not in _META and not k.endswith("_edges")}
        buffers = {}
        inst_probe = cls.__init__
        params = inspect.signature(inst_probe).parameters
        for b in ("runningMean", "runningVar"):
            if b in kw and b not in params:
                buffers[b] = kw.pop(b)
        m = _construct(cls, kw)
        subs = d.get("subModules", [])
        if subs and hasattr(m, "_set_children"):
            m._set_children([load_module_dict(s, ctx) for s in subs])
        elif subs and _has_children_type(m):
            for s in subs:
                m.add(load_module_dict(s, ctx))
        if _one(d, "hasParameters", False):
            ws = [_tensor_from(t, ctx) for t in d.get("parameters", [])]
            p = m.parameters()
            if p and p[0]:
                if len(p[0]) != len(ws):
                    raise ValueError(f"{cls.__name__}: {len(ws)} serialized parameters, module has {len(p[0])}")
                with torch.no_grad():
                    for dst, src in zip(p[0], ws):
                        dst.copy_(src.reshape(dst.shape).to(dst.dtype))
        for b, t in buffers.items():
            if t is not None and getattr(m, b, None) is not None:
                getattr(m, b).copy_(t.reshape(getattr(m, b).shape))
        nested = _value(attrs["nested_buffers"], ctx) if "nested_buffers" in attrs else None
        if nested:
            dst = _nested_buffers(m)
            if len(dst) != len(nested):
                raise ValueError(f"{cls.__name__}: {len(nested)} serialized nested buffers, module has {len(dst)}")
            with torch.no_grad():
                for a, b in zip(dst, nested):
                    a.copy_(b.reshape(a.shape).to(a.dtype))
    name = _one(d, "name")
    if name:
        m.setName(name)
    if _one(d, "train", False):
        m.training()
    else:
        m.evaluate()
    if mid:
        ctx.modules[mid] = m
    return m


def _has_children_type(m):
    return hasattr(m, "add") and hasattr(m, "modules") and isinstance(m.modules, list)


def load_bigdl(path, weightPath=None):
    """Reference ``Module.loadModule(path, weightPath)`` for bigdl.proto files."""
    with open(path, "rb") as f:
        root = SCHEMA.decode("BigDLModule", f.read())
    storages = {}
    if weightPath is not None:
        storages.update(_read_weights(weightPath))
    ctx = _LoadCtx(storages)
    gs = _attr_map(root.get("attr")).get("global_storage")
    if gs:
        for entry in _one(gs, "nameAttrListValue", {}).get("attr", []):
            tv = _one(_one(entry, "value", {}), "tensorValue")
            if tv is not None:
                _tensor_from(tv, ctx)
    return load_module_dict(root, ctx)


def is_bigdl_proto(path):
    """True when ``path`` holds a BigDLModule message rather than this package's safetensors format."""
    with open(path, "rb") as f:
        head = f.read(16)
    if len(head) >= 8 and head[8:9] == b"{":   # safetensors: u64 header length + JSON
        return False
    return len(head) > 0 and head[0] in (0x0A, 0x12, 0x3A, 0x42, 0x4A, 0x50, 0x5A, 0x60)
