"""Module persistence (reference: S/utils/serializer/ModuleSerializer.scala:36-285, ModuleLoader.scala:37-363
(``loadFromFile`` :47, ``saveToFile`` :230, separate weight file :257), bigdl.proto BigDLModule :4-31).

Format: ONE safetensors file. Tensors (parameters, buffers, tensor-valued constructor args) are stored as
safetensors entries; the module tree is a JSON document in the safetensors metadata under
``"bigdl_module"`` — class name, recorded constructor arguments, container children / graph topology,
plain-value attributes (set through setters such as ``setNumInputDims``), name, train / frozen state.
Loading never executes anything from the file: classes are looked up in this package's module registry and
tensors are read by safetensors. An optional separate weight file mirrors the reference's
``saveModule(path, weightPath)``.
"""
import json
import os

import torch

from ..nn.abstractnn import module_key

from ..utils.table import Table

FORMAT_VERSION = 1
_SKIP_ATTRS = {"output", "gradInput", "modules", "forward_time", "backward_time"}
_SIMPLE = (int, float, bool, str, type(None))


def _is_simple(v):
    if isinstance(v, _SIMPLE):
        return True
    if isinstance(v, (list, tuple)):
        return all(_is_simple(x) for x in v)
    return False


class _Ctx:
    def __init__(self):
        self.tensors = {}
        self.counter = 0

    def add_tensor(self, t):
        key = f"t{self.counter}"
        self.counter += 1
        self.tensors[key] = t.detach().to("cpu").contiguous().clone()
        return key


def _enc(v, ctx):
    from ..nn.abstractnn import AbstractCriterion, AbstractModule

    if isinstance(v, _SIMPLE):
        return v
    if isinstance(v, torch.Tensor):
        return {"__tensor__": ctx.add_tensor(v)}
    if isinstance(v, AbstractModule):
        return {"__module__": encode_module(v, ctx)}
    if isinstance(v, AbstractCriterion):
        return {"__criterion__": module_key(type(v)), "args": _enc_args(v, ctx)}
    if isinstance(v, (list, tuple)):
        return {"__seq__": [_enc(x, ctx) for x in v], "tuple": isinstance(v, tuple)}
    if isinstance(v, dict):
        return {"__dict__": [[_enc(k, ctx), _enc(x, ctx)] for k, x in v.items()]}
    if isinstance(v, Table):
        return {"__table__": [[_enc(k, ctx), _enc(x, ctx)] for k, x in v.items()]}
    # init methods, regularizers and other small config objects: class + public state
    cls = type(v)
    return {"__obj__": f"{cls.__module__}:{cls.__qualname__}",
            "state": {k: _enc(x, ctx) for k, x in vars(v).items() if _is_simple(x) or isinstance(x, torch.Tensor)}}


def _enc_args(m, ctx):
    args, kw = getattr(m, "_init_args", ((), {}))
    return {"args": [_enc(a, ctx) for a in args], "kw": {k: _enc(x, ctx) for k, x in kw.items()}}


def encode_module(m, ctx):
    from ..nn.graph import Graph

    d = {"class": module_key(type(m)), "init": _enc_args(m, ctx), "name": m._name, "train": m.train,
         "frozen": m._frozen}
    d["attrs"] = {k: v for k, v in vars(m).items()
                  if not k.startswith("_") and k not in _SKIP_ATTRS and _is_simple(v)}
    d["params"] = {}
    for w, g in m._params:
        t = getattr(m, w, None)
        if t is not None:
            d["params"][w] = ctx.add_tensor(t)
    d["buffers"] = {}
    for b in m._buffers:
        t = getattr(m, b, None)
        if t is not None:
            d["buffers"][b] = ctx.add_tensor(t)
    for k in ("wRegularizer", "bRegularizer"):
        r = getattr(m, k, None)
        if r is not None:
            d[k] = _enc(r, ctx)
    if isinstance(m, Graph):
        idx = {n.id: i for i, n in enumerate(m.order)}
        d["graph"] = {
            "nodes": [{"module": encode_module(n.element, ctx), "prevs": [idx[p.id] for p in n.prevs],
                       "prev_index": list(n.prev_index)} for n in m.order],
            "inputs": [idx[n.id] for n in m.inputs_nodes],
            "outputs": [idx[n.id] for n in m.output_nodes],
            "dynamic": type(m).__name__ == "DynamicGraph",
            "generateBackward": bool(getattr(m, "generateBackward", True)),
        }
    elif hasattr(m, "modules") and isinstance(m.modules, list) and not _init_has_modules(m):
        d["children"] = [encode_module(c, ctx) for c in m.modules]
    return d


def _init_has_modules(m):
    from ..nn.abstractnn import AbstractModule

    args, kw = getattr(m, "_init_args", ((), {}))
    return any(isinstance(a, AbstractModule) for a in list(args) + list(kw.values())) and \
        type(m).__name__ in ("Bottle", "MapTable", "TimeDistributed")


def _dec(v, tensors):
    if isinstance(v, _SIMPLE):
        return v
    if "__tensor__" in v:
        return tensors[v["__tensor__"]]
    if "__module__" in v:
        return decode_module(v["__module__"], tensors)
    if "__criterion__" in v:
        from ..nn.abstractnn import module_class

        args = v["args"]
        return module_class(v["__criterion__"])(*[_dec(a, tensors) for a in args["args"]],
                                               **{k: _dec(x, tensors) for k, x in args["kw"].items()})
    if "__seq__" in v:
        seq = [_dec(x, tensors) for x in v["__seq__"]]
        return tuple(seq) if v.get("tuple") else seq
    if "__dict__" in v:
        return {_dec(k, tensors): _dec(x, tensors) for k, x in v["__dict__"]}
    if "__table__" in v:
        t = Table()
        for k, x in v["__table__"]:
            t[_dec(k, tensors)] = _dec(x, tensors)
        return t
    if "__obj__" in v:
        modname, qual = v["__obj__"].split(":")
        if not modname.startswith("bigdl_amd."):
            raise ValueError(f"refusing to instantiate foreign class {v['__obj__']}")
        import importlib

        cls = importlib.import_module(modname)
        for part in qual.split("."):
            cls = getattr(cls, part)
        obj = cls.__new__(cls)
        for k, x in v["state"].items():
            setattr(obj, k, _dec(x, tensors))
        return obj
    raise ValueError(f"cannot decode {v!r}")


def decode_module(d, tensors):
    from ..nn.abstractnn import module_class
    from ..nn.graph import Graph, Node

    cls = module_class(d["class"])
    if "graph" in d:
        g = d["graph"]
        nodes = []
        for nd in g["nodes"]:
            n = Node(decode_module(nd["module"], tensors))
            nodes.append(n)
        for nd, n in zip(g["nodes"], nodes):
            for p, k in zip(nd["prevs"], nd.get("prev_index") or [None] * len(nd["prevs"])):
                nodes[p].add_next(n, k)
        for i in g["inputs"]:
            nodes[i]._is_input = True
        if g.get("dynamic"):
            m = Graph.dynamic([nodes[i] for i in g["inputs"]], [nodes[i] for i in g["outputs"]], None,
                              g.get("generateBackward", True))
        else:
            m = Graph([nodes[i] for i in g["inputs"]], [nodes[i] for i in g["outputs"]])
    else:
        args = [_dec(a, tensors) for a in d["init"]["args"]]
        kw = {k: _dec(x, tensors) for k, x in d["init"]["kw"].items()}
        m = cls(*args, **kw)
        if "children" in d:
            children = [decode_module(c, tensors) for c in d["children"]]
            if hasattr(m, "_set_children"):   # modules whose constructor builds their own sub-structure
                m._set_children(children)
            else:
                m.modules = []
                for c in children:
                    m.add(c)
    for k, v in d.get("attrs", {}).items():
        try:
            setattr(m, k, tuple(v) if isinstance(getattr(m, k, None), tuple) else v)
        except AttributeError:
            pass
    for w, key in d.get("params", {}).items():
        cur = getattr(m, w, None)
        t = tensors[key]
        if cur is not None and cur.shape == t.shape:
            cur.data.copy_(t)
        else:
            setattr(m, w, t.clone())
    for b, key in d.get("buffers", {}).items():
        setattr(m, b, tensors[key].clone())
    for k in ("wRegularizer", "bRegularizer"):
        if k in d:
            setattr(m, k, _dec(d[k], tensors))
    m._name = d.get("name")
    m.train = d.get("train", True)
    m._frozen = d.get("frozen", False)
    return m


def save_module(module, path, weightPath=None, overWrite=False, format=None):
    """``format``: "safetensors" (default; engine-native, every attribute) or "bigdl" (the reference's
    bigdl.proto ``BigDLModule``, utils/bigdl_proto.py). The default follows the ``bigdl.modelFormat`` engine
    property."""
    from safetensors.torch import save_file

    if format is None:
        from .engine import Engine

        format = Engine.getProperty("bigdl.modelFormat", "safetensors")
    if format in ("bigdl", "protobuf", "proto"):
        from .bigdl_proto import save_bigdl

        save_bigdl(module, path, weightPath, overWrite)
        return path

    for p in (path, weightPath):
        if p is not None and os.path.exists(p) and not overWrite:
            raise FileExistsError(f"{p} exists (use overWrite=True)")
    ctx = _Ctx()
    doc = {"version": FORMAT_VERSION, "module": encode_module(module, ctx)}
    meta = {"bigdl_module": json.dumps(doc), "format": "bigdl_amd"}
    if weightPath is not None:
        save_file(ctx.tensors, weightPath, metadata={"format": "bigdl_amd-weights"})
        meta["weights"] = os.path.basename(weightPath)
        save_file({}, path, metadata=meta)
    else:
        save_file(ctx.tensors, path, metadata=meta)
    return path


def load_module(path, weightPath=None):
    """Loads either format: safetensors files written by this package, or bigdl.proto ``BigDLModule`` files
    (reference ModuleLoader.loadFromFile)."""
    from safetensors import safe_open
    from safetensors.torch import load_file

    from .bigdl_proto import is_bigdl_proto, load_bigdl

    if is_bigdl_proto(path):
        return load_bigdl(path, weightPath)

    with safe_open(path, framework="pt") as f:
        meta = f.metadata() or {}
    if "bigdl_module" not in meta:
        raise ValueError(f"{path} is not a bigdl_amd module file")
    doc = json.loads(meta["bigdl_module"])
    tensors = load_file(path)
    if "weights" in meta:
        wp = weightPath or os.path.join(os.path.dirname(path), meta["weights"])
        tensors.update(load_file(wp))
    return decode_module(doc["module"], tensors)


class ModuleSerializer:
    """Reference S/utils/serializer/ModuleSerializer.scala:36 (serialize / load of one module)."""

    serialize = staticmethod(encode_module)
    load = staticmethod(decode_module)


class ModuleLoader:
    """Reference ModuleLoader.scala:37 ``loadFromFile(path, weightPath)``."""

    @staticmethod
    def loadFromFile(modelPath, weightPath=None):
        return load_module(modelPath, weightPath)


class ModulePersister:
    """Reference ModuleLoader.scala:230 ``saveToFile(path, weightPath, module, overwrite)``."""

    @staticmethod
    def saveToFile(modelPath, weightPath, module, overwrite=False):
        return save_module(module, modelPath, weightPath, overwrite)
