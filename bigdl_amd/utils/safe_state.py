"""Pickle-free persistence of framework objects (optimizer methods, LR schedules, state tables).

A saved object is ONE safetensors file: every tensor in the object graph is a safetensors entry and the
structure is a JSON document in the file's metadata. Loading executes nothing from the file: classes are
resolved only inside the ``bigdl_amd`` package and only if they derive from an allow-listed base class
(reference counterpart: OptimMethod.save / load, S/optim/OptimMethod.scala:93-124, which uses Java
serialization; here the format is safe to open from an untrusted checkpoint directory).
"""
import importlib
import json
import math

import torch

FORMAT = "bigdl_amd.safe_state/1"
# attributes bound by the runtime (device views, per-rank offsets) that a checkpoint must not carry
_RUNTIME_ONLY = frozenset({"_shadow16", "_wd_segments", "_seg_base", "_calculated_scale", "_lr_dev"})


def _allowed_bases():
    from ..optim.optim_method import OptimMethod
    from ..optim.sgd import LearningRateSchedule, Regime
    from .table import Table

    return (OptimMethod, LearningRateSchedule, Regime, Table)


def _is_allowed_class(cls):
    return cls.__module__.startswith("bigdl_amd.") and issubclass(cls, _allowed_bases())


class _Enc:
    def __init__(self):
        self.tensors = {}

    def enc(self, v):
        from .table import Table

        if v is None or isinstance(v, (bool, str)):
            return v
        if isinstance(v, int):
            return v
        if isinstance(v, float):
            if math.isfinite(v):
                return v
            return {"__float__": repr(v)}
        if isinstance(v, torch.Tensor):
            key = f"t{len(self.tensors)}"
            self.tensors[key] = v.detach().to("cpu").clone().contiguous()
            return {"__tensor__": key}
        if isinstance(v, (list, tuple)):
            return {"__list__" if isinstance(v, list) else "__tuple__": [self.enc(x) for x in v]}
        if isinstance(v, Table):
            return {"__table__": [[self.enc(k), self.enc(x)] for k, x in v.items()]}
        if isinstance(v, dict):
            return {"__dict__": [[self.enc(k), self.enc(x)] for k, x in v.items()]}
        if callable(v) and hasattr(v, "__qualname__") and not isinstance(v, type) and "<" not in v.__qualname__ \
                and getattr(v, "__module__", "").startswith("bigdl_amd."):
            return {"__fn__": f"{v.__module__}:{v.__qualname__}"}
        cls = type(v)
        if _is_allowed_class(cls):
            d = {k: x for k, x in v.__dict__.items() if k not in _RUNTIME_ONLY}
            return {"__obj__": f"{cls.__module__}:{cls.__qualname__}", "state": self.enc(d)}
        raise TypeError(f"safe_state: cannot persist a value of type {cls.__module__}.{cls.__qualname__}")


def _resolve(path):
    mod, _, name = path.partition(":")
    if not mod.startswith("bigdl_amd."):
        raise ValueError(f"safe_state: refusing to load {path!r} (outside bigdl_amd)")
    obj = importlib.import_module(mod)
    for part in name.split("."):
        obj = getattr(obj, part)
    return obj


def _dec(v, tensors):
    from .table import Table

    if not isinstance(v, dict):
        return v
    if "__float__" in v:
        return float(v["__float__"])
    if "__tensor__" in v:
        return tensors[v["__tensor__"]]
    if "__list__" in v:
        return [_dec(x, tensors) for x in v["__list__"]]
    if "__tuple__" in v:
        return tuple(_dec(x, tensors) for x in v["__tuple__"])
    if "__table__" in v:
        t = Table()
        for k, x in v["__table__"]:
            t[_dec(k, tensors)] = _dec(x, tensors)
        return t
    if "__dict__" in v:
        return {_dec(k, tensors): _dec(x, tensors) for k, x in v["__dict__"]}
    if "__fn__" in v:
        fn = _resolve(v["__fn__"])
        if isinstance(fn, type) or not callable(fn):
            raise ValueError(f"safe_state: {v['__fn__']} is not a function")
        return fn
    if "__obj__" in v:
        cls = _resolve(v["__obj__"])
        if not isinstance(cls, type) or not _is_allowed_class(cls):
            raise ValueError(f"safe_state: class {v['__obj__']} is not allowed")
        obj = cls.__new__(cls)
        obj.__dict__.update(_dec(v["state"], tensors))
        return obj
    raise ValueError(f"safe_state: malformed node {list(v)[:3]}")


def save(obj, path):
    from safetensors.torch import save_file

    e = _Enc()
    doc = e.enc(obj)
    save_file(e.tensors, path, metadata={"format": FORMAT, "doc": json.dumps(doc)})


def load(path, device=None):
    from safetensors import safe_open

    with safe_open(path, framework="pt", device="cpu") as f:
        meta = f.metadata() or {}
        if meta.get("format") != FORMAT:
            raise ValueError(f"{path}: not a {FORMAT} file")
        tensors = {k: f.get_tensor(k) for k in f.keys()}
    if device is not None:
        tensors = {k: t.to(device) for k, t in tensors.items()}
    return _dec(json.loads(meta["doc"]), tensors)
