"""Shared conversions for the pyspark-style facade: snake_case keyword arguments -> the engine's camelCase
constructor arguments, numpy <-> torch activities."""
import inspect
import re

import numpy as np
import torch

# reference Python names whose camelCase form differs from the engine's argument name
_ALIASES = {"data_format": "format", "epsilon": "Epsilon", "leaningrate_schedule": "learningRateSchedule",
            "learningrate_schedule": "learningRateSchedule", "learningrate": "learningRate",
            "learningrate_decay": "learningRateDecay", "weightdecay": "weightDecay", "decayrate": "decayRate",
            "learningrate_power": "learningRatePower", "max_iter": "maxIter", "max_eval": "maxEval",
            "tolfun": "tolFun", "tolx": "tolX", "ncorrection": "nCorrection", "linesearch": "lineSearch",
            "linesearch_options": "lineSearchOptions", "min_lr": "minLr", "size_average": "sizeAverage"}


def camel(name):
    if name in _ALIASES:
        return _ALIASES[name]
    return re.sub(r"_([a-z0-9])", lambda m: m.group(1).upper(), name)


def to_torch(x):
    if isinstance(x, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(x))
        return t.float() if t.dtype == torch.float64 else t
    if isinstance(x, (list, tuple)) and x and all(isinstance(v, np.ndarray) for v in x):
        from ..utils.table import Table

        t = Table()
        for i, v in enumerate(x, 1):
            t[i] = to_torch(v)
        return t
    return x


def to_numpy(x):
    from ..utils.table import Table

    if isinstance(x, torch.Tensor):
        return x.detach().float().cpu().numpy() if x.is_floating_point() else x.detach().cpu().numpy()
    if isinstance(x, Table):
        return [to_numpy(x[i]) for i in range(1, x.length() + 1)]
    if isinstance(x, (list, tuple)):
        return [to_numpy(v) for v in x]
    return x


def convert_kwargs(cls, kwargs):
    """Map reference-style keyword arguments onto ``cls``'s constructor: drops ``bigdl_type``, converts
    snake_case names and numpy initial values. Unknown names raise TypeError naming the accepted ones."""
    kwargs = {k: v for k, v in kwargs.items() if k != "bigdl_type"}
    try:
        params = inspect.signature(cls.__init__).parameters
    except (TypeError, ValueError):
        params = {}
    accepts_var = any(p.kind == inspect.Parameter.VAR_KEYWORD for p in params.values())
    out = {}
    for k, v in kwargs.items():
        name = k if k in params else camel(k)
        if name not in params and not accepts_var:
            lower = {p.lower(): p for p in params}
            name = lower.get(k.replace("_", "").lower(), name)
        if name not in params and not accepts_var:
            raise TypeError(f"{cls.__name__}: unexpected argument {k!r} (accepts {list(params)[1:]})")
        out[name] = to_torch(v) if isinstance(v, np.ndarray) else v
    return out
