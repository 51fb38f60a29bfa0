"""Loader for the in-tree native HIP extension (``bigdl_amd/_C*.so``).

GPU tensors are always routed to the native kernels: if the extension is missing on a machine with a GPU
the call raises instead of silently falling back to another implementation.
"""
import os

_C = None
_ERR = None


def get():
    """Return the native module or raise a RuntimeError explaining how to build it."""
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        from bigdl_amd import _C as mod  # noqa: WPS433
    except ImportError as e:  # pragma: no cover - depends on build state
        _ERR = e
        raise RuntimeError(
            "bigdl_amd native extension (bigdl_amd/_C*.so) is not built or failed to load: "
            f"{e}. Build it with `python setup.py build_ext --inplace` (hipcc --offload-arch=gfx950)."
        ) from e
    _C = mod
    return _C


def available():
    try:
        get()
        return True
    except RuntimeError:
        return False


def so_path():
    mod = get()
    return os.path.abspath(mod.__file__)
