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


class PersistentKernelTimeout(RuntimeError):
    """A whole-sequence persistent kernel (csrc/lstm_seq.hip) gave up waiting for a co-resident workgroup: its
    outputs of that launch are NaN-poisoned and the iteration must not be trusted."""


def check_persistent(clear=True):
    """Raise PersistentKernelTimeout if a persistent kernel recorded a timeout since the last check. Reads a
    host-mapped word the kernels write with system scope: no device synchronisation. Called by every persistent
    launch site and by ``TrainStep.throttle`` once the device has finished an iteration."""
    if _C is None:
        return
    n = int(_C.persistent_error(bool(clear)))
    if n:
        raise PersistentKernelTimeout(
            "a persistent recurrent kernel timed out waiting for a co-resident workgroup (another stream held CUs "
            "past the bound set by set_seq_timeout_us); the affected outputs were poisoned with NaN")
