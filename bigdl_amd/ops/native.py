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
    _check_build()          # raises on a stale build under BIGDL_STRICT_BUILD=1 before the module is published
    if hasattr(mod, "set_deterministic"):
        mod.set_deterministic(1 if _DET[0] else 0)
    _C = mod
    return _C


BUILD_INFO = None


def _check_build():
    """Compare the content hash recorded at build time (bigdl_amd/_build_info.json, setup.py) with the sources in
    this tree: a stale extension warns, or raises with BIGDL_STRICT_BUILD=1. Trees without csrc/ (installed copies)
    skip the comparison."""
    global BUILD_INFO
    import json
    import warnings

    pkg = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    path = os.path.join(pkg, "_build_info.json")
    try:
        with open(path) as f:
            BUILD_INFO = json.load(f)
    except OSError:
        BUILD_INFO = None
        return
    root = os.path.dirname(pkg)
    if not os.path.isdir(os.path.join(root, "csrc")):
        return
    from .. import _buildhash

    now = _buildhash.source_digest(root, BUILD_INFO.get("hip_flags", []))
    BUILD_INFO["source_matches"] = now == BUILD_INFO.get("source_sha256")
    if not BUILD_INFO["source_matches"]:
        msg = ("bigdl_amd/_C was built from different sources than csrc/ in this tree (stale build): "
               "run `python setup.py build_ext --inplace`")
        if os.environ.get("BIGDL_STRICT_BUILD", "0") == "1":
            raise RuntimeError(msg)
        warnings.warn(msg, RuntimeWarning, stacklevel=3)


def available():
    try:
        get()
        return True
    except RuntimeError:
        return False


def so_path():
    mod = get()
    return os.path.abspath(mod.__file__)


_DET = [os.environ.get("BIGDL_DETERMINISTIC", "0") not in ("0", "", "false", "False")]


def deterministic():
    """Deterministic mode (``bigdl.deterministic`` / BIGDL_DETERMINISTIC=1): every GPU reduction that would land
    through float atomics from several workgroups runs in a fixed order instead (BN statistics and backward sums in
    one-writer slots outside the GEMM epilogues, weight gradients through workspace partials + a fixed-order reduce,
    bias gradients, loss and norms in one row block), so two training runs from the same seed are bitwise equal.
    Costs speed (tools/det_check.py records how much)."""
    return _DET[0]


def set_deterministic(on=True):
    _DET[0] = bool(on)
    if _C is not None:
        _C.set_deterministic(1 if on else 0)


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
