"""The start-up check that DEBUG_HIP_FORCE_GRAPH_QUEUES took effect (bigdl_amd/__init__.py GRAPH_ONE_QUEUE) and the
side-stream policy that follows from it: no forks inside a capture when the one-queue mode is not known to hold."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _probe(pre_env, init_first):
    code = ("import os, torch\n"
            + ("torch.cuda.is_initialized = lambda: True\n" if init_first else "")
            + "import warnings; warnings.simplefilter('ignore')\n"
            "import bigdl_amd; print(int(bigdl_amd.graph_one_queue()), os.environ['DEBUG_HIP_FORCE_GRAPH_QUEUES'])\n")
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("DEBUG_HIP_FORCE_GRAPH_QUEUES", None)
    if pre_env is not None:
        env["DEBUG_HIP_FORCE_GRAPH_QUEUES"] = pre_env
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    return out.stdout.split()


@pytest.mark.parametrize("pre_env,init_first,expect", [
    (None, False, ["1", "1"]),     # set by bigdl_amd before HIP starts: in effect
    (None, True, ["0", "1"]),      # HIP already initialised: setting it now cannot take effect
    ("1", True, ["1", "1"]),       # preset in the environment: in effect whatever the import order
    ("0", False, ["0", "0"]),      # explicitly disabled by the user: respected, forks disabled
])
def test_graph_queue_check(pre_env, init_first, expect):
    assert _probe(pre_env, init_first) == expect


def test_no_side_stream_fork_in_capture_without_one_queue(monkeypatch):
    import torch

    import bigdl_amd
    from bigdl_amd.ops import side_stream

    monkeypatch.setattr(bigdl_amd, "GRAPH_ONE_QUEUE", False)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: True)

    class FakeCuda:
        is_cuda = True

    t = torch.zeros(1)
    monkeypatch.setattr(torch.Tensor, "is_cuda", property(lambda self: True))
    assert side_stream.stream_for(t) is None
