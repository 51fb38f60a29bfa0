"""ConvertModel CLI, ThreadPool (invokeAndWait2 timeouts), LoggerFilter routing."""
import logging
import os
import time

import torch

from bigdl_amd import nn


def test_convert_model_bigdl_caffe_torch_roundtrip(tmp_path):
    from bigdl_amd.nn.module import Module
    from bigdl_amd.tools.convert_model import main

    torch.manual_seed(0)
    m = nn.Sequential().add(nn.SpatialConvolution(3, 4, 3, 3)).add(nn.ReLU()).add(nn.View(4 * 6 * 6)) \
        .add(nn.Linear(144, 5))
    m.evaluate()
    x = torch.randn(2, 3, 8, 8)
    ref = m.forward(x)
    src = str(tmp_path / "m.bigdl")
    m.saveModule(src, overWrite=True)
    assert main(["--from", "bigdl", "--to", "caffe", "--input", src, "--output", str(tmp_path / "c.caffemodel")]) == 0
    assert main(["--from", "caffe", "--to", "torch", "--prototxt", str(tmp_path / "c.prototxt"),
                 "--input", str(tmp_path / "c.caffemodel"), "--output", str(tmp_path / "t.t7")]) == 0
    t = Module.loadTorch(str(tmp_path / "t.t7"))
    t.evaluate()
    assert torch.allclose(t.forward(x), ref, atol=1e-5)
    assert main(["--from", "bigdl", "--to", "bigdl", "--input", src, "--output", str(tmp_path / "q.bigdl"),
                 "--quantize", "true"]) == 0


def test_thread_pool_invoke_and_wait2_cancels_stragglers():
    from bigdl_amd.utils.thread_pool import ThreadPool

    p = ThreadPool(4)
    assert p.invokeAndWait([lambda i=i: i * i for i in range(5)]) == [0, 1, 4, 9, 16]
    futs = p.invokeAndWait2([lambda: 1, lambda: time.sleep(0.5) or 2], timeout=0.1)
    assert futs[0].done() and futs[0].result() == 1
    assert not futs[1].done() or futs[1].cancelled() or futs[1].result() == 2
    p.shutdown()


def test_logger_filter_routes_third_party_to_file(tmp_path, monkeypatch):
    from bigdl_amd.utils.logger_filter import redirectSparkInfoLogs

    monkeypatch.setenv("BIGDL_LOGGERFILTER_LOGFILE", str(tmp_path / "bigdl.log"))
    path = redirectSparkInfoLogs()
    logging.getLogger("torch").info("third-party message")
    logging.getLogger("bigdl_amd.test").info("framework message")
    for h in logging.getLogger("torch").handlers + logging.getLogger("bigdl_amd").handlers:
        h.flush()
    text = open(path).read()
    for name in ("bigdl_amd", "torch", "urllib3", "matplotlib", "PIL", "filelock", "fsspec", "asyncio"):
        lg = logging.getLogger(name)
        for h in list(lg.handlers):
            lg.removeHandler(h)
            h.close()
        lg.propagate = True
        lg.setLevel(logging.NOTSET)
    assert "third-party message" in text and "framework message" in text
