"""Torch7 .t7 reader/writer (reference T/utils/TorchFileSpec + the t7 image fixtures in
spark/dl/src/test/resources/torch, read when present)."""
import glob
import os

import pytest
import torch

from bigdl_amd import nn
from bigdl_amd.interop.torchfile import TorchObject, load_torch, read_t7, save_torch, write_t7
from bigdl_amd.nn.module import Module

REF_T7 = sorted(glob.glob("/root/reference/spark/dl/src/test/resources/torch/*.t7"))


@pytest.mark.skipif(not REF_T7, reason="reference t7 fixtures not present")
def test_reads_reference_tensors():
    for f in REF_T7:
        t = read_t7(f)
        assert t.shape == (3, 224, 224) and t.dtype == torch.float32 and torch.isfinite(t).all()


def test_tensor_table_roundtrip(tmp_path):
    p = str(tmp_path / "a.t7")
    obj = {"x": torch.arange(6.0).reshape(2, 3).t(), "n": 3, "s": "hi", "b": True,
           "l": torch.tensor([1, 2], dtype=torch.int64)}
    write_t7(p, obj)
    back = read_t7(p)
    assert torch.equal(back["x"], obj["x"]) and back["n"] == 3 and back["s"] == "hi" and back["b"] is True
    assert back["l"].dtype == torch.int64


def test_module_roundtrip(tmp_path):
    m = nn.Sequential().add(nn.SpatialConvolution(3, 4, 3, 3, 1, 1, 1, 1)).add(nn.SpatialBatchNormalization(4)) \
        .add(nn.ReLU()).add(nn.SpatialMaxPooling(2, 2, 2, 2)).add(nn.View(4 * 4 * 4)) \
        .add(nn.Linear(64, 5)).add(nn.LogSoftMax())
    m.evaluate()
    p = str(tmp_path / "m.t7")
    m.saveTorch(p)
    back = Module.loadTorch(p)
    back.evaluate()
    x = torch.randn(2, 3, 8, 8)
    assert torch.allclose(back.forward(x), m.forward(x), atol=1e-6)
    with pytest.raises(FileExistsError):
        save_torch(m, p)


def test_refuses_lua_functions(tmp_path):
    import struct

    p = tmp_path / "f.t7"
    p.write_bytes(struct.pack("<i", 6) + b"\0" * 8)
    with pytest.raises(ValueError):
        read_t7(str(p))
