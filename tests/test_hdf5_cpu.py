"""Native HDF5 reader / writer for Keras weight files (utils/hdf5.py; reference P/keras/converter.py
WeightLoader.load_weights_from_hdf5). h5py and .h5 fixtures are absent here, so files are produced by the native
writer in the Keras save_weights / model.save layouts: parity with h5py-written files is unpinned."""
import json

import numpy as np
import pytest
import torch

from bigdl_amd.utils.hdf5 import File, HDF5Error, read_keras_weights, write_h5, write_keras_weights


def test_write_read_tree_roundtrip(tmp_path):
    p = str(tmp_path / "t.h5")
    rng = np.random.default_rng(0)
    a = rng.standard_normal((3, 4)).astype(np.float32)
    b = np.arange(7, dtype=np.int64)
    c = rng.standard_normal((2, 2, 2)).astype(np.float64)
    tree = {"@attrs": {"title": "x", "names": ["alpha", "b", "gamma_long_name"], "scale": np.float32(2.5)},
            "a": a, "grp": {"@attrs": {"k": np.array([1, 2, 3], np.int32)}, "b": b, "deep": {"c": c}}}
    # enough members to need several symbol-table nodes under the group B-tree
    for i in range(20):
        tree[f"m{i:02d}"] = np.full((2,), i, np.float32)
    write_h5(p, tree)
    with File(p) as f:
        assert f.attrs["title"] == b"x"
        assert f.attrs["names"] == [b"alpha", b"b", b"gamma_long_name"]
        assert float(f.attrs["scale"]) == 2.5
        assert np.array_equal(f["a"][()], a)
        assert np.array_equal(f["grp/b"][()], b)
        assert np.array_equal(f["grp"]["deep/c"][()], c)
        assert list(f["grp"].attrs["k"]) == [1, 2, 3]
        assert sorted(k for k in f.keys() if k.startswith("m")) == [f"m{i:02d}" for i in range(20)]
        assert np.array_equal(f["m13"][()], np.full((2,), 13, np.float32))
        assert "grp/deep" in f and "nope" not in f


def test_not_hdf5_rejected(tmp_path):
    p = tmp_path / "x.h5"
    p.write_bytes(b"not an hdf5 file at all")
    with pytest.raises(HDF5Error):
        File(str(p))


def test_keras_weights_file_loads_into_model(tmp_path):
    from bigdl_amd.keras.converter import load_keras

    cfg = {"class_name": "Sequential", "config": [
        {"class_name": "Dense", "config": {"name": "fc1", "output_dim": 5, "activation": "relu", "bias": True,
                                           "batch_input_shape": [None, 4]}},
        {"class_name": "Dense", "config": {"name": "fc2", "output_dim": 3, "activation": "linear", "bias": True}},
    ]}
    rng = np.random.default_rng(1)
    w = {"fc1": [rng.standard_normal((4, 5)).astype(np.float32), rng.standard_normal(5).astype(np.float32)],
         "fc2": [rng.standard_normal((5, 3)).astype(np.float32), rng.standard_normal(3).astype(np.float32)]}
    h5 = str(tmp_path / "weights.h5")
    write_keras_weights(h5, w)
    got = read_keras_weights(h5)
    assert set(got) == {"fc1", "fc2"} and all(np.array_equal(g, e) for g, e in zip(got["fc1"], w["fc1"]))
    js = tmp_path / "model.json"
    js.write_text(json.dumps(cfg))
    m = load_keras(json_path=str(js), hdf5_path=h5)
    x = rng.standard_normal((2, 4)).astype(np.float32)
    ref = np.maximum(x @ w["fc1"][0] + w["fc1"][1], 0) @ w["fc2"][0] + w["fc2"][1]
    assert np.allclose(m.forward(torch.from_numpy(x)).numpy(), ref, atol=1e-5)


def test_model_save_layout_with_model_weights_group(tmp_path):
    p = str(tmp_path / "full.h5")
    W = np.ones((2, 3), np.float32)
    write_h5(p, {"@attrs": {"model_config": json.dumps({"class_name": "Sequential"})},
                 "model_weights": {"@attrs": {"layer_names": ["dense_1", "dropout_1"]},
                                   "dense_1": {"@attrs": {"weight_names": ["dense_1_W", "dense_1_b"]},
                                               "dense_1_W": W, "dense_1_b": np.zeros(3, np.float32)},
                                   "dropout_1": {}}})
    got = read_keras_weights(p)
    assert np.array_equal(got["dense_1"][0], W) and got["dropout_1"] == []
