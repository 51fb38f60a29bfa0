"""Keras 1.2.2 JSON + weights -> bigdl_amd.keras (reference P/keras/converter.py; T: pyspark keras test_load_model /
test_layer compare against Keras itself — Keras is not installed here, so the expected outputs are computed from the
Keras 1 layer equations in numpy: parity vs the Keras runtime is unpinned)."""
import json

import numpy as np
import torch

from bigdl_amd.keras.converter import DefinitionLoader, WeightLoader, load_keras


def _hard_sigmoid(x):
    return np.clip(0.2 * x + 0.5, 0, 1)


def test_sequential_dense_conv_json():
    cfg = {"class_name": "Sequential", "config": [
        {"class_name": "Convolution2D", "config": {"name": "conv1", "nb_filter": 4, "nb_row": 3, "nb_col": 3,
                                                   "activation": "relu", "border_mode": "same", "subsample": [1, 1],
                                                   "dim_ordering": "th", "bias": True,
                                                   "batch_input_shape": [None, 2, 6, 6]}},
        {"class_name": "Flatten", "config": {"name": "flat"}},
        {"class_name": "Dense", "config": {"name": "fc", "output_dim": 3, "activation": "softmax", "bias": True}},
    ]}
    m = DefinitionLoader.from_json_str(json.dumps(cfg))
    rng = np.random.default_rng(0)
    W = rng.standard_normal((4, 2, 3, 3)).astype(np.float32)
    b = rng.standard_normal(4).astype(np.float32)
    Wd = rng.standard_normal((144, 3)).astype(np.float32)
    bd = rng.standard_normal(3).astype(np.float32)
    WeightLoader.load_weights_from_dict(m, {"conv1": [W, b], "fc": [Wd, bd]})
    x = rng.standard_normal((2, 2, 6, 6)).astype(np.float32)
    y = m.forward(torch.from_numpy(x)).numpy()
    conv = torch.nn.functional.conv2d(torch.from_numpy(x), torch.from_numpy(W), torch.from_numpy(b), padding=1)
    h = torch.relu(conv).reshape(2, -1).numpy() @ Wd + bd
    ref = np.exp(h) / np.exp(h).sum(1, keepdims=True)
    assert np.allclose(y, ref, atol=1e-5)


def test_lstm_gru_weights_follow_keras_equations():
    rng = np.random.default_rng(1)
    T_, D, H = 4, 3, 5
    x = rng.standard_normal((2, T_, D)).astype(np.float32)
    for kind in ("LSTM", "GRU"):
        cfg = {"class_name": "Sequential", "config": [
            {"class_name": kind, "config": {"name": "rnn", "output_dim": H, "return_sequences": False,
                                            "activation": "tanh", "inner_activation": "hard_sigmoid",
                                            "batch_input_shape": [None, T_, D]}}]}
        m = DefinitionLoader.from_config(cfg)
        gates = ["i", "c", "f", "o"] if kind == "LSTM" else ["z", "r", "h"]
        ws, P = [], {}
        for g in gates:
            P[g] = (rng.standard_normal((D, H)).astype(np.float32) * 0.5,
                    rng.standard_normal((H, H)).astype(np.float32) * 0.5,
                    rng.standard_normal(H).astype(np.float32) * 0.1)
            ws += list(P[g])
        WeightLoader.load_weights_from_dict(m, {"rnn": ws})
        y = m.forward(torch.from_numpy(x)).numpy()
        h = np.zeros((2, H), np.float32)
        c = np.zeros((2, H), np.float32)
        for t in range(T_):
            xt = x[:, t]
            if kind == "LSTM":
                i = _hard_sigmoid(xt @ P["i"][0] + h @ P["i"][1] + P["i"][2])
                f = _hard_sigmoid(xt @ P["f"][0] + h @ P["f"][1] + P["f"][2])
                cc = np.tanh(xt @ P["c"][0] + h @ P["c"][1] + P["c"][2])
                o = _hard_sigmoid(xt @ P["o"][0] + h @ P["o"][1] + P["o"][2])
                c = f * c + i * cc
                h = o * np.tanh(c)
            else:
                z = _hard_sigmoid(xt @ P["z"][0] + h @ P["z"][1] + P["z"][2])
                r = _hard_sigmoid(xt @ P["r"][0] + h @ P["r"][1] + P["r"][2])
                hh = np.tanh(xt @ P["h"][0] + (r * h) @ P["h"][1] + P["h"][2])
                h = z * h + (1 - z) * hh
        assert np.allclose(y, h, atol=1e-4), kind


def test_functional_model_json():
    cfg = {"class_name": "Model", "config": {
        "layers": [
            {"name": "in1", "class_name": "InputLayer", "config": {"batch_input_shape": [None, 4], "name": "in1"},
             "inbound_nodes": []},
            {"name": "d1", "class_name": "Dense", "config": {"output_dim": 3, "name": "d1"},
             "inbound_nodes": [[["in1", 0, 0]]]},
            {"name": "d2", "class_name": "Dense", "config": {"output_dim": 3, "name": "d2"},
             "inbound_nodes": [[["in1", 0, 0]]]},
            {"name": "m", "class_name": "Merge", "config": {"mode": "sum", "name": "m"},
             "inbound_nodes": [[["d1", 0, 0], ["d2", 0, 0]]]},
        ],
        "input_layers": [["in1", 0, 0]], "output_layers": [["m", 0, 0]]}}
    w1, w2 = np.ones((4, 3), np.float32), 2 * np.ones((4, 3), np.float32)
    m = load_keras(json_str=json.dumps(cfg), weights={"d1": [w1, np.zeros(3, np.float32)],
                                                      "d2": [w2, np.ones(3, np.float32)]})
    x = torch.randn(2, 4)
    assert torch.allclose(m.forward(x), x @ torch.from_numpy(w1 + w2) + 1, atol=1e-5)
