"""Caffe loader / persister (reference T/utils/CaffeLoaderSpec.scala, CaffePersisterSpec.scala) against the
reference's own fixtures (tests/fixtures/caffe/test.prototxt + test.caffemodel, copied from
spark/dl/src/test/resources/caffe)."""
import os

import pytest
import torch

from bigdl_amd import nn
from bigdl_amd.interop import caffe as C
from bigdl_amd.nn.module import Module

FIX = os.path.join(os.path.dirname(__file__), "fixtures", "caffe")
PROTO, MODEL = os.path.join(FIX, "test.prototxt"), os.path.join(FIX, "test.caffemodel")
DUMMY = {"Dummy": lambda layer: nn.Identity().setName("Dummy")}


def _static():
    return nn.Sequential().add(nn.SpatialConvolution(3, 4, 2, 2).setName("conv")) \
        .add(nn.SpatialConvolution(4, 3, 2, 2).setName("conv2")).add(nn.View(27).setName("view")) \
        .add(nn.Linear(27, 2, withBias=False).setName("ip")).add(nn.SoftMax().setName("softmax"))


def test_load_matches_reference_parameters():
    m = C.load_caffe_into(_static(), PROTO, MODEL, matchAll=True)
    p = m.getParametersTable()
    w = p["conv"]["weight"].reshape(-1)
    assert abs(float(w[0]) - 0.4156779647) < 1e-6 and abs(float(w[-1]) + 0.4590228796) < 1e-6
    assert torch.allclose(p["conv"]["bias"], torch.tensor([0.0458712392, -0.0029324144, -0.0251041390,
                                                            0.0052924110]), atol=1e-6)
    assert abs(float(p["conv2"]["weight"].reshape(-1)[0]) - 0.0154178329) < 1e-6
    assert torch.all(p["conv2"]["bias"] == 0)
    lw = p["ip"]["weight"].reshape(-1)
    assert abs(float(lw[0]) - 0.0189033747) < 1e-6 and abs(float(lw[-1]) - 0.2072965205) < 1e-6


def test_match_all_raises_on_missing_layer():
    m = _static()
    m.modules[1].setName("conv3")
    with pytest.raises(ValueError):
        C.load_caffe_into(m, PROTO, MODEL, matchAll=True)
    C.load_caffe_into(m, PROTO, MODEL, matchAll=False)


def test_dynamic_graph_equals_static_and_criterion():
    static = C.load_caffe_into(_static(), PROTO, MODEL)
    dyn, crit = C.load_caffe(PROTO, MODEL, customizedConverters=DUMMY)
    x = torch.rand(1, 3, 5, 5)
    assert torch.allclose(static.forward(x), dyn.forward(x), atol=1e-6)
    assert len(crit.criterions) == 1 and isinstance(crit.criterions[0], nn.ClassNLLCriterion)
    with pytest.raises(ValueError):
        C.load_caffe(PROTO, MODEL)          # unknown "Dummy" without a customized converter


def test_module_loaders_and_persist_roundtrip(tmp_path):
    dyn = Module.loadCaffeModel(PROTO, MODEL, DUMMY)
    assert isinstance(dyn, nn.Graph)
    static = C.load_caffe_into(_static(), PROTO, MODEL)
    pt, cm = str(tmp_path / "n.prototxt"), str(tmp_path / "n.caffemodel")
    static.saveCaffe(pt, cm, overwrite=True)
    back, _ = C.load_caffe(pt, cm)
    x = torch.rand(2, 3, 5, 5)
    assert torch.allclose(back.forward(x), static.forward(x), atol=1e-6)
    assert "convolution_param" in open(pt).read()


def test_text_format_parser_features():
    net = C.SCHEMA.parse_text("NetParameter", '''
        name: "n"  # comment
        input: "data" input_dim: 1 input_dim: 3
        layer { name: 'p' type: "Pooling" bottom: "data" top: "p"
                pooling_param { pool: AVE kernel_size: 3 stride: 2 global_pooling: false } }
        layer < name: "r" type: "ReLU" bottom: "p" top: "p" relu_param { negative_slope: 0.1 } >''')
    l0, l1 = net["layer"]
    assert C._g(C._g(l0, "pooling_param"), "pool") == "AVE" and C._g(l1, "name") == "r"
    assert abs(C._g(C._g(l1, "relu_param"), "negative_slope") - 0.1) < 1e-9
    enc = C.SCHEMA.encode("NetParameter", net)
    assert C.SCHEMA.decode("NetParameter", enc)["layer"][0]["pooling_param"][0]["pool"] == ["AVE"]


def test_recurrent_layer_roundtrip(tmp_path):
    """Caffe "Recurrent" / "RNN" layers (Converter.scala:200-202,653-654; LayerConverter.scala:530-532): export writes
    type Recurrent with the cell's weights as blobs; import builds a bare Recurrent container of that name, and
    load_caffe_into puts the blobs back into a model that has the cell."""
    torch.manual_seed(0)

    def build():
        return nn.Sequential().add(nn.Recurrent().add(nn.LSTM(4, 6, 0)).setName("rnn1")) \
            .add(nn.Select(2, -1)).add(nn.Linear(6, 3).setName("fc"))

    src = build()
    pt, cm = str(tmp_path / "r.prototxt"), str(tmp_path / "r.caffemodel")
    C.save_caffe(nn.Sequential().add(src.modules[0]), pt, cm, overwrite=True)
    text = open(pt).read()
    assert 'type: "Recurrent"' in text and 'name: "rnn1"' in text
    g, _ = C.load_caffe(pt, cm)
    rec = [m for m in g.flattened_layers() if isinstance(m, nn.Recurrent)] or \
          [n.element for n in g.order if isinstance(n.element, nn.Recurrent)]
    assert rec and rec[0].getName() == "rnn1" and rec[0].cell is None
    # the same prototxt with the legacy "RNN" type string
    open(pt, "w").write(text.replace('type: "Recurrent"', 'type: "RNN"'))
    g2, _ = C.load_caffe(pt)
    assert any(isinstance(n.element, nn.Recurrent) for n in g2.order)
    # weights back into a model with the cell
    dst = build()
    C.load_caffe_into(dst, pt, cm, matchAll=False)
    for a, b in zip(src.modules[0].parameters()[0], dst.modules[0].parameters()[0]):
        assert torch.equal(a, b)
