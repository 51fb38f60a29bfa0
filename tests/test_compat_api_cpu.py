"""Reference-style Python scripts run against the bigdl_amd facade (reference P/models/lenet/lenet5.py +
utils.py, P/optim/optimizer.py, P/nn/layer.py, P/util/common.py). The LeNet script body below is the
reference's build_model / preprocess / Optimizer / set_validation / set_checkpoint / optimize / Model.load /
evaluate flow with ``from bigdl.* import *`` imports, on synthetic MNIST-shaped data (no downloads)."""
import os
import sys

import numpy as np
import pytest


@pytest.fixture
def bigdl():
    import bigdl_amd.compat as compat

    saved = {k: sys.modules.get(k) for k in compat._MODULES}
    compat.install()
    yield
    for k, v in saved.items():
        if v is None:
            sys.modules.pop(k, None)
        else:
            sys.modules[k] = v


LENET = '''
from bigdl.dataset import mnist
from bigdl.dataset.transformer import *
from bigdl.nn.layer import *
from bigdl.nn.criterion import *
from bigdl.optim.optimizer import *
from bigdl.util.common import *


def build_model(class_num):
    model = Sequential()
    model.add(Reshape([1, 28, 28]))
    model.add(SpatialConvolution(1, 6, 5, 5))
    model.add(Tanh())
    model.add(SpatialMaxPooling(2, 2, 2, 2))
    model.add(SpatialConvolution(6, 12, 5, 5))
    model.add(Tanh())
    model.add(SpatialMaxPooling(2, 2, 2, 2))
    model.add(Reshape([12 * 4 * 4]))
    model.add(Linear(12 * 4 * 4, 100))
    model.add(Tanh())
    model.add(Linear(100, class_num))
    model.add(LogSoftMax())
    return model


def get_mnist(sc, images, labels):
    images = sc.parallelize(images)
    labels = sc.parallelize(labels + 1)  # Target start from 1 in BigDL
    return images.zip(labels)


def run(images, labels, ckpt):
    sc = SparkContext(appName="lenet5", conf=create_spark_conf())
    redire_spark_logs(log_path=ckpt + "/bigdl.log")
    show_bigdl_info_logs()
    init_engine()
    train_data = get_mnist(sc, images, labels)\\
        .map(lambda rec_tuple: (normalizer(rec_tuple[0], mnist.TRAIN_MEAN, mnist.TRAIN_STD), rec_tuple[1]))\\
        .map(lambda t: Sample.from_ndarray(t[0], t[1]))
    test_data = train_data
    optimizer = Optimizer(
        model=build_model(10),
        training_rdd=train_data,
        criterion=ClassNLLCriterion(),
        optim_method=SGD(learningrate=0.05, learningrate_decay=0.0002),
        end_trigger=MaxEpoch(3),
        batch_size=16)
    optimizer.set_validation(batch_size=16, val_rdd=test_data, trigger=EveryEpoch(), val_method=[Top1Accuracy()])
    optimizer.set_checkpoint(EveryEpoch(), ckpt)
    trained_model = optimizer.optimize()
    parameters = trained_model.parameters()
    model = Model.load(ckpt + "/model.latest")
    results = model.evaluate(test_data, 16, [Top1Accuracy()])
    sc.stop()
    return trained_model, parameters, results
'''


def test_reference_lenet_script_trains_checkpoints_and_evaluates(bigdl, tmp_path):
    rng = np.random.RandomState(0)
    labels = rng.randint(0, 10, size=96).astype(np.float32)
    # learnable synthetic digits: a class-dependent bright bar on noise
    images = rng.randint(0, 60, size=(96, 28, 28, 1)).astype(np.float32)
    for i, l in enumerate(labels.astype(int)):
        images[i, 2 * l + 3:2 * l + 6, 4:24, 0] = 250
    ns = {}
    exec(compile(LENET, "lenet5_reference_style.py", "exec"), ns)
    model, params, results = ns["run"](images.reshape(96, 784), labels, str(tmp_path))
    assert os.path.exists(tmp_path / "model.latest")
    assert set(params) and all("weight" in v for v in params.values())
    acc = results[0].result
    assert results[0].total_num == 96 and acc > 0.5, acc
    # the trained model predicts with the ndarray API
    pred = model.predict_class(images.reshape(96, 784))
    assert pred.shape == (96,) and pred.min() >= 1


def test_local_optimizer_and_layer_ndarray_api(bigdl):
    from bigdl.nn.criterion import MSECriterion
    from bigdl.nn.layer import Linear, Model, Input, ReLU, Sequential
    from bigdl.optim.optimizer import Adam, MaxIteration, Optimizer
    from bigdl.util.common import JTensor, Sample

    rng = np.random.RandomState(1)
    X = rng.randn(64, 4).astype(np.float32)
    W = rng.randn(4, 2).astype(np.float32)
    Y = X @ W
    inp = Input()
    out = Linear(4, 2, with_bias=False)(inp)
    model = Model([inp], [out])
    opt = Optimizer.create(model, (X, Y), MSECriterion(), MaxIteration(300), 16, Adam(learningrate=0.05))
    trained = opt.optimize()
    assert np.abs(trained.forward(X) - Y).mean() < 0.05
    seq = Sequential().add(Linear(4, 3)).add(ReLU())
    w = [np.ones((3, 4), np.float32), np.zeros(3, np.float32)]
    seq.set_weights(w)
    assert np.allclose(seq.get_weights()[0], 1.0)
    seq.forward(X[:2])
    g = seq.backward(X[:2], np.ones((2, 3), np.float32))
    assert g.shape == (2, 4)
    seq.zero_grad_parameters()
    s = Sample.from_ndarray(np.arange(6).reshape(2, 3), np.array([1.0]))
    assert s.feature.to_ndarray().shape == (2, 3)
    assert np.allclose(JTensor.sparse(np.array([1.0, 2.0]), np.array([0, 1, 1, 2]), [2, 3]).to_ndarray(),
                       [[0, 1, 0], [0, 0, 2]])


def test_snake_case_keywords_map_to_engine_arguments(bigdl):
    from bigdl.nn.layer import SpatialConvolution, Linear
    from bigdl.optim.optimizer import SGD, Plateau, SequentialSchedule, Warmup, Poly

    conv = SpatialConvolution(n_input_plane=3, n_output_plane=4, kernel_w=3, kernel_h=3, stride_w=2, pad_w=1,
                              pad_h=1, with_bias=False, bigdl_type="float")
    assert conv.value.nInputPlane == 3 and conv.value.strideW == 2 and conv.value.bias is None
    lin = Linear(2, 3, init_weight=np.ones((3, 2), np.float32), init_bias=np.zeros(3, np.float32))
    assert np.allclose(lin.get_weights()[0], 1.0)
    with pytest.raises(TypeError):
        Linear(2, 3, no_such_argument=1)
    sched = SequentialSchedule(5).add(Warmup(0.1), 3).add(Poly(0.5, 100), 100)
    sgd = SGD(learningrate=0.1, momentum=0.9, leaningrate_schedule=sched)
    assert sgd.value.momentum == 0.9 and sgd.value.learningRateSchedule is sched.value
    assert Plateau("score").value is not None


def test_initialization_method_and_dataset_base_modules(tmp_path, capsys):
    import torch

    from bigdl_amd.compat.dataset.base import Progbar, display_table, maybe_download
    from bigdl_amd.compat.nn import initialization_method as im

    w = torch.empty(100, 50)
    im.RandomUniform(0.5, -0.5).init(w)           # reference order: (upper, lower)
    assert float(w.min()) >= -0.5 and float(w.max()) <= 0.5 and float(w.max()) > 0.4
    im.ConstInitMethod(3.0).init(w)
    assert float(w.mean()) == 3.0
    for cls in (im.Zeros, im.Ones, im.Xavier, im.MsraFiller, im.BilinearFiller):
        assert isinstance(cls(), im.InitializationMethod)
    assert isinstance(im.RandomNormal(0.0, 1.0), im.InitializationMethod)
    p = Progbar(10)
    p.update(5, [("loss", 1.0)])
    p.add(5, [("loss", 3.0)])
    display_table([["a", "b"]], [5, 10])
    out = capsys.readouterr().out
    assert "10/10" in out and "loss: 2.0000" in out and out.rstrip().endswith("b")
    (tmp_path / "f.bin").write_bytes(b"x")
    assert maybe_download("f.bin", str(tmp_path)) == str(tmp_path / "f.bin")
    try:
        maybe_download("missing.bin", str(tmp_path), "http://example")
        raise AssertionError("expected FileNotFoundError")
    except FileNotFoundError:
        pass


def test_reference_dataset_helper_modules(tmp_path):
    import numpy as np

    from bigdl_amd.compat.dataset import movielens, news20, sentence

    root = tmp_path / "20news-18828"
    for i, grp in enumerate(["alt.atheism", "comp.graphics"]):
        (root / grp).mkdir(parents=True)
        (root / grp / "101").write_text(f"text {i}", encoding="latin-1")
        (root / grp / "notes.txt").write_text("skip")
    texts = news20.get_news20(str(tmp_path))
    assert texts == [("text 0", 1), ("text 1", 2)]
    (tmp_path / "glove.6B").mkdir()
    (tmp_path / "glove.6B" / "glove.6B.2d.txt").write_text("the 0.5 -1\ncat 1 2\n")
    assert news20.get_glove_w2v(str(tmp_path), 2)["cat"] == [1.0, 2.0]
    (tmp_path / "ml-1m").mkdir()
    (tmp_path / "ml-1m" / "ratings.dat").write_text("1::10::5::999\n2::20::3::998\n")
    assert np.array_equal(movielens.get_id_ratings(str(tmp_path)), np.array([[1, 10, 5], [2, 20, 3]]))
    assert sentence.sentences_split("Hello there. How are you?") == ["Hello there.", "How are you?"]
    assert sentence.sentence_tokenizer("Hi, you.") == ["Hi", ",", "you", "."]
    assert sentence.sentences_bipadding("a b") == "SENTENCESTART a b SENTENCEEND"


def test_reference_engine_version_and_model_broadcast(tmp_path, monkeypatch):
    """bigdl.util.engine version helpers / prepare_env, bigdl.version, and bigdl.models.utils.model_broadcast:
    a broadcast handle pickles to its saved path and loads an independent copy with the same outputs."""
    import pickle
    import sys

    import numpy as np

    from bigdl_amd import compat

    compat.install()
    from bigdl.models.utils.model_broadcast import broadcast_model
    from bigdl.nn.layer import Linear, Sequential, ReLU
    from bigdl.util.common import SparkContext
    from bigdl.util.engine import compare_version, get_bigdl_classpath, is_spark_below_2_2, prepare_env
    from bigdl.version import __version__

    assert compare_version("2.10", "2.2") == 1 and compare_version("1.6", "2.2") == -1
    assert compare_version("2.2.0", "2.2") == 0 and __version__.startswith("0.")
    assert is_spark_below_2_2() is False and get_bigdl_classpath() == ""
    monkeypatch.setenv("BIGDL_PACKAGES", str(tmp_path))
    monkeypatch.setattr(sys, "path", list(sys.path))
    prepare_env()
    assert sys.path[0] == str(tmp_path)

    model = Sequential().add(Linear(4, 3)).add(ReLU())
    bc = broadcast_model(SparkContext(), model)
    assert bc.value is model
    remote = pickle.loads(pickle.dumps(bc))            # what a task would receive
    x = np.random.RandomState(0).randn(2, 4).astype(np.float32)
    got = remote.value
    assert got is not model
    np.testing.assert_allclose(got.forward(x), model.forward(x), rtol=1e-6, atol=1e-6)
    bc.unpersist()


def test_reference_onnx_layers():
    """bigdl.nn.onnx.layer (P/nn/onnx/layer.py) over nn.onnx Shape / Reshape (S/nn/onnx/*.scala), nn.Gemm,
    tf Const and Gather: ONNX semantics (0 copies a size, shape from a Table input, float sizes)."""
    import numpy as np
    import torch

    from bigdl_amd import compat
    from bigdl_amd.nn import onnx as nn_onnx
    from bigdl_amd.utils.table import T

    compat.install()
    from bigdl.nn.onnx.layer import Constant, Gather, Gemm, Reshape, Shape

    x = np.random.RandomState(0).rand(2, 3, 4).astype(np.float32)
    assert Shape().forward(x).tolist() == [2.0, 3.0, 4.0]
    assert Reshape([0, -1]).forward(x).shape == (2, 12)
    np.testing.assert_array_equal(Constant(np.ones((2, 2))).forward(x), np.ones((2, 2)))
    b, c = np.random.RandomState(1).rand(5, 4), np.random.RandomState(2).rand(3, 5)
    a = np.random.RandomState(3).rand(3, 4).astype(np.float32)
    np.testing.assert_allclose(Gemm(b, c, 0.5, 2.0, 0, 1).forward(a), 0.5 * a @ b.T + 2.0 * c, rtol=1e-5)
    got = Gather().forward([np.arange(12, dtype=np.float32).reshape(4, 3), np.array([2, 0], dtype=np.int32)])
    np.testing.assert_array_equal(got, [[6, 7, 8], [0, 1, 2]])

    r = nn_onnx.Reshape()
    data = torch.arange(24.0).reshape(2, 3, 4)
    y = r.forward(T(data, torch.tensor([4.0, 6.0])))
    assert y.shape == (4, 6) and r.shape == [4, 6]
    gi = r.backward(T(data, torch.tensor([4.0, 6.0])), torch.ones(4, 6))
    assert gi[1].shape == (2, 3, 4)
    try:
        nn_onnx.Reshape().forward(data)
        raise AssertionError("expected ValueError")
    except ValueError:
        pass


def test_reference_keras_layer_and_topology():
    """bigdl.nn.keras.layer / topology (P/nn/keras/*.py): snake_case keywords (input_dim, W_regularizer,
    batch_size, nb_epoch) over the engine's keras layers; Sequential and functional Model train / predict."""
    import numpy as np

    from bigdl_amd import compat

    compat.install()
    from bigdl.nn.keras.layer import Activation, Dense
    from bigdl.nn.keras.topology import Input, Model, Sequential

    rs = np.random.RandomState(0)
    x = rs.rand(64, 4).astype(np.float32)
    y = np.eye(3)[rs.randint(0, 3, 64)].astype(np.float32)
    m = Sequential().add(Dense(8, input_dim=4, activation="relu", W_regularizer=None)).add(Dense(3)) \
        .add(Activation("softmax"))
    m.compile("sgd", "categorical_crossentropy")
    m.fit(x, y, batch_size=16, nb_epoch=2)
    p = m.predict(x)
    assert p.shape == (64, 3) and np.allclose(p.sum(1), 1.0, atol=1e-5)
    assert m.get_output_shape()[-1] == 3

    inp = Input(shape=(4,))
    out = Dense(2)(inp)
    fm = Model(inp, out)
    assert fm.predict(x).shape == (64, 2)


def test_reference_vision_image_facade():
    """bigdl.transform.vision.image (P/transform/vision/image.py): snake_case transformer constructors over the
    engine transformers, LocalImageFrame from ndarrays, get_image (CHW) / get_label, same values as the engine."""
    import numpy as np
    import torch

    from bigdl_amd import compat
    from bigdl_amd.transform.vision import image as eng

    compat.install()
    from bigdl.transform.vision.image import ChannelNormalize, LocalImageFrame, MatToTensor, Resize

    rs = np.random.RandomState(0)
    imgs = [(rs.rand(20, 30, 3) * 255).astype(np.float32) for _ in range(2)]
    frame = LocalImageFrame(imgs, [np.array([1.0]), np.array([2.0])])
    for t in (Resize(resize_h=10, resize_w=12), ChannelNormalize(100.0, 110.0, 120.0), MatToTensor(to_rgb=False)):
        frame = frame.transform(t)
    got = frame.get_image()
    assert frame.is_local() and [g.shape for g in got] == [(3, 10, 12)] * 2
    assert [l.tolist() for l in frame.get_label()] == [[1.0], [2.0]]
    f = eng.ImageFeature()
    f[eng.ImageFeature.mat] = torch.as_tensor(imgs[0])
    f[eng.ImageFeature.originalSize] = imgs[0].shape
    for t in (eng.Resize(10, 12), eng.ChannelNormalize(100.0, 110.0, 120.0), eng.MatToTensor(toRGB=False)):
        f = t.transform(f)
    np.testing.assert_allclose(got[0], f[eng.ImageFeature.imageTensor].numpy(), rtol=1e-6, atol=1e-5)
