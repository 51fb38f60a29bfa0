"""Keras-style API (reference T/nn/keras/*Spec: every layer's inferred output shape matches a forward pass;
Sequential / functional Model; compile+fit+evaluate+predict; serialization)."""
import os

import pytest
import torch

from bigdl_amd import keras as K
from bigdl_amd.utils.random_generator import RNG

CASES = [
    (lambda: K.Dense(5, activation="relu", inputShape=(7,)), (7,)),
    (lambda: K.Dense(5, inputShape=(4, 7)), (4, 7)),
    (lambda: K.Activation("tanh", inputShape=(6,)), (6,)),
    (lambda: K.Activation("softmax", inputShape=(3, 6)), (3, 6)),
    (lambda: K.Dropout(0.3, inputShape=(6,)), (6,)),
    (lambda: K.Flatten(inputShape=(2, 3, 4)), (2, 3, 4)),
    (lambda: K.Reshape([4, -1], inputShape=(2, 3, 4)), (2, 3, 4)),
    (lambda: K.Permute([2, 1], inputShape=(3, 5)), (3, 5)),
    (lambda: K.RepeatVector(4, inputShape=(5,)), (5,)),
    (lambda: K.Highway(activation="relu", inputShape=(6,)), (6,)),
    (lambda: K.MaxoutDense(3, 4, inputShape=(6,)), (6,)),
    (lambda: K.ELU(inputShape=(6,)), (6,)),
    (lambda: K.LeakyReLU(0.2, inputShape=(6,)), (6,)),
    (lambda: K.ThresholdedReLU(0.5, inputShape=(6,)), (6,)),
    (lambda: K.SReLU(inputShape=(4, 5)), (4, 5)),
    (lambda: K.Convolution1D(4, 3, inputShape=(10, 5)), (10, 5)),
    (lambda: K.Convolution1D(4, 3, borderMode="same", subsampleLength=2, inputShape=(10, 5)), (10, 5)),
    (lambda: K.AtrousConvolution1D(4, 3, atrousRate=2, inputShape=(12, 5)), (12, 5)),
    (lambda: K.Convolution2D(6, 3, 3, inputShape=(3, 10, 9)), (3, 10, 9)),
    (lambda: K.Convolution2D(6, 3, 3, borderMode="same", subsample=(2, 2), inputShape=(3, 10, 9)), (3, 10, 9)),
    (lambda: K.Convolution2D(6, 3, 3, dimOrdering="tf", inputShape=(10, 9, 3)), (10, 9, 3)),
    (lambda: K.AtrousConvolution2D(4, 3, 3, atrousRate=(2, 2), inputShape=(2, 12, 12)), (2, 12, 12)),
    (lambda: K.Deconvolution2D(4, 3, 3, subsample=(2, 2), inputShape=(2, 5, 5)), (2, 5, 5)),
    (lambda: K.SeparableConvolution2D(6, 3, 3, depthMultiplier=2, inputShape=(3, 8, 8)), (3, 8, 8)),
    (lambda: K.LocallyConnected1D(4, 3, inputShape=(8, 5)), (8, 5)),
    (lambda: K.LocallyConnected2D(4, 3, 3, inputShape=(2, 6, 6)), (2, 6, 6)),
    (lambda: K.Convolution3D(4, 2, 3, 3, inputShape=(2, 5, 6, 6)), (2, 5, 6, 6)),
    (lambda: K.MaxPooling1D(2, inputShape=(9, 4)), (9, 4)),
    (lambda: K.AveragePooling1D(3, 2, inputShape=(9, 4)), (9, 4)),
    (lambda: K.MaxPooling2D(inputShape=(3, 9, 8)), (3, 9, 8)),
    (lambda: K.AveragePooling2D((3, 3), (2, 2), borderMode="same", inputShape=(3, 9, 8)), (3, 9, 8)),
    (lambda: K.MaxPooling3D(inputShape=(2, 4, 6, 6)), (2, 4, 6, 6)),
    (lambda: K.AveragePooling3D(inputShape=(2, 4, 6, 6)), (2, 4, 6, 6)),
    (lambda: K.GlobalMaxPooling1D(inputShape=(7, 3)), (7, 3)),
    (lambda: K.GlobalAveragePooling1D(inputShape=(7, 3)), (7, 3)),
    (lambda: K.GlobalMaxPooling2D(inputShape=(3, 5, 6)), (3, 5, 6)),
    (lambda: K.GlobalAveragePooling2D(dimOrdering="tf", inputShape=(5, 6, 3)), (5, 6, 3)),
    (lambda: K.GlobalMaxPooling3D(inputShape=(2, 3, 4, 5)), (2, 3, 4, 5)),
    (lambda: K.GlobalAveragePooling3D(inputShape=(2, 3, 4, 5)), (2, 3, 4, 5)),
    (lambda: K.BatchNormalization(inputShape=(3, 5, 5)), (3, 5, 5)),
    (lambda: K.BatchNormalization(inputShape=(6,)), (6,)),
    (lambda: K.SimpleRNN(5, inputShape=(4, 3)), (4, 3)),
    (lambda: K.LSTM(5, returnSequences=True, inputShape=(4, 3)), (4, 3)),
    (lambda: K.GRU(5, goBackwards=True, inputShape=(4, 3)), (4, 3)),
    (lambda: K.Bidirectional(K.LSTM(5, returnSequences=True), inputShape=(4, 3)), (4, 3)),
    (lambda: K.ConvLSTM2D(4, 3, returnSequences=True, inputShape=(3, 2, 6, 6)), (3, 2, 6, 6)),
    (lambda: K.TimeDistributed(K.Dense(4), inputShape=(3, 6)), (3, 6)),
    (lambda: K.ZeroPadding1D(2, inputShape=(5, 3)), (5, 3)),
    (lambda: K.ZeroPadding2D((1, 2), inputShape=(3, 5, 5)), (3, 5, 5)),
    (lambda: K.ZeroPadding3D(inputShape=(2, 3, 3, 3)), (2, 3, 3, 3)),
    (lambda: K.Cropping1D((1, 2), inputShape=(8, 3)), (8, 3)),
    (lambda: K.Cropping2D((1, 1), (2, 0), inputShape=(2, 6, 6)), (2, 6, 6)),
    (lambda: K.Cropping3D(inputShape=(2, 5, 5, 5)), (2, 5, 5, 5)),
    (lambda: K.UpSampling1D(2, inputShape=(4, 3)), (4, 3)),
    (lambda: K.UpSampling2D(inputShape=(2, 4, 3)), (2, 4, 3)),
    (lambda: K.UpSampling3D(inputShape=(2, 2, 3, 3)), (2, 2, 3, 3)),
    (lambda: K.GaussianNoise(0.1, inputShape=(6,)), (6,)),
    (lambda: K.GaussianDropout(0.1, inputShape=(6,)), (6,)),
    (lambda: K.SpatialDropout1D(0.2, inputShape=(4, 6)), (4, 6)),
    (lambda: K.SpatialDropout2D(0.2, inputShape=(3, 4, 4)), (3, 4, 4)),
    (lambda: K.SpatialDropout3D(0.2, inputShape=(2, 3, 4, 4)), (2, 3, 4, 4)),
    (lambda: K.Masking(0.0, inputShape=(4, 3)), (4, 3)),
    (lambda: K.Embedding(20, 6, inputShape=(5,)), (5,)),
]


@pytest.mark.parametrize("i", range(len(CASES)))
def test_layer_shape_inference(i):
    RNG.setSeed(i)
    build, shape = CASES[i]
    m = K.Sequential().add(build())
    if isinstance(m.labor.modules[0], K.Embedding):
        x = torch.randint(0, 20, (3,) + shape).float()
    else:
        x = torch.randn((3,) + shape)
    m.training()
    y = m.forward(x)
    assert list(y.shape[1:]) == list(m.getOutputShape()[1:]), (list(y.shape), m.getOutputShape())
    y.sum()
    g = m.backward(x, torch.ones_like(y))
    assert g.shape == x.shape


def test_sequential_fit_evaluate_predict():
    RNG.setSeed(3)
    torch.manual_seed(3)
    x = torch.randn(256, 8)
    w = torch.randn(8, 3)
    y = (x @ w).argmax(1).float() + 1
    m = K.Sequential()
    m.add(K.Dense(32, activation="relu", inputShape=(8,)))
    m.add(K.Dense(3))
    m.add(K.Activation("softmax"))
    m.compile(optimizer="adam", loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    m.fit(x, y, batchSize=32, nbEpoch=15)
    res = m.evaluate(x, y, batchSize=64)
    acc = res[0][0].result()[0]
    assert acc > 0.8
    p = m.predict(x[:10])
    assert p.shape == (10, 3) and torch.allclose(p.sum(1), torch.ones(10), atol=1e-5)


def test_functional_model_with_merge(tmp_path):
    RNG.setSeed(5)
    a = K.Input(inputShape=(6,))
    b = K.Input(inputShape=(4,))
    ha = K.Dense(5, activation="tanh")(a)
    hb = K.Dense(5)(b)
    s = K.merge([ha, hb], mode="sum")
    c = K.merge([ha, hb], mode="concat")
    out = K.Dense(2)(K.merge([s, c], mode="concat"))
    model = K.Model([a, b], out)
    assert model.getOutputShape() == [None, 2]
    from bigdl_amd.utils.table import T
    xa, xb = torch.randn(3, 6), torch.randn(3, 4)
    y = model.forward(T(xa, xb))
    assert y.shape == (3, 2)
    p = os.path.join(tmp_path, "kmodel.bigdl")
    model.saveModule(p, overWrite=True)
    from bigdl_amd.nn.module import Module
    m2 = Module.loadModule(p)
    assert torch.allclose(m2.forward(T(xa, xb)), y)


def test_sequential_serialization(tmp_path):
    RNG.setSeed(9)
    m = K.Sequential()
    m.add(K.Convolution2D(4, 3, 3, activation="relu", inputShape=(2, 8, 8)))
    m.add(K.Flatten()).add(K.Dense(3, activation="softmax"))
    m.evaluate()
    x = torch.randn(2, 2, 8, 8)
    y = m.forward(x)
    p = os.path.join(tmp_path, "kseq.bigdl")
    m.saveModule(p, overWrite=True)
    from bigdl_amd.nn.module import Module
    m2 = Module.loadModule(p)
    assert torch.allclose(m2.forward(x), y, atol=1e-6)
    assert m2.getOutputShape() == [None, 3]


def test_first_layer_needs_input_shape():
    with pytest.raises(RuntimeError):
        K.Sequential().add(K.Dense(3))
