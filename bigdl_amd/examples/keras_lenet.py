"""Train LeNet with the Keras-style API (Sequential / compile / fit / evaluate / predict).

Reference: S/example/keras/Train.scala and S/example/keras/LeNet.scala (Keras-1.2.2-style LeNet:
Reshape -> Convolution2D(tanh) -> MaxPooling2D -> Convolution2D(tanh) -> MaxPooling2D -> Flatten -> Dense(tanh)
-> Dense(softmax), compiled with SGD + ClassNLL and Top-1 accuracy).
"""
import argparse
import tempfile

import torch


def build_lenet():
    from ..keras.layers import Convolution2D, Dense, Flatten, MaxPooling2D, Reshape
    from ..keras.engine import Sequential

    m = Sequential()
    m.add(Reshape([1, 28, 28], inputShape=[28, 28, 1]))
    m.add(Convolution2D(6, 5, 5, activation="tanh"))
    m.add(MaxPooling2D())
    m.add(Convolution2D(12, 5, 5, activation="tanh"))
    m.add(MaxPooling2D())
    m.add(Flatten())
    m.add(Dense(100, activation="tanh"))
    m.add(Dense(10, activation="softmax"))
    return m


def run(args):
    from ..optim.sgd import SGD
    from .lenet_local import load, write_synthetic_mnist

    with tempfile.TemporaryDirectory() as d:
        write_synthetic_mnist(d, n_train=384, n_test=96)
        train, test = load(d, True), load(d, False)
    xs = torch.stack([s.feature().reshape(28, 28, 1) for s in train])
    ys = torch.stack([s.label().reshape(1) for s in train])
    xt = torch.stack([s.feature().reshape(28, 28, 1) for s in test])
    yt = torch.stack([s.label().reshape(1) for s in test])
    torch.manual_seed(0)
    model = build_lenet()
    model.compile(optimizer=SGD(learningRate=args.learningRate, momentum=0.9, dampening=0.0),
                  loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    model.fit(xs, ys, batchSize=args.batchSize, nbEpoch=args.maxEpoch, validationData=(xt, yt))
    (res, _), = model.evaluate(xt, yt, batchSize=args.batchSize)
    probs = model.predict(xt[:8])
    return {"test_accuracy": float(res.result()[0]), "predict_shape": list(probs.shape)}


def build_parser():
    p = argparse.ArgumentParser(prog="keras")
    p.add_argument("--batchSize", type=int, default=32)
    p.add_argument("--maxEpoch", type=int, default=4)
    p.add_argument("--learningRate", type=float, default=0.05)
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
