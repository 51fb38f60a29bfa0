"""MNIST autoencoder (S/models/autoencoder/Autoencoder.scala)."""
from .. import nn

ROW_N = COL_N = 28
FEATURE_SIZE = ROW_N * COL_N


def Autoencoder(classNum):
    return nn.Sequential().add(nn.Reshape([FEATURE_SIZE])).add(nn.Linear(FEATURE_SIZE, classNum)).add(nn.ReLU()) \
        .add(nn.Linear(classNum, FEATURE_SIZE)).add(nn.Sigmoid())


def AutoencoderGraph(classNum):
    inp = nn.Input()
    x = nn.Reshape([FEATURE_SIZE]).inputs(inp)
    x = nn.ReLU().inputs(nn.Linear(FEATURE_SIZE, classNum).inputs(x))
    return nn.Graph(inp, nn.Sigmoid().inputs(nn.Linear(classNum, FEATURE_SIZE).inputs(x)))
