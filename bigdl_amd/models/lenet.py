"""LeNet-5 (reference S/models/lenet/LeNet5.scala:28-60): Reshape(1,28,28) -> conv(1->6,5x5) -> Tanh ->
maxpool 2x2 -> Tanh -> conv(6->12,5x5) -> maxpool 2x2 -> Reshape(12*4*4) -> Linear(192->100) -> Tanh ->
Linear(100->classNum) -> LogSoftMax."""
from .. import nn


def LeNet5(classNum=10):
    model = nn.Sequential()
    (model.add(nn.Reshape([1, 28, 28]))
     .add(nn.SpatialConvolution(1, 6, 5, 5).setName("conv1_5x5"))
     .add(nn.Tanh())
     .add(nn.SpatialMaxPooling(2, 2, 2, 2))
     .add(nn.Tanh())
     .add(nn.SpatialConvolution(6, 12, 5, 5).setName("conv2_5x5"))
     .add(nn.SpatialMaxPooling(2, 2, 2, 2))
     .add(nn.Reshape([12 * 4 * 4]))
     .add(nn.Linear(12 * 4 * 4, 100).setName("fc1"))
     .add(nn.Tanh())
     .add(nn.Linear(100, classNum).setName("fc2"))
     .add(nn.LogSoftMax()))
    return model


def LeNet5Graph(classNum=10):
    inp = nn.Reshape([1, 28, 28]).inputs()
    c1 = nn.SpatialConvolution(1, 6, 5, 5).setName("conv1_5x5").inputs(inp)
    t1 = nn.Tanh().inputs(c1)
    p1 = nn.SpatialMaxPooling(2, 2, 2, 2).inputs(t1)
    t2 = nn.Tanh().inputs(p1)
    c2 = nn.SpatialConvolution(6, 12, 5, 5).setName("conv2_5x5").inputs(t2)
    p2 = nn.SpatialMaxPooling(2, 2, 2, 2).inputs(c2)
    r2 = nn.Reshape([12 * 4 * 4]).inputs(p2)
    f1 = nn.Linear(12 * 4 * 4, 100).setName("fc1").inputs(r2)
    t3 = nn.Tanh().inputs(f1)
    f2 = nn.Linear(100, classNum).setName("fc2").inputs(t3)
    out = nn.LogSoftMax().inputs(f2)
    return nn.Graph([inp], [out])
