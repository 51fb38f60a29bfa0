"""ResNet builders (reference S/models/resnet/ResNet.scala:75-449: depth table :227-240, ImageNet stem
:249-260, bottleneck / basic blocks, shortcut types A/B/C, ``graph`` variant, ``modelInit``).

ResNet-50 here is v1.5 exactly as the reference builds it: stride on the 3x3 conv of the bottleneck,
convs with bias and L2Regularizer(1e-4), SpatialBatchNormalization eps=1e-3 (last BN of each residual
branch zero-initialised), Linear(2048, classNum) with RandomNormal(0, 0.01) init.
"""
from .. import nn
from ..nn.init_methods import MsraFiller, Ones, RandomNormal, Zeros
from ..optim.regularizer import L2Regularizer


class ShortcutType:
    A = "A"
    B = "B"
    C = "C"


class DatasetType:
    ImageNet = "ImageNet"
    CIFAR10 = "CIFAR10"


def Convolution(nIn, nOut, kW, kH, sW=1, sH=1, pW=0, pH=0, nGroup=1, propagateBack=True, optnet=True,
                weightDecay=1e-4):
    cls = nn.SpatialShareConvolution if optnet else nn.SpatialConvolution
    conv = cls(nIn, nOut, kW, kH, sW, sH, pW, pH, nGroup, propagateBack,
               wRegularizer=L2Regularizer(weightDecay), bRegularizer=L2Regularizer(weightDecay))
    conv.setInitMethod(MsraFiller(False), Zeros())
    return conv


def Sbn(nOutput, eps=1e-3, momentum=0.1, affine=True):
    return nn.SpatialBatchNormalization(nOutput, eps, momentum, affine).setInitMethod(Ones(), Zeros())


class _Builder:
    def __init__(self, shortcutType, optnet):
        self.iChannels = 0
        self.shortcutType = shortcutType
        self.optnet = optnet

    def shortcut(self, nIn, nOut, stride):
        useConv = self.shortcutType == ShortcutType.C or (self.shortcutType == ShortcutType.B and nIn != nOut)
        if useConv:
            return nn.Sequential().add(Convolution(nIn, nOut, 1, 1, stride, stride, optnet=self.optnet)).add(Sbn(nOut))
        if nIn != nOut:
            return (nn.Sequential().add(nn.SpatialAveragePooling(1, 1, stride, stride))
                    .add(nn.Concat(2).add(nn.Identity()).add(nn.MulConstant(0.0))))
        return nn.Identity()

    def basicBlock(self, n, stride):
        nIn = self.iChannels
        self.iChannels = n
        s = nn.Sequential()
        s.add(Convolution(nIn, n, 3, 3, stride, stride, 1, 1, optnet=self.optnet))
        s.add(Sbn(n)).add(nn.ReLU(True))
        s.add(Convolution(n, n, 3, 3, 1, 1, 1, 1, optnet=self.optnet))
        s.add(Sbn(n))
        return (nn.Sequential().add(nn.ConcatTable().add(s).add(self.shortcut(nIn, n, stride)))
                .add(nn.CAddTable(True)).add(nn.ReLU(True)))

    def bottleneck(self, n, stride):
        nIn = self.iChannels
        self.iChannels = n * 4
        s = nn.Sequential()
        s.add(Convolution(nIn, n, 1, 1, 1, 1, 0, 0, optnet=self.optnet)).add(Sbn(n)).add(nn.ReLU(True))
        s.add(Convolution(n, n, 3, 3, stride, stride, 1, 1, optnet=self.optnet)).add(Sbn(n)).add(nn.ReLU(True))
        s.add(Convolution(n, n * 4, 1, 1, 1, 1, 0, 0, optnet=self.optnet)).add(Sbn(n * 4).setInitMethod(Zeros(), Zeros()))
        return (nn.Sequential().add(nn.ConcatTable().add(s).add(self.shortcut(nIn, n * 4, stride)))
                .add(nn.CAddTable(True)).add(nn.ReLU(True)))

    def layer(self, block, features, count, stride=1):
        s = nn.Sequential()
        for i in range(1, count + 1):
            s.add(block(features, stride if i == 1 else 1))
        return s


_CFG = {18: ((2, 2, 2, 2), 512, "basic"), 34: ((3, 4, 6, 3), 512, "basic"), 50: ((3, 4, 6, 3), 2048, "bottleneck"),
        101: ((3, 4, 23, 3), 2048, "bottleneck"), 152: ((3, 8, 36, 3), 2048, "bottleneck"),
        200: ((3, 24, 36, 3), 2048, "bottleneck")}


def ResNet(classNum, depth=18, shortcutType=ShortcutType.B, dataSet=DatasetType.CIFAR10, optnet=True):
    b = _Builder(shortcutType, optnet)
    model = nn.Sequential()
    if dataSet == DatasetType.ImageNet:
        if depth not in _CFG:
            raise ValueError(f"Invalid depth {depth}")
        loop, nFeatures, kind = _CFG[depth]
        block = b.bottleneck if kind == "bottleneck" else b.basicBlock
        b.iChannels = 64
        (model.add(Convolution(3, 64, 7, 7, 2, 2, 3, 3, optnet=optnet, propagateBack=False))
         .add(Sbn(64)).add(nn.ReLU(True)).add(nn.SpatialMaxPooling(3, 3, 2, 2, 1, 1))
         .add(b.layer(block, 64, loop[0])).add(b.layer(block, 128, loop[1], 2))
         .add(b.layer(block, 256, loop[2], 2)).add(b.layer(block, 512, loop[3], 2))
         .add(nn.SpatialAveragePooling(7, 7, 1, 1)).add(nn.View(nFeatures).setNumInputDims(3))
         .add(nn.Linear(nFeatures, classNum, True, L2Regularizer(1e-4), L2Regularizer(1e-4))
              .setInitMethod(RandomNormal(0.0, 0.01), Zeros())))
    elif dataSet == DatasetType.CIFAR10:
        assert (depth - 2) % 6 == 0, "depth should be one of 20, 32, 44, 56, 110, 1202"
        n = (depth - 2) // 6
        b.iChannels = 16
        model.add(Convolution(3, 16, 3, 3, 1, 1, 1, 1, optnet=optnet, propagateBack=False))
        model.add(nn.SpatialBatchNormalization(16)).add(nn.ReLU(True))
        model.add(b.layer(b.basicBlock, 16, n)).add(b.layer(b.basicBlock, 32, n, 2)).add(b.layer(b.basicBlock, 64, n, 2))
        model.add(nn.SpatialAveragePooling(8, 8, 1, 1)).add(nn.View(64).setNumInputDims(3)).add(nn.Linear(64, 10))
    else:
        raise ValueError(f"Invalid dataset {dataSet}")
    return model


def ResNetGraph(classNum, depth=18, shortcutType=ShortcutType.B, dataSet=DatasetType.CIFAR10, optnet=True):
    """Graph (DAG) variant of the same network (reference ResNet.graph)."""
    st = {"c": 0}

    def shortcut(nIn, nOut, stride, inp):
        useConv = shortcutType == ShortcutType.C or (shortcutType == ShortcutType.B and nIn != nOut)
        if useConv:
            c = Convolution(nIn, nOut, 1, 1, stride, stride, optnet=optnet).inputs(inp)
            return Sbn(nOut).inputs(c)
        if nIn != nOut:
            p = nn.SpatialAveragePooling(1, 1, stride, stride).inputs(inp)
            m = nn.MulConstant(0.0).inputs(p)
            return nn.JoinTable(2, 0).inputs(p, m)
        return inp

    def bottleneck(n, stride, inp):
        nIn = st["c"]
        st["c"] = n * 4
        c1 = Convolution(nIn, n, 1, 1, 1, 1, 0, 0, optnet=optnet).inputs(inp)
        r1 = nn.ReLU(True).inputs(Sbn(n).inputs(c1))
        c2 = Convolution(n, n, 3, 3, stride, stride, 1, 1, optnet=optnet).inputs(r1)
        r2 = nn.ReLU(True).inputs(Sbn(n).inputs(c2))
        c3 = Convolution(n, n * 4, 1, 1, 1, 1, 0, 0, optnet=optnet).inputs(r2)
        b3 = Sbn(n * 4).setInitMethod(Zeros(), Zeros()).inputs(c3)
        add = nn.CAddTable(True).inputs(b3, shortcut(nIn, n * 4, stride, inp))
        return nn.ReLU(True).inputs(add)

    def basic(n, stride, inp):
        nIn = st["c"]
        st["c"] = n
        c1 = Convolution(nIn, n, 3, 3, stride, stride, 1, 1, optnet=optnet).inputs(inp)
        r1 = nn.ReLU(True).inputs(Sbn(n).inputs(c1))
        c2 = Convolution(n, n, 3, 3, 1, 1, 1, 1, optnet=optnet).inputs(r1)
        b2 = Sbn(n).inputs(c2)
        add = nn.CAddTable(True).inputs(b2, shortcut(nIn, n, stride, inp))
        return nn.ReLU(True).inputs(add)

    def layer(block, features, count, stride, inp):
        x = inp
        for i in range(1, count + 1):
            x = block(features, stride if i == 1 else 1, x)
        return x

    inp = nn.Input()
    if dataSet == DatasetType.ImageNet:
        loop, nFeatures, kind = _CFG[depth]
        block = bottleneck if kind == "bottleneck" else basic
        st["c"] = 64
        x = Convolution(3, 64, 7, 7, 2, 2, 3, 3, optnet=optnet, propagateBack=False).inputs(inp)
        x = nn.SpatialMaxPooling(3, 3, 2, 2, 1, 1).inputs(nn.ReLU(True).inputs(Sbn(64).inputs(x)))
        x = layer(block, 64, loop[0], 1, x)
        x = layer(block, 128, loop[1], 2, x)
        x = layer(block, 256, loop[2], 2, x)
        x = layer(block, 512, loop[3], 2, x)
        x = nn.View(nFeatures).setNumInputDims(3).inputs(nn.SpatialAveragePooling(7, 7, 1, 1).inputs(x))
        out = (nn.Linear(nFeatures, classNum, True, L2Regularizer(1e-4), L2Regularizer(1e-4))
               .setInitMethod(RandomNormal(0.0, 0.01), Zeros()).inputs(x))
    else:
        n = (depth - 2) // 6
        st["c"] = 16
        x = Convolution(3, 16, 3, 3, 1, 1, 1, 1, optnet=optnet, propagateBack=False).inputs(inp)
        x = nn.ReLU(True).inputs(nn.SpatialBatchNormalization(16).inputs(x))
        x = layer(basic, 16, n, 1, x)
        x = layer(basic, 32, n, 2, x)
        x = layer(basic, 64, n, 2, x)
        x = nn.View(64).setNumInputDims(3).inputs(nn.SpatialAveragePooling(8, 8, 1, 1).inputs(x))
        out = nn.Linear(64, 10).inputs(x)
    return nn.Graph([inp], [out])


def modelInit(model):
    """Reference ResNet.modelInit: conv weights ~ N(0, sqrt(2 / (k*k*nOut))), zero bias; BN (1, 0)."""
    import math

    for m in model.flattened_layers():
        if isinstance(m, nn.SpatialConvolution):
            n = m.kernelW * m.kernelW * m.nOutputPlane
            RandomNormal(0.0, math.sqrt(2.0 / n)).init(m.weight)
            if m.bias is not None:
                m.bias.zero_()
        elif isinstance(m, nn.BatchNormalization) and m.affine:
            m.weight.fill_(1.0)
            m.bias.zero_()
        elif isinstance(m, nn.Linear) and m.bias is not None:
            m.bias.zero_()
    return model


def ResNet50(classNum=1000):
    return ResNet(classNum, 50, ShortcutType.B, DatasetType.ImageNet)
