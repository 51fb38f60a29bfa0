"""VGG models (S/models/vgg/VggForCifar10.scala: VggForCifar10, Vgg_16, Vgg_19 and their graph variants)."""
from .. import nn

_CIFAR = [(3, 64, 0.3), (64, 64, None), "M", (64, 128, 0.4), (128, 128, None), "M", (128, 256, 0.4),
          (256, 256, 0.4), (256, 256, None), "M", (256, 512, 0.4), (512, 512, 0.4), (512, 512, None), "M",
          (512, 512, 0.4), (512, 512, 0.4), (512, 512, None), "M"]
_VGG16 = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]
_VGG19 = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]


def VggForCifar10(classNum, hasDropout=True):
    """Conv-BN(eps 1e-3)-ReLU stacks with dropout, ceil-mode 2x2 pooling, BN classifier, LogSoftMax."""
    m = nn.Sequential()
    for item in _CIFAR:
        if item == "M":
            m.add(nn.SpatialMaxPooling(2, 2, 2, 2).ceil())
            continue
        cin, cout, drop = item
        m.add(nn.SpatialConvolution(cin, cout, 3, 3, 1, 1, 1, 1))
        m.add(nn.SpatialBatchNormalization(cout, 1e-3))
        m.add(nn.ReLU(True))
        if hasDropout and drop is not None:
            m.add(nn.Dropout(drop))
    m.add(nn.View(512))
    cls = nn.Sequential()
    if hasDropout:
        cls.add(nn.Dropout(0.5))
    cls.add(nn.Linear(512, 512)).add(nn.BatchNormalization(512)).add(nn.ReLU(True))
    if hasDropout:
        cls.add(nn.Dropout(0.5))
    cls.add(nn.Linear(512, classNum)).add(nn.LogSoftMax())
    return m.add(cls)


def VggForCifar10Graph(classNum, hasDropout=True):
    x = inp = nn.Input()
    for item in _CIFAR:
        if item == "M":
            x = nn.SpatialMaxPooling(2, 2, 2, 2).ceil().inputs(x)
            continue
        cin, cout, drop = item
        x = nn.SpatialConvolution(cin, cout, 3, 3, 1, 1, 1, 1).inputs(x)
        x = nn.SpatialBatchNormalization(cout, 1e-3).inputs(x)
        x = nn.ReLU(True).inputs(x)
        if hasDropout and drop is not None:
            x = nn.Dropout(drop).inputs(x)
    x = nn.View(512).inputs(x)
    if hasDropout:
        x = nn.Dropout(0.5).inputs(x)
    x = nn.ReLU(True).inputs(nn.BatchNormalization(512).inputs(nn.Linear(512, 512).inputs(x)))
    if hasDropout:
        x = nn.Dropout(0.5).inputs(x)
    out = nn.LogSoftMax().inputs(nn.Linear(512, classNum).inputs(x))
    return nn.Graph(inp, out)


def _vgg(cfg, classNum, hasDropout):
    m = nn.Sequential()
    cin = 3
    for v in cfg:
        if v == "M":
            m.add(nn.SpatialMaxPooling(2, 2, 2, 2))
        else:
            m.add(nn.SpatialConvolution(cin, v, 3, 3, 1, 1, 1, 1)).add(nn.ReLU(True))
            cin = v
    m.add(nn.View(512 * 7 * 7))
    m.add(nn.Linear(512 * 7 * 7, 4096)).add(nn.Threshold(0, 1e-6))
    if hasDropout:
        m.add(nn.Dropout(0.5))
    m.add(nn.Linear(4096, 4096)).add(nn.Threshold(0, 1e-6))
    if hasDropout:
        m.add(nn.Dropout(0.5))
    return m.add(nn.Linear(4096, classNum)).add(nn.LogSoftMax())


def _vgg_graph(cfg, classNum, hasDropout):
    x = inp = nn.Input()
    cin = 3
    for v in cfg:
        if v == "M":
            x = nn.SpatialMaxPooling(2, 2, 2, 2).inputs(x)
        else:
            x = nn.ReLU(True).inputs(nn.SpatialConvolution(cin, v, 3, 3, 1, 1, 1, 1).inputs(x))
            cin = v
    x = nn.View(512 * 7 * 7).inputs(x)
    x = nn.Threshold(0, 1e-6).inputs(nn.Linear(512 * 7 * 7, 4096).inputs(x))
    if hasDropout:
        x = nn.Dropout(0.5).inputs(x)
    x = nn.Threshold(0, 1e-6).inputs(nn.Linear(4096, 4096).inputs(x))
    if hasDropout:
        x = nn.Dropout(0.5).inputs(x)
    return nn.Graph(inp, nn.LogSoftMax().inputs(nn.Linear(4096, classNum).inputs(x)))


def Vgg_16(classNum, hasDropout=True):
    return _vgg(_VGG16, classNum, hasDropout)


def Vgg_16Graph(classNum, hasDropout=True):
    return _vgg_graph(_VGG16, classNum, hasDropout)


def Vgg_19(classNum, hasDropout=True):
    return _vgg(_VGG19, classNum, hasDropout)


def Vgg_19Graph(classNum, hasDropout=True):
    return _vgg_graph(_VGG19, classNum, hasDropout)
