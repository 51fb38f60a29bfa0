"""GoogLeNet / BN-Inception (S/models/inception/Inception_v1.scala:26-352, Inception_v2.scala): layer builders
in module form (Concat of branch Sequentials) and graph form (JoinTable of branch nodes), with and without the
auxiliary classifiers. Channel concat runs as zero-copy slices of one NHWC output on the GPU engine."""
from .. import nn


def _conv(cin, cout, k, s=1, p=0, name=None, xavier=True, bias_const=0.1, withBias=True):
    c = nn.SpatialConvolution(cin, cout, k, k, s, s, p, p, withBias=withBias)
    if xavier:
        c.setInitMethod(nn.Xavier(), nn.ConstInitMethod(bias_const))
    return c.setName(name) if name else c


def Inception_Layer_v1(inputSize, config, namePrefix=""):
    """config: ((c1x1,), (c3x3_reduce, c3x3), (c5x5_reduce, c5x5), (pool_proj,))."""
    (c1,), (r3, c3), (r5, c5), (pp,) = config
    p = namePrefix
    concat = nn.Concat(2)
    concat.add(nn.Sequential().add(_conv(inputSize, c1, 1, name=p + "1x1")).add(nn.ReLU(True).setName(p + "relu_1x1")))
    concat.add(nn.Sequential().add(_conv(inputSize, r3, 1, name=p + "3x3_reduce"))
               .add(nn.ReLU(True).setName(p + "relu_3x3_reduce"))
               .add(_conv(r3, c3, 3, 1, 1, name=p + "3x3")).add(nn.ReLU(True).setName(p + "relu_3x3")))
    concat.add(nn.Sequential().add(_conv(inputSize, r5, 1, name=p + "5x5_reduce"))
               .add(nn.ReLU(True).setName(p + "relu_5x5_reduce"))
               .add(_conv(r5, c5, 5, 1, 2, name=p + "5x5")).add(nn.ReLU(True).setName(p + "relu_5x5")))
    concat.add(nn.Sequential().add(nn.SpatialMaxPooling(3, 3, 1, 1, 1, 1).ceil().setName(p + "pool"))
               .add(_conv(inputSize, pp, 1, name=p + "pool_proj")).add(nn.ReLU(True).setName(p + "relu_pool_proj")))
    return concat.setName(p + "output")


def Inception_Layer_v1_node(x, inputSize, config, namePrefix):
    (c1,), (r3, c3), (r5, c5), (pp,) = config
    p = namePrefix
    b1 = nn.ReLU(True).setName(p + "relu_1x1").inputs(_conv(inputSize, c1, 1, name=p + "1x1").inputs(x))
    b3 = nn.ReLU(True).setName(p + "relu_3x3_reduce").inputs(_conv(inputSize, r3, 1, name=p + "3x3_reduce").inputs(x))
    b3 = nn.ReLU(True).setName(p + "relu_3x3").inputs(_conv(r3, c3, 3, 1, 1, name=p + "3x3").inputs(b3))
    b5 = nn.ReLU(True).setName(p + "relu_5x5_reduce").inputs(_conv(inputSize, r5, 1, name=p + "5x5_reduce").inputs(x))
    b5 = nn.ReLU(True).setName(p + "relu_5x5").inputs(_conv(r5, c5, 5, 1, 2, name=p + "5x5").inputs(b5))
    bp = nn.SpatialMaxPooling(3, 3, 1, 1, 1, 1).ceil().setName(p + "pool").inputs(x)
    bp = nn.ReLU(True).setName(p + "relu_pool_proj").inputs(_conv(inputSize, pp, 1, name=p + "pool_proj").inputs(bp))
    return nn.JoinTable(2, 0).inputs(b1, b3, b5, bp)


_V1 = {
    "3a": (192, ((64,), (96, 128), (16, 32), (32,))), "3b": (256, ((128,), (128, 192), (32, 96), (64,))),
    "4a": (480, ((192,), (96, 208), (16, 48), (64,))), "4b": (512, ((160,), (112, 224), (24, 64), (64,))),
    "4c": (512, ((128,), (128, 256), (24, 64), (64,))), "4d": (512, ((112,), (144, 288), (32, 64), (64,))),
    "4e": (528, ((256,), (160, 320), (32, 128), (128,))), "5a": (832, ((256,), (160, 320), (32, 128), (128,))),
    "5b": (832, ((384,), (192, 384), (48, 128), (128,))),
}


def _v1_stem(seq):
    seq.add(_conv(3, 64, 7, 2, 3, name="conv1/7x7_s2", withBias=True))
    seq.add(nn.ReLU(True).setName("conv1/relu_7x7"))
    seq.add(nn.SpatialMaxPooling(3, 3, 2, 2).ceil().setName("pool1/3x3_s2"))
    seq.add(nn.SpatialCrossMapLRN(5, 0.0001, 0.75).setName("pool1/norm1"))
    seq.add(_conv(64, 64, 1, name="conv2/3x3_reduce")).add(nn.ReLU(True).setName("conv2/relu_3x3_reduce"))
    seq.add(_conv(64, 192, 3, 1, 1, name="conv2/3x3")).add(nn.ReLU(True).setName("conv2/relu_3x3"))
    seq.add(nn.SpatialCrossMapLRN(5, 0.0001, 0.75).setName("conv2/norm2"))
    seq.add(nn.SpatialMaxPooling(3, 3, 2, 2).ceil().setName("pool2/3x3_s2"))
    return seq


def _v1(seq, key):
    cin, cfg = _V1[key]
    return seq.add(Inception_Layer_v1(cin, cfg, f"inception_{key}/"))


def _head_v1(seq, classNum, hasDropout):
    seq.add(nn.SpatialAveragePooling(7, 7, 1, 1).setName("pool5/7x7_s1"))
    if hasDropout:
        seq.add(nn.Dropout(0.4).setName("pool5/drop_7x7_s1"))
    seq.add(nn.View(1024).setNumInputDims(3))
    seq.add(nn.Linear(1024, classNum).setInitMethod(nn.Xavier(), nn.Zeros()).setName("loss3/classifier"))
    return seq.add(nn.LogSoftMax().setName("loss3/loss3"))


def Inception_v1_NoAuxClassifier(classNum, hasDropout=True):
    m = _v1_stem(nn.Sequential())
    _v1(m, "3a"), _v1(m, "3b")
    m.add(nn.SpatialMaxPooling(3, 3, 2, 2).ceil().setName("pool3/3x3_s2"))
    for k in ("4a", "4b", "4c", "4d", "4e"):
        _v1(m, k)
    m.add(nn.SpatialMaxPooling(3, 3, 2, 2).ceil().setName("pool4/3x3_s2"))
    _v1(m, "5a"), _v1(m, "5b")
    return _head_v1(m, classNum, hasDropout)


def Inception_v1_NoAuxClassifierGraph(classNum, hasDropout=True):
    inp = nn.Input()
    stem = _v1_stem(nn.Sequential())
    x = stem.inputs(inp)
    for k in ("3a", "3b"):
        x = Inception_Layer_v1_node(x, *_V1[k], f"inception_{k}/")
    x = nn.SpatialMaxPooling(3, 3, 2, 2).ceil().setName("pool3/3x3_s2").inputs(x)
    for k in ("4a", "4b", "4c", "4d", "4e"):
        x = Inception_Layer_v1_node(x, *_V1[k], f"inception_{k}/")
    x = nn.SpatialMaxPooling(3, 3, 2, 2).ceil().setName("pool4/3x3_s2").inputs(x)
    for k in ("5a", "5b"):
        x = Inception_Layer_v1_node(x, *_V1[k], f"inception_{k}/")
    out = _head_v1(nn.Sequential(), classNum, hasDropout).inputs(x)
    return nn.Graph(inp, out)


def _aux_v1(prefix, cin, classNum, hasDropout, ceil):
    s = nn.Sequential()
    pool = nn.SpatialAveragePooling(5, 5, 3, 3)
    if ceil:
        pool.ceil()
    s.add(pool.setName(f"{prefix}/ave_pool"))
    s.add(nn.SpatialConvolution(cin, 128, 1, 1, 1, 1).setName(f"{prefix}/conv"))
    s.add(nn.ReLU(True).setName(f"{prefix}/relu_conv")).add(nn.View(128 * 4 * 4).setNumInputDims(3))
    s.add(nn.Linear(128 * 4 * 4, 1024).setName(f"{prefix}/fc")).add(nn.ReLU(True).setName(f"{prefix}/relu_fc"))
    if hasDropout:
        s.add(nn.Dropout(0.7).setName(f"{prefix}/drop_fc"))
    s.add(nn.Linear(1024, classNum).setName(f"{prefix}/classifier"))
    return s.add(nn.LogSoftMax().setName(f"{prefix}/loss"))


def Inception_v1(classNum, hasDropout=True):
    """GoogLeNet with both auxiliary classifiers; output = concat(loss3, loss2, loss1) along dim 2."""
    f1 = _v1_stem(nn.Sequential())
    _v1(f1, "3a"), _v1(f1, "3b")
    f1.add(nn.SpatialMaxPooling(3, 3, 2, 2).ceil().setName("pool3/3x3_s2"))
    _v1(f1, "4a")
    out1 = _aux_v1("loss1", 512, classNum, hasDropout, True)
    f2 = nn.Sequential()
    for k in ("4b", "4c", "4d"):
        _v1(f2, k)
    out2 = _aux_v1("loss2", 528, classNum, hasDropout, False)
    out3 = nn.Sequential()
    _v1(out3, "4e")
    out3.add(nn.SpatialMaxPooling(3, 3, 2, 2).ceil().setName("pool4/3x3_s2"))
    _v1(out3, "5a"), _v1(out3, "5b")
    _head_v1(out3, classNum, hasDropout)
    split2 = nn.Concat(2).setName("split2").add(out3).add(out2)
    main = nn.Sequential().add(f2).add(split2)
    split1 = nn.Concat(2).setName("split1").add(main).add(out1)
    return nn.Sequential().add(f1).add(split1)


# ---------------------------------------------------------------------------------------------- v2
def _cbr(seq, cin, cout, k, s, p, name):
    seq.add(nn.SpatialConvolution(cin, cout, k, k, s, s, p, p).setName(name))
    seq.add(nn.SpatialBatchNormalization(cout, 1e-3).setName(name + "/bn"))
    return seq.add(nn.ReLU(True).setName(name + "/bn/sc/relu"))


def Inception_Layer_v2(inputSize, config, namePrefix):
    """config: ((c1x1,), (r3, c3), (rd, cd), (pool_type, pool_proj)); pool ("max", 0) = stride-2 reduction."""
    (c1,), (r3, c3), (rd, cd), (ptype, pp) = config
    p = namePrefix
    reduce_ = ptype == "max" and pp == 0
    st = 2 if reduce_ else 1
    concat = nn.Concat(2)
    if c1 != 0:
        concat.add(_cbr(nn.Sequential(), inputSize, c1, 1, 1, 0, p + "1x1"))
    b3 = _cbr(nn.Sequential(), inputSize, r3, 1, 1, 0, p + "3x3_reduce")
    concat.add(_cbr(b3, r3, c3, 3, st, 1, p + "3x3"))
    bd = _cbr(nn.Sequential(), inputSize, rd, 1, 1, 0, p + "double3x3_reduce")
    _cbr(bd, rd, cd, 3, 1, 1, p + "double3x3a")
    concat.add(_cbr(bd, cd, cd, 3, st, 1, p + "double3x3b"))
    pool = nn.Sequential()
    if ptype == "max":
        pool.add((nn.SpatialMaxPooling(3, 3, 1, 1, 1, 1) if pp != 0 else nn.SpatialMaxPooling(3, 3, 2, 2))
                 .ceil().setName(p + "pool"))
    elif ptype == "avg":
        pool.add(nn.SpatialAveragePooling(3, 3, 1, 1, 1, 1).ceil().setName(p + "pool"))
    else:
        raise ValueError(ptype)
    if pp != 0:
        _cbr(pool, inputSize, pp, 1, 1, 0, p + "pool_proj")
    concat.add(pool)
    return concat.setName(p + "output")


_V2 = [("3a", 192, ((64,), (64, 64), (64, 96), ("avg", 32))), ("3b", 256, ((64,), (64, 96), (64, 96), ("avg", 64))),
       ("3c", 320, ((0,), (128, 160), (64, 96), ("max", 0))),
       ("4a", 576, ((224,), (64, 96), (96, 128), ("avg", 128))),
       ("4b", 576, ((192,), (96, 128), (96, 128), ("avg", 128))),
       ("4c", 576, ((160,), (128, 160), (128, 160), ("avg", 96))),
       ("4d", 576, ((96,), (128, 192), (160, 192), ("avg", 96))),
       ("4e", 576, ((0,), (128, 192), (192, 256), ("max", 0))),
       ("5a", 1024, ((352,), (192, 320), (160, 224), ("avg", 128))),
       ("5b", 1024, ((352,), (192, 320), (192, 224), ("max", 128)))]


def _v2_stem(seq):
    _cbr(seq, 3, 64, 7, 2, 3, "conv1/7x7_s2")
    seq.add(nn.SpatialMaxPooling(3, 3, 2, 2).ceil().setName("pool1/3x3_s2"))
    _cbr(seq, 64, 64, 1, 1, 0, "conv2/3x3_reduce")
    _cbr(seq, 64, 192, 3, 1, 1, "conv2/3x3")
    return seq.add(nn.SpatialMaxPooling(3, 3, 2, 2).ceil().setName("pool2/3x3_s2"))


def _v2_layers(seq, keys):
    for k, cin, cfg in _V2:
        if k in keys:
            seq.add(Inception_Layer_v2(cin, cfg, f"inception_{k}/"))
    return seq


def _v2_head(seq, classNum):
    seq.add(nn.SpatialAveragePooling(7, 7, 1, 1).ceil().setName("pool5/7x7_s1"))
    seq.add(nn.View(1024).setNumInputDims(3))
    seq.add(nn.Linear(1024, classNum).setName("loss3/classifier"))
    return seq.add(nn.LogSoftMax().setName("loss3/loss"))


def Inception_v2_NoAuxClassifier(classNum):
    m = _v2_stem(nn.Sequential())
    _v2_layers(m, [k for k, _, _ in _V2])
    return _v2_head(m, classNum)


def _aux_v2(prefix, pool_name, cin, side, classNum):
    s = nn.Sequential().add(nn.SpatialAveragePooling(5, 5, 3, 3).ceil().setName(pool_name))
    _cbr(s, cin, 128, 1, 1, 0, f"{prefix}/conv")
    s.add(nn.View(128 * side * side).setNumInputDims(3))
    s.add(nn.Linear(128 * side * side, 1024).setName(f"{prefix}/fc")).add(nn.ReLU(True).setName(f"{prefix}/fc/bn/sc/relu"))
    s.add(nn.Linear(1024, classNum).setName(f"{prefix}/classifier"))
    return s.add(nn.LogSoftMax().setName(f"{prefix}/loss"))


def Inception_v2(classNum):
    f1 = _v2_layers(_v2_stem(nn.Sequential()), ["3a", "3b", "3c"])
    out1 = _aux_v2("loss1", "pool3/5x5_s3", 576, 4, classNum)
    f2 = _v2_layers(nn.Sequential(), ["4a", "4b", "4c", "4d", "4e"])
    out2 = _aux_v2("loss2", "pool4/5x5_s3", 1024, 2, classNum)
    out3 = _v2_head(_v2_layers(nn.Sequential(), ["5a", "5b"]), classNum)
    split2 = nn.Concat(2).add(out3).add(out2)
    split1 = nn.Concat(2).add(nn.Sequential().add(f2).add(split2)).add(out1)
    return nn.Sequential().add(f1).add(split1)


# ---------------------------------------------------------------------------------------------- Inception-v3
# Inception-v3 (Szegedy et al. 2015, "Rethinking the Inception Architecture"), the model of BASELINE config 4
# (the reference ships v1 / v2 builders and loads v3 through its Caffe / TF importers). Every convolution is
# conv (no bias) + BatchNorm(eps=1e-3) + ReLU; factorised 1x7 / 7x1 and 1x3 / 3x1 kernels run on the same
# implicit-GEMM conv kernels as square ones. Input 3 x 299 x 299.
def _cbr3(cin, cout, kh, kw, sh=1, sw=1, ph=0, pw=0, name=""):
    s = nn.Sequential()
    s.add(nn.SpatialConvolution(cin, cout, kw, kh, sw, sh, pw, ph, withBias=False)
          .setInitMethod(nn.Xavier(), nn.Zeros()).setName(name + "conv"))
    s.add(nn.SpatialBatchNormalization(cout, 1e-3).setName(name + "bn"))
    s.add(nn.ReLU(True).setName(name + "relu"))
    return s


def _branch(*mods):
    s = nn.Sequential()
    for m in mods:
        s.add(m)
    return s


def _inception_a(cin, pool_features, p):
    c = nn.Concat(2)
    c.add(_cbr3(cin, 64, 1, 1, name=p + "b1x1_"))
    c.add(_branch(_cbr3(cin, 48, 1, 1, name=p + "b5x5_1_"), _cbr3(48, 64, 5, 5, ph=2, pw=2, name=p + "b5x5_2_")))
    c.add(_branch(_cbr3(cin, 64, 1, 1, name=p + "b3x3dbl_1_"), _cbr3(64, 96, 3, 3, ph=1, pw=1, name=p + "b3x3dbl_2_"),
                  _cbr3(96, 96, 3, 3, ph=1, pw=1, name=p + "b3x3dbl_3_")))
    c.add(_branch(nn.SpatialAveragePooling(3, 3, 1, 1, 1, 1).setName(p + "pool"),
                  _cbr3(cin, pool_features, 1, 1, name=p + "bpool_")))
    return c.setName(p + "concat")


def _inception_b(cin, p):
    c = nn.Concat(2)
    c.add(_cbr3(cin, 384, 3, 3, 2, 2, name=p + "b3x3_"))
    c.add(_branch(_cbr3(cin, 64, 1, 1, name=p + "b3x3dbl_1_"), _cbr3(64, 96, 3, 3, ph=1, pw=1, name=p + "b3x3dbl_2_"),
                  _cbr3(96, 96, 3, 3, 2, 2, name=p + "b3x3dbl_3_")))
    c.add(nn.SpatialMaxPooling(3, 3, 2, 2).setName(p + "pool"))
    return c.setName(p + "concat")


def _inception_c(cin, c7, p):
    c = nn.Concat(2)
    c.add(_cbr3(cin, 192, 1, 1, name=p + "b1x1_"))
    c.add(_branch(_cbr3(cin, c7, 1, 1, name=p + "b7x7_1_"), _cbr3(c7, c7, 1, 7, pw=3, name=p + "b7x7_2_"),
                  _cbr3(c7, 192, 7, 1, ph=3, name=p + "b7x7_3_")))
    c.add(_branch(_cbr3(cin, c7, 1, 1, name=p + "b7x7dbl_1_"), _cbr3(c7, c7, 7, 1, ph=3, name=p + "b7x7dbl_2_"),
                  _cbr3(c7, c7, 1, 7, pw=3, name=p + "b7x7dbl_3_"), _cbr3(c7, c7, 7, 1, ph=3, name=p + "b7x7dbl_4_"),
                  _cbr3(c7, 192, 1, 7, pw=3, name=p + "b7x7dbl_5_")))
    c.add(_branch(nn.SpatialAveragePooling(3, 3, 1, 1, 1, 1).setName(p + "pool"),
                  _cbr3(cin, 192, 1, 1, name=p + "bpool_")))
    return c.setName(p + "concat")


def _inception_d(cin, p):
    c = nn.Concat(2)
    c.add(_branch(_cbr3(cin, 192, 1, 1, name=p + "b3x3_1_"), _cbr3(192, 320, 3, 3, 2, 2, name=p + "b3x3_2_")))
    c.add(_branch(_cbr3(cin, 192, 1, 1, name=p + "b7x7x3_1_"), _cbr3(192, 192, 1, 7, pw=3, name=p + "b7x7x3_2_"),
                  _cbr3(192, 192, 7, 1, ph=3, name=p + "b7x7x3_3_"), _cbr3(192, 192, 3, 3, 2, 2, name=p + "b7x7x3_4_")))
    c.add(nn.SpatialMaxPooling(3, 3, 2, 2).setName(p + "pool"))
    return c.setName(p + "concat")


def _inception_e(cin, p):
    c = nn.Concat(2)
    c.add(_cbr3(cin, 320, 1, 1, name=p + "b1x1_"))
    b3 = nn.Sequential().add(_cbr3(cin, 384, 1, 1, name=p + "b3x3_1_"))
    b3.add(nn.Concat(2).add(_cbr3(384, 384, 1, 3, pw=1, name=p + "b3x3_2a_"))
           .add(_cbr3(384, 384, 3, 1, ph=1, name=p + "b3x3_2b_")))
    c.add(b3)
    bd = nn.Sequential().add(_cbr3(cin, 448, 1, 1, name=p + "b3x3dbl_1_"))
    bd.add(_cbr3(448, 384, 3, 3, ph=1, pw=1, name=p + "b3x3dbl_2_"))
    bd.add(nn.Concat(2).add(_cbr3(384, 384, 1, 3, pw=1, name=p + "b3x3dbl_3a_"))
           .add(_cbr3(384, 384, 3, 1, ph=1, name=p + "b3x3dbl_3b_")))
    c.add(bd)
    c.add(_branch(nn.SpatialAveragePooling(3, 3, 1, 1, 1, 1).setName(p + "pool"),
                  _cbr3(cin, 192, 1, 1, name=p + "bpool_")))
    return c.setName(p + "concat")


def Inception_v3(classNum=1000, hasDropout=True):
    """Inception-v3 for 299 x 299 inputs (no auxiliary classifier). 2048-channel 8 x 8 final map."""
    m = nn.Sequential()
    m.add(_cbr3(3, 32, 3, 3, 2, 2, name="Conv2d_1a_3x3_"))
    m.add(_cbr3(32, 32, 3, 3, name="Conv2d_2a_3x3_"))
    m.add(_cbr3(32, 64, 3, 3, ph=1, pw=1, name="Conv2d_2b_3x3_"))
    m.add(nn.SpatialMaxPooling(3, 3, 2, 2).setName("MaxPool_3a_3x3"))
    m.add(_cbr3(64, 80, 1, 1, name="Conv2d_3b_1x1_"))
    m.add(_cbr3(80, 192, 3, 3, name="Conv2d_4a_3x3_"))
    m.add(nn.SpatialMaxPooling(3, 3, 2, 2).setName("MaxPool_5a_3x3"))
    m.add(_inception_a(192, 32, "Mixed_5b_"))
    m.add(_inception_a(256, 64, "Mixed_5c_"))
    m.add(_inception_a(288, 64, "Mixed_5d_"))
    m.add(_inception_b(288, "Mixed_6a_"))
    m.add(_inception_c(768, 128, "Mixed_6b_"))
    m.add(_inception_c(768, 160, "Mixed_6c_"))
    m.add(_inception_c(768, 160, "Mixed_6d_"))
    m.add(_inception_c(768, 192, "Mixed_6e_"))
    m.add(_inception_d(768, "Mixed_7a_"))
    m.add(_inception_e(1280, "Mixed_7b_"))
    m.add(_inception_e(2048, "Mixed_7c_"))
    m.add(nn.SpatialAveragePooling(8, 8, 1, 1).setName("AvgPool_1a_8x8"))
    if hasDropout:
        m.add(nn.Dropout(0.2).setName("Dropout_1b"))
    m.add(nn.View(2048).setNumInputDims(3))
    m.add(nn.Linear(2048, classNum).setName("Logits"))
    m.add(nn.LogSoftMax().setName("Predictions"))
    return m
