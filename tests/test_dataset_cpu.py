"""Data pipeline on the CPU: MNIST/CIFAR readers, BGR/grey image transformers, multi-threaded batching,
vision ImageFeature augmentations, text pipeline (reference T/dataset/**, T/transform/vision/image/**)."""
import io

import numpy as np
import pytest
import torch

from bigdl_amd import dataset as D
from bigdl_amd.dataset.image import encode_bgr_record
from bigdl_amd.dataset.mnist_cifar import load_cifar_file, write_mnist
from bigdl_amd.transform.vision import image as V
from bigdl_amd.utils.random_generator import RNG


def test_mnist_reader_and_grey_pipeline(tmp_path):
    imgs = np.random.RandomState(0).randint(0, 256, (10, 28, 28)).astype(np.uint8)
    labels = np.arange(10) % 10
    write_mnist(tmp_path / "x", tmp_path / "y", imgs, labels)
    recs = D.load_mnist(str(tmp_path / "x"), str(tmp_path / "y"))
    assert len(recs) == 10 and recs[3].label == 4.0
    pipe = D.BytesToGreyImg(28, 28) >> D.GreyImgNormalizer(0.13, 0.31) >> D.GreyImgCropper(24, 24) >> \
        D.GreyImgToBatch(4)
    batches = list(pipe(iter(recs)))
    assert [b.size() for b in batches] == [4, 4, 2]
    assert batches[0].getInput().shape == (4, 24, 24)
    first = torch.tensor(imgs[0], dtype=torch.float32) / 255.0
    assert abs(float(((first - 0.13) / 0.31).max()) - float(batches[0].getInput()[0].max())) < 0.6


def test_cifar_reader_layout(tmp_path):
    rec = np.zeros((2, 3073), dtype=np.uint8)
    rec[0, 0], rec[1, 0] = 3, 7
    rec[0, 1:1025] = 200            # R plane
    rec[0, 1025:2049] = 100         # G plane
    rec[0, 2049:] = 50              # B plane
    p = tmp_path / "b.bin"
    p.write_bytes(rec.tobytes())
    recs = load_cifar_file(str(p), [])
    assert recs[0].label == 4.0 and recs[1].label == 8.0
    img = D.BGRImage().copy(recs[0].data)
    assert img.content.shape == (32, 32, 3)
    assert img.content[0, 0].tolist() == [50.0, 100.0, 200.0]        # B, G, R
    assert img.toTensor(True)[:, 0, 0].tolist() == [200.0, 100.0, 50.0]


def test_bgr_transformers_and_mt_batching():
    RNG.setSeed(1)
    recs = [D.ByteRecord(encode_bgr_record(torch.randint(0, 256, (36, 36, 3), dtype=torch.uint8)), i % 3 + 1)
            for i in range(10)]
    norm = D.BGRImgNormalizer(0.5, 0.5, 0.5, 0.25, 0.25, 0.25)
    tf = D.BytesToBGRImg() >> D.BGRImgRdmCropper(32, 32, 4) >> D.HFlip(0.5) >> norm >> D.ColorJitter() >> \
        D.Lighting()
    mt = D.MTLabeledBGRImgToBatch(32, 32, 4, tf, threads=3)
    batches = list(mt(iter(recs)))
    assert sum(b.size() for b in batches) == 10
    assert batches[0].getInput().shape == (4, 3, 32, 32)
    labels = sorted(float(v) for b in batches for v in b.getTarget())
    assert labels == sorted(float(i % 3 + 1) for i in range(10))
    single = list((D.BytesToBGRImg() >> D.BGRImgCropper(30, 30, D.CropCenter) >> D.BGRImgToBatch(5))(iter(recs)))
    assert single[0].getInput().shape == (5, 3, 30, 30)


def test_local_image_files_and_reader(tmp_path):
    from PIL import Image

    for c in ("cat", "dog"):
        (tmp_path / c).mkdir()
        for i in range(2):
            Image.fromarray(np.full((20, 30, 3), 40 * i, dtype=np.uint8)).save(tmp_path / c / f"{i}.png")
    paths = D.LocalImageFiles.readPaths(str(tmp_path))
    assert [p.label for p in paths] == [1.0, 1.0, 2.0, 2.0]
    imgs = list(D.LocalImgReader(scaleTo=10)(iter(paths)))
    assert imgs[0].content.shape == (10, 15, 3)


def _feature(h=40, w=50):
    from PIL import Image

    arr = np.random.RandomState(2).randint(0, 256, (h, w, 3)).astype(np.uint8)
    buf = io.BytesIO()
    Image.fromarray(arr).save(buf, format="PNG")
    return V.ImageFeature(buf.getvalue(), label=torch.tensor([2.0]), uri="x.png"), arr


def test_vision_pipeline_and_frame():
    RNG.setSeed(3)
    f, arr = _feature()
    frame = V.ImageFrame.array([f])
    pipe = V.BytesToMat() >> V.Resize(36, 48) >> V.Brightness(-10, 10) >> V.Contrast(0.8, 1.2) >> \
        V.Saturation(0.8, 1.2) >> V.Hue(-10, 10) >> V.RandomCrop(32, 32) >> V.HFlip() >> \
        V.ChannelNormalize(123, 117, 104, 58, 57, 57) >> V.MatToTensor(toRGB=True) >> \
        V.ImageFrameToSample(targetKeys=["label"])
    frame.transform(pipe)
    out = frame.array[0]
    assert out.isValid() and out[V.ImageFeature.imageTensor].shape == (3, 32, 32)
    assert out.getOriginalSize() == (40, 50, 3)
    mb = list(V.ImageFeatureToMiniBatch(1).apply(iter(frame.array)))
    assert mb[0].getInput().shape == (1, 3, 32, 32)


def test_hsv_roundtrip_and_geometry():
    m = torch.randint(0, 256, (8, 9, 3)).float()
    assert torch.allclose(V.hsv_to_bgr(V.bgr_to_hsv(m)), m, atol=1e-3)
    f = V.ImageFeature()
    f[V.ImageFeature.mat] = m
    V.Expand(minExpandRatio=2, maxExpandRatio=2).transform(f)
    assert f.opencvMat().shape == (16, 18, 3)
    V.CenterCrop(6, 4).transform(f)
    assert f.opencvMat().shape == (4, 6, 3)
    V.Filler(0, 0, 0.5, 0.5, 7).transform(f)
    assert float(f.opencvMat()[0, 0, 0]) == 7.0
    f2 = V.ImageFeature()
    f2[V.ImageFeature.mat] = torch.rand(300, 400, 3) * 255
    V.RandomAlterAspect(cropLength=64).transform(f2)
    assert f2.opencvMat().shape == (64, 64, 3)
    V.ScaleResize(32, 50).transform(f2)
    assert f2.opencvMat().shape[0] == 32
    bad = V.ImageFeature(b"not an image")
    V.BytesToMat().transform(bad)
    assert not bad.isValid()


def test_text_pipeline():
    text = ["The cat sat. The dog ran!", "A cat ran."]
    sents = [s for p in D.SentenceSplitter()(iter(text)) for s in p]
    toks = list(D.SentenceTokenizer()(iter(sents)))
    assert toks[0] == ["the", "cat", "sat", "."]
    padded = list(D.SentenceBiPadding()(iter(toks)))
    dic = D.Dictionary(padded, vocabSize=6)
    assert dic.getVocabSize() == 6 and dic.getIndex("zebra") == 5
    ls = list(D.TextToLabeledSentence(dic)(iter(padded)))
    s = list(D.LabeledSentenceToSample(dic.getVocabSize(), fixDataLength=7, fixLabelLength=7)(iter(ls)))
    assert s[0].feature().shape == (7, 6) and s[0].label().shape == (7,)
    assert float(s[0].label().min()) >= 1


def test_row_transformer_atomic_and_numeric():
    import pandas as pd
    from bigdl_amd.dataset.datamining import RowTransformer

    df = pd.DataFrame({"name": ["a", "b"], "x": [1.0, 3.0], "y": [2, 4], "z": [0.5, 0.25]})
    rows = [r for _, r in df.iterrows()]
    t = list(RowTransformer.atomicWithNumeric(["name"], {"xy": ["x", "y"], "z": ["z"]}).apply(iter(rows)))
    assert t[1]["name"] == ["b"] and t[1]["xy"].tolist() == [3.0, 4.0] and t[0]["z"].tolist() == [0.5]
    allnum = list(RowTransformer.numeric().apply(iter([{"a": 1, "b": 2.5, "c": "s"}])))
    assert allnum[0]["all"].tolist() == [1.0, 2.5]


def test_reference_named_vision_transforms(tmp_path):
    """FixExpand (Expand.scala:102), RandomAspectScale / AspectScale sizing (Resize.scala:117-160), Pipeline,
    PixelNormalize, the ROI transforms and SeqFileFolder.files_to_image_frame under the reference's names."""
    import os

    import torch

    import bigdl_amd.transform.vision.image as V
    from bigdl_amd.dataset.seqfile import generate_seq_files
    from bigdl_amd.examples.seqfile_generator import _synthetic_imagenet
    from bigdl_amd.transform.vision.image.augmentation import aspect_scale_hw
    from bigdl_amd.transform.vision.image.feature import ImageFeature

    f = ImageFeature()
    f[ImageFeature.mat] = torch.ones(10, 20, 3)
    V.FixExpand(30, 40).transform(f)
    m, bb = f[ImageFeature.mat], f[ImageFeature.boundingBox]
    assert m.shape == (30, 40, 3) and float(m.sum()) == 600.0 and float(m[10:20, 10:30].sum()) == 600.0
    assert (bb.x1, bb.y1, bb.x2, bb.y2) == (10.0, 10.0, 30.0, 20.0)
    assert aspect_scale_hw(375, 500, 600, 1000) == (600, 800)
    assert aspect_scale_hw(375, 500, 600, 1000, 32) == (576, 800)
    assert aspect_scale_hw(300, 2000, 600, 1000) == (150, 1000)
    g = ImageFeature()
    g[ImageFeature.mat] = torch.rand(375, 500, 3) * 255
    V.Pipeline([V.RandomAspectScale([600], 32, 1000), V.HFlip()]).transform(g)
    assert tuple(g[ImageFeature.mat].shape) == (576, 800, 3)
    p = ImageFeature()
    p[ImageFeature.mat] = torch.full((2, 2, 3), 5.0)
    V.PixelNormalize(torch.ones(12).tolist()).transform(p)
    assert float(p[ImageFeature.mat].sum()) == 48.0
    _synthetic_imagenet(str(tmp_path / "train"))
    generate_seq_files(str(tmp_path / "train"), str(tmp_path / "seq"), blockSize=5)
    frame = V.SeqFileFolder.files_to_image_frame(str(tmp_path / "seq"), 2)
    assert len(frame.array) == 8 and all(float(x[ImageFeature.label][0]) <= 2 for x in frame.array)
    assert all(hasattr(V, n) for n in ("RoiHFlip", "RoiNormalize", "RoiProject", "RoiResize", "RandomSampler"))


def test_sparse_minibatch_wide_and_deep_training():
    """SampleToMiniBatch turns samples with sparse COO features into a SparseMiniBatch (reference
    S/dataset/MiniBatch.scala:588): the sparse wide features become one [batch, D] sparse tensor with the sample
    index as leading coordinate, dense deep features are stacked; a wide & deep model (SparseLinear + Linear)
    trains on it through Optimizer.optimize()."""
    from bigdl_amd import nn
    from bigdl_amd import optim as O
    from bigdl_amd.dataset.core import DataSet, Sample, SampleToMiniBatch, SparseMiniBatch
    from bigdl_amd.utils.random_generator import RNG

    RNG.setSeed(3)
    g = torch.Generator().manual_seed(0)
    D = 200
    samples = []
    for i in range(64):
        cols = torch.randperm(D, generator=g)[:5]
        wide = torch.sparse_coo_tensor(cols.unsqueeze(0), torch.ones(5), (D,))
        deep = torch.randn(8, generator=g)
        label = torch.tensor(float(1 + (int(cols.min()) % 2)))
        samples.append(Sample([wide, deep], label))
    batches = list(SampleToMiniBatch(16, partitionNum=1).apply(iter(samples[:32])))
    mb = batches[0]
    assert isinstance(mb, SparseMiniBatch) and mb.size() == 16
    x = mb.getInput()
    assert x[1].is_sparse and tuple(x[1].shape) == (16, D) and x[1]._nnz() == 80
    assert tuple(x[2].shape) == (16, 8)
    dense0 = samples[0].features[0].to_dense()
    assert torch.equal(x[1].to_dense()[0], dense0)
    sub = mb.slice(3, 4)
    assert sub.size() == 4 and torch.equal(sub.getInput()[1].to_dense()[0], samples[2].features[0].to_dense())

    model = nn.Sequential()
    model.add(nn.ParallelTable().add(nn.SparseLinear(D, 2)).add(nn.Linear(8, 2)))
    model.add(nn.CAddTable()).add(nn.LogSoftMax())
    opt = O.Optimizer(model, DataSet.array(samples), nn.ClassNLLCriterion(), batchSize=16,
                      optimMethod=O.SGD(0.5), endTrigger=O.Trigger.maxIteration(24))
    opt.device = torch.device("cpu")
    first = []
    opt._iteration_hook = lambda n: first.append(float(opt.state.get("Loss", float("nan"))))
    opt.setLogInterval(1)
    opt.optimize()
    losses = [v for v in first if v == v]
    assert losses[-1] < losses[0], losses
