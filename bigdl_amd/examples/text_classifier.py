"""Text classification with a 1-D convolutional network over pre-trained word vectors.

Reference: S/example/textclassification/TextClassifier.scala + S/example/utils/TextClassifier.scala (loadRawData,
analyzeTexts: frequency-ranked vocabulary minus the 10 most frequent words, shaping to maxSequenceLength,
vectorization with GloVe, buildModel: TemporalConvolution(embDim, 256, 5) -> ReLU -> TemporalMaxPooling ->
Linear(256, 128) -> Dropout -> ReLU -> Linear(128, classNum) -> LogSoftMax, trained with Adagrad and validated
with Top1Accuracy every epoch).

Data: ``--baseDir`` holding ``20news-18828/<category>/<numeric file names>`` and (optionally)
``glove.6B/glove.6B.<dim>d.txt``; without it a synthetic corpus (class keywords mixed into random filler text)
is generated. Words without a GloVe vector get a fixed random vector.
"""
import argparse
import collections
import os
import random

import torch

from .. import nn
from ..dataset.core import DataSet, Sample
from ..optim import Adagrad, Optimizer, Top1Accuracy, Trigger
from ._common import device_of, load_glove, tokens


def load_raw_data(text_dir):
    texts, labels = [], []
    cats = sorted(d for d in os.listdir(text_dir) if os.path.isdir(os.path.join(text_dir, d)))
    for label, cat in enumerate(cats, start=1):
        p = os.path.join(text_dir, cat)
        for fn in sorted(f for f in os.listdir(p) if f.isdigit()):
            with open(os.path.join(p, fn), encoding="ISO-8859-1") as f:
                texts.append(f.read())
            labels.append(float(label))
    return texts, labels, len(cats)


def synthetic_corpus(n_docs=240, classes=4, seed=1):
    rng = random.Random(seed)
    filler = [f"w{i}" for i in range(300)]
    keywords = [[f"k{c}_{i}" for i in range(12)] for c in range(classes)]
    texts, labels = [], []
    for d in range(n_docs):
        c = d % classes
        words = [rng.choice(filler) for _ in range(60)] + [rng.choice(keywords[c]) for _ in range(12)]
        rng.shuffle(words)
        texts.append(" ".join(words))
        labels.append(float(c + 1))
    return texts, labels, classes


def analyze_texts(texts, max_words, drop_top):
    freq = collections.Counter(t for text in texts for t in tokens(text))
    ranked = [w for w, _ in sorted(freq.items(), key=lambda kv: (-kv[1], kv[0]))][drop_top:max_words]
    return {w: i + 1 for i, w in enumerate(ranked)}          # 1-based word index (reference WordMeta.index)


def vectorize(texts, word2index, seq_len, dim, glove, seed=7):
    g = torch.Generator().manual_seed(seed)
    table = torch.randn(len(word2index) + 1, dim, generator=g) * 0.5
    table[0] = 0.0                                           # padding
    for idx, v in glove.items():
        table[idx] = v
    feats = []
    for text in texts:
        ids = [word2index[t] for t in tokens(text) if t in word2index][:seq_len]
        ids = ids + [0] * (seq_len - len(ids))                # shaping: pad at the end
        feats.append(table[torch.tensor(ids)])
    return feats


def build_model(emb_dim, seq_len, class_num):
    return (nn.Sequential()
            .add(nn.TemporalConvolution(emb_dim, 256, 5))
            .add(nn.ReLU())
            .add(nn.TemporalMaxPooling(seq_len - 5 + 1))
            .add(nn.Squeeze(2))
            .add(nn.Linear(256, 128))
            .add(nn.Dropout(0.2))
            .add(nn.ReLU())
            .add(nn.Linear(128, class_num))
            .add(nn.LogSoftMax()))


def build_parser():
    p = argparse.ArgumentParser(prog="textclassification")
    p.add_argument("--baseDir", default=None)
    p.add_argument("--maxSequenceLength", type=int, default=100)
    p.add_argument("--maxWordsNum", type=int, default=20000)
    p.add_argument("--trainingSplit", type=float, default=0.8)
    p.add_argument("--batchSize", type=int, default=32)
    p.add_argument("--embeddingDim", type=int, default=100)
    p.add_argument("--learningRate", type=float, default=0.01)
    p.add_argument("--maxEpoch", type=int, default=20)
    p.add_argument("--dropTop", type=int, default=10, help="drop the N most frequent words (reference: 10)")
    p.add_argument("--device", default="auto")
    return p


def run(args):
    if args.baseDir:
        texts, labels, classes = load_raw_data(os.path.join(args.baseDir, "20news-18828"))
    else:
        texts, labels, classes = synthetic_corpus()
        args.dropTop = 0
    word2index = analyze_texts(texts, args.maxWordsNum, args.dropTop)
    glove = {}
    if args.baseDir:
        gp = os.path.join(args.baseDir, "glove.6B", f"glove.6B.{args.embeddingDim}d.txt")
        if os.path.exists(gp):
            glove = load_glove(gp, word2index, args.embeddingDim)
    feats = vectorize(texts, word2index, args.maxSequenceLength, args.embeddingDim, glove)
    samples = [Sample(f, torch.tensor([l])) for f, l in zip(feats, labels)]
    random.Random(3).shuffle(samples)
    n_train = int(len(samples) * args.trainingSplit)
    train, val = samples[:n_train], samples[n_train:]
    model = build_model(args.embeddingDim, args.maxSequenceLength, classes)
    dev = device_of(args.device)
    opt = Optimizer(model=model, dataset=DataSet.array(train), criterion=nn.ClassNLLCriterion(),
                    batchSize=args.batchSize)
    opt.device = dev
    opt.setOptimMethod(Adagrad(learningRate=args.learningRate, learningRateDecay=0.001))
    opt.setValidation(Trigger.everyEpoch(), DataSet.array(val), [Top1Accuracy()], args.batchSize)
    opt.setEndWhen(Trigger.maxEpoch(args.maxEpoch))
    trained = opt.optimize()
    trained.evaluate()
    correct = 0
    with torch.no_grad():
        x = torch.stack([s.feature() for s in val])
        y = torch.tensor([float(s.label()[0]) for s in val])
        pred = trained.forward(x.to(dev)).float().cpu().argmax(1) + 1
        correct = int((pred == y.long()).sum())
    return {"classes": classes, "train": len(train), "val": len(val), "val_top1": correct / max(len(val), 1),
            "loss": opt.state.get("Loss")}


def main(argv=None):
    res = run(build_parser().parse_args(argv))
    print(res)
    return 0
