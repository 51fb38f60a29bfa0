"""Sentiment classification of every node of a constituency tree with a Binary Tree-LSTM.

Reference: S/example/treeLSTMSentiment/TreeSentiment.scala (model: ParallelTable(LookupTable word embedding,
Identity tree) -> BinaryTreeLSTM(embDim, hidden) -> TimeDistributed(Dropout) -> TimeDistributed(Linear(hidden,
classNum)) -> TimeDistributed(LogSoftMax)), Train.scala (SST parents / labels / sents files, labels shifted to
1..5, padding label -1 ignored by ClassNLLCriterion, Adagrad with weight decay, TreeNNAccuracy on the root) and
Utils.scala (parent-pointer lists -> TensorTree encoding).

Data: ``--dataDir`` with ``{train,dev}/{sents,parents,labels}.txt`` (Stanford TreeLSTM preprocessing); without
it, synthetic sentences whose node labels follow the summed polarity of the words under each node.
This example drives the model through the module API (forward / backward / getParameters + OptimMethod), the
reference's LocalOptimizer-free training style.
"""
import argparse
import os
import random

import torch

from .. import nn
from ..nn.tree_lstm import TensorTree
from ..optim import Adagrad
from ..utils.table import Table
from ._common import device_of


def parents_to_tree(parents):
    """Parent-pointer list (1-based, 0 = root; leaves are the first len(sentence) nodes) -> (N, 3) encoding."""
    n = len(parents)
    t = TensorTree(torch.zeros(n, 3))
    leaf = 0
    for i, p in enumerate(parents, start=1):
        if p == 0:
            t.markAsRoot(i)
        else:
            t.addChild(p, i)
    for i in range(1, n + 1):          # leaves: nodes without children, in order -> word positions
        if t.noChild(i):
            leaf += 1
            t.markAsLeaf(i, leaf) if t.c[i - 1][-1] != -1 else None
    return t.content


def read_split(d, vocab):
    with open(os.path.join(d, "sents.txt")) as f:
        sents = [l.split() for l in f]
    with open(os.path.join(d, "parents.txt")) as f:
        parents = [[int(x) for x in l.split()] for l in f]
    with open(os.path.join(d, "labels.txt")) as f:
        labels = [[(int(x) + 3 if x != "#" else -1) for x in l.split()] for l in f]
    out = []
    for s, p, l in zip(sents, parents, labels):
        ids = [vocab.setdefault(w, len(vocab) + 1) for w in s]
        out.append((torch.tensor(ids, dtype=torch.float32), parents_to_tree(p), torch.tensor(l, dtype=torch.float32)))
    return out


def synthetic_trees(n, length=8, vocab=40, seed=2):
    """Random binary trees over `length` words; node label = 1/2/3 for negative / neutral / positive span sum."""
    rng = random.Random(seed)
    pol = {w: (1 if w <= vocab // 3 else -1 if w > 2 * vocab // 3 else 0) for w in range(1, vocab + 1)}
    data = []
    for _ in range(n):
        words = [rng.randint(1, vocab) for _ in range(length)]
        # nodes 1..L are leaves; merge random adjacent spans bottom-up
        spans = [(i + 1, [i]) for i in range(length)]
        parents = [0] * (2 * length - 1)
        nxt = length + 1
        while len(spans) > 1:
            k = rng.randrange(len(spans) - 1)
            (a, sa), (b, sb) = spans[k], spans[k + 1]
            parents[a - 1] = nxt
            parents[b - 1] = nxt
            spans[k:k + 2] = [(nxt, sa + sb)]
            nxt += 1
        members = {i + 1: [i] for i in range(length)}
        for node in range(length + 1, 2 * length):
            kids = [i + 1 for i, p in enumerate(parents) if p == node]
            members[node] = sum((members[c] for c in kids), [])
        labels = []
        for node in range(1, 2 * length):
            s = sum(pol[words[i]] for i in members[node])
            labels.append(3.0 if s > 0 else 1.0 if s < 0 else 2.0)
        data.append((torch.tensor(words, dtype=torch.float32), parents_to_tree(parents),
                     torch.tensor(labels)))
    return data


def build_model(vocab, emb_dim, hidden, classes, p=0.5, embeddings=None):
    emb = nn.LookupTable(vocab, emb_dim)
    if embeddings is not None:
        emb.weight.data.copy_(embeddings)
    tree = (nn.Sequential()
            .add(nn.BinaryTreeLSTM(emb_dim, hidden, withGraph=True))
            .add(nn.TimeDistributed(nn.Dropout(p)))
            .add(nn.TimeDistributed(nn.Linear(hidden, classes)))
            .add(nn.TimeDistributed(nn.LogSoftMax())))
    return nn.Sequential().add(nn.ParallelTable().add(emb).add(nn.Identity())).add(tree)


def _batch(items, dev):
    L = max(int(w.numel()) for w, _, _ in items)
    N = max(int(t.shape[0]) for _, t, _ in items)
    words = torch.ones(len(items), L)
    trees = torch.full((len(items), N, 3), -1.0)
    labels = torch.full((len(items), N), -1.0)
    for b, (w, t, l) in enumerate(items):
        words[b, :w.numel()] = w
        trees[b, :t.shape[0]] = t
        labels[b, :l.numel()] = l
    return Table(words.to(dev), trees.to(dev)), labels.to(dev)


def _root_index(trees):
    return (trees[..., -1] == -1).float().argmax(dim=1)


def run(args):
    dev = device_of(args.device)
    if args.dataDir:
        vocab = {}
        train = read_split(os.path.join(args.dataDir, "train"), vocab)
        val = read_split(os.path.join(args.dataDir, "dev"), vocab)
        V, classes = len(vocab) + 1, 5
    else:
        data = synthetic_trees(args.synthetic)
        cut = int(len(data) * 0.8)
        train, val = data[:cut], data[cut:]
        V, classes = 40, 3
    torch.manual_seed(0)
    model = build_model(V, args.embeddingDim, args.hiddenSize, classes, args.p).to(dev)
    crit = nn.TimeDistributedCriterion(nn.ClassNLLCriterion(paddingValue=-1), sizeAverage=True)
    w, g = model.getParameters()
    om = Adagrad(learningRate=args.learningRate, weightDecay=args.regRate)
    rng = random.Random(0)
    for _ in range(args.epoch):
        model.training()
        rng.shuffle(train)
        for i in range(0, len(train), args.batchSize):
            x, y = _batch(train[i:i + args.batchSize], dev)

            def feval(_w):
                model.zeroGradParameters()
                out = model.forward(x)
                loss = crit.forward(out, y)
                model.backward(x, crit.backward(out, y))
                return loss, g
            om.optimize(feval, w)
    model.evaluate()
    correct = 0
    with torch.no_grad():
        for i in range(0, len(val), 64):
            x, y = _batch(val[i:i + 64], dev)
            out = model.forward(x).float()
            r = _root_index(x[2])
            pred = out[torch.arange(out.shape[0]), r].argmax(-1) + 1
            correct += int((pred == y[torch.arange(y.shape[0]), r].long()).sum())
    return {"train_trees": len(train), "val_trees": len(val), "root_accuracy": correct / max(len(val), 1)}


def build_parser():
    p = argparse.ArgumentParser(prog="treelstm")
    p.add_argument("--dataDir", default=None)
    p.add_argument("--batchSize", type=int, default=32)
    p.add_argument("--hiddenSize", type=int, default=150)
    p.add_argument("--embeddingDim", type=int, default=64)
    p.add_argument("--learningRate", type=float, default=0.05)
    p.add_argument("--regRate", type=float, default=1e-4)
    p.add_argument("--p", type=float, default=0.5)
    p.add_argument("--epoch", type=int, default=5)
    p.add_argument("--synthetic", type=int, default=400)
    p.add_argument("--device", default="auto")
    return p


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
