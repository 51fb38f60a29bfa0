"""Word-level language model on a PTB-style corpus.

Reference: S/example/languagemodel/PTBModel.scala (``lstm``: LookupTable(vocab, hidden) -> Dropout -> stacked
Recurrent(LSTM) -> TimeDistributed(Linear(hidden, vocab)); ``transformer``: the Transformer language model) and
PTBWordLM.scala (SequencePreprocess reader: fixed-length windows of numSteps + 1 word ids, input = first numSteps,
target = the next word at every step; Adagrad; TimeDistributedCriterion(CrossEntropyCriterion, sizeAverage=false);
Loss validation every epoch). Perplexity = exp(mean per-word cross entropy).

Data: ``--dataFolder`` with ptb.train.txt / ptb.valid.txt (one sentence per line, ``<eos>`` appended); without it a
synthetic corpus from a sparse first-order Markov chain over a small vocabulary (learnable structure).
"""
import argparse
import collections
import math
import os
import random

import torch

from .. import nn
from ..dataset.core import DataSet, Sample
from ..optim import Adagrad, Loss, Optimizer, Trigger
from ._common import device_of


def read_words(path):
    with open(path) as f:
        return [w for line in f for w in line.split() + ["<eos>"]]


def build_vocab(words, vocab_size):
    freq = collections.Counter(words)
    ranked = [w for w, _ in sorted(freq.items(), key=lambda kv: (-kv[1], kv[0]))][:vocab_size - 1]
    vocab = {w: i + 1 for i, w in enumerate(ranked)}          # 1-based ids; vocab_size = unknown word
    return vocab


def to_ids(words, vocab, vocab_size):
    return [vocab.get(w, vocab_size) for w in words]


def markov_corpus(n_words, vocab_size, seed=5):
    rng = random.Random(seed)
    nxt = {w: [rng.randrange(1, vocab_size + 1) for _ in range(3)] for w in range(1, vocab_size + 1)}
    ids, w = [], 1
    for _ in range(n_words):
        w = rng.choice(nxt[w]) if rng.random() < 0.9 else rng.randrange(1, vocab_size + 1)
        ids.append(w)
    return ids


def windows(ids, num_steps):
    """Non-overlapping windows of num_steps + 1 ids -> (input ids, next-word targets), both 1-based."""
    out = []
    for s in range(0, len(ids) - num_steps - 1, num_steps):
        seg = torch.tensor(ids[s:s + num_steps + 1], dtype=torch.float32)
        out.append(Sample(seg[:-1], seg[1:]))
    return out


def lstm_model(vocab, hidden, num_layers, keep_prob):
    m = nn.Sequential().add(nn.LookupTable(vocab, hidden))
    if keep_prob < 1:
        m.add(nn.Dropout(1 - keep_prob))
    for _ in range(num_layers):
        m.add(nn.Recurrent().add(nn.LSTM(hidden, hidden)))
    return m.add(nn.TimeDistributed(nn.Linear(hidden, vocab)))


def transformer_model(vocab, hidden, num_layers, keep_prob):
    from ..nn.transformer import Transformer

    return (nn.Sequential()
            .add(Transformer(vocabSize=vocab, hiddenSize=hidden, numHeads=4, filterSize=hidden * 4,
                             numHiddenlayers=num_layers, embeddingDropout=1 - keep_prob, attentionDropout=0.1,
                             ffnDropout=0.1))
            .add(nn.TimeDistributed(nn.Linear(hidden, vocab))))


def build_parser():
    p = argparse.ArgumentParser(prog="languagemodel")
    p.add_argument("--dataFolder", default=None)
    p.add_argument("--vocabSize", type=int, default=10000)
    p.add_argument("--hiddenSize", type=int, default=200)
    p.add_argument("--numLayers", type=int, default=2)
    p.add_argument("--numSteps", type=int, default=20)
    p.add_argument("--batchSize", type=int, default=20)
    p.add_argument("--learningRate", type=float, default=0.1)
    p.add_argument("--keepProb", type=float, default=2.0, help=">= 1 disables dropout (reference default 2.0)")
    p.add_argument("--maxEpoch", type=int, default=4)
    p.add_argument("--model", choices=["lstm", "transformer"], default="lstm")
    p.add_argument("--syntheticWords", type=int, default=20000)
    p.add_argument("--device", default="auto")
    return p


def perplexity(model, data, dev, vocab):
    crit = nn.CrossEntropyCriterion()
    model.evaluate()
    tot, n = 0.0, 0
    with torch.no_grad():
        for i in range(0, len(data), 32):
            xs = torch.stack([s.feature() for s in data[i:i + 32]]).to(dev)
            ys = torch.stack([s.label() for s in data[i:i + 32]]).to(dev)
            out = model.forward(xs).float()
            tot += float(crit.forward(out.reshape(-1, vocab), ys.reshape(-1))) * ys.numel()
            n += ys.numel()
    return math.exp(tot / max(n, 1))


def run(args):
    if args.dataFolder:
        tr = read_words(os.path.join(args.dataFolder, "ptb.train.txt"))
        va = read_words(os.path.join(args.dataFolder, "ptb.valid.txt"))
        vocab = build_vocab(tr, args.vocabSize)
        train_ids, val_ids = to_ids(tr, vocab, args.vocabSize), to_ids(va, vocab, args.vocabSize)
    else:
        ids = markov_corpus(args.syntheticWords, args.vocabSize)
        cut = int(len(ids) * 0.9)
        train_ids, val_ids = ids[:cut], ids[cut:]
    train, val = windows(train_ids, args.numSteps), windows(val_ids, args.numSteps)
    build = lstm_model if args.model == "lstm" else transformer_model
    model = build(args.vocabSize, args.hiddenSize, args.numLayers, args.keepProb)
    dev = device_of(args.device)
    crit = nn.TimeDistributedCriterion(nn.CrossEntropyCriterion(), sizeAverage=False, dimension=2)
    opt = Optimizer(model=model, dataset=DataSet.array(train), criterion=crit, batchSize=args.batchSize)
    opt.device = dev
    opt.setOptimMethod(Adagrad(learningRate=args.learningRate, learningRateDecay=0.001))
    opt.setValidation(Trigger.everyEpoch(), DataSet.array(val),
                      [Loss(nn.TimeDistributedCriterion(nn.CrossEntropyCriterion(), sizeAverage=True, dimension=2))],
                      args.batchSize)
    opt.setEndWhen(Trigger.maxEpoch(args.maxEpoch))
    before = perplexity(model.to(dev), val, dev, args.vocabSize)
    trained = opt.optimize()
    after = perplexity(trained, val, dev, args.vocabSize)
    return {"train_windows": len(train), "val_perplexity_before": before, "val_perplexity": after}


def main(argv=None):
    print(run(build_parser().parse_args(argv)))
    return 0
