"""Shared helpers of the example applications."""
import re

import torch

_TOKEN = re.compile(r"[A-Za-z0-9']+")


def tokens(text):
    """Lower-cased word tokens (reference SimpleTokenizer.toTokens)."""
    return [t.lower() for t in _TOKEN.findall(text)]


def device_of(arg):
    if arg in (None, "auto"):
        return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(arg)


def load_glove(path, word2index, dim):
    """word index -> vector from a GloVe text file (words not in the vocabulary are skipped)."""
    vecs = {}
    with open(path, encoding="ISO-8859-1") as f:
        for line in f:
            parts = line.rstrip().split(" ")
            w = parts[0]
            if w in word2index and len(parts) == dim + 1:
                vecs[word2index[w]] = torch.tensor([float(v) for v in parts[1:]])
    return vecs
