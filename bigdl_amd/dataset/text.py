"""Text pipeline (reference S/dataset/text/*: Dictionary.scala:32, SentenceTokenizer, SentenceSplitter,
SentenceBiPadding, TextToLabeledSentence, LabeledSentenceToSample, LabeledSentence)."""
import re
from collections import Counter

import torch

from .core import Sample, Transformer

SENTENCE_START, SENTENCE_END = "SENTENCESTART", "SENTENCEEND"


class Dictionary:
    """Vocabulary of the ``vocabSize`` most frequent words; unknown words map to the last index
    (Dictionary.scala). Indices are 0-based (``getIndex``); samples add 1 for 1-based lookup tables."""

    def __init__(self, sentences=None, vocabSize=10000):
        self._word2index, self._index2word, self._discard = {}, {}, []
        if sentences is not None:
            counts = Counter(w for s in sentences for w in s)
            words = [w for w, _ in sorted(counts.items(), key=lambda kv: (-kv[1], kv[0]))]
            keep = words[:max(vocabSize - 1, 0)]
            self._discard = words[len(keep):]
            for i, w in enumerate(keep):
                self._word2index[w] = i
                self._index2word[i] = w
            unk = len(keep)
            self._word2index["<unk>"] = unk
            self._index2word[unk] = "<unk>"

    def getVocabSize(self):
        return len(self._word2index)

    def getIndex(self, word):
        return self._word2index.get(word, self._word2index.get("<unk>", len(self._word2index)))

    def getWord(self, index):
        return self._index2word.get(int(index), "<unk>")

    def word2Index(self):
        return dict(self._word2index)

    def index2Word(self):
        return dict(self._index2word)

    def discardVocab(self):
        return list(self._discard)

    def addWord(self, word):
        if word not in self._word2index:
            i = len(self._word2index)
            self._word2index[word] = i
            self._index2word[i] = word
        return self

    def save(self, folder):
        import json
        import os

        os.makedirs(folder, exist_ok=True)
        json.dump(self._word2index, open(os.path.join(folder, "dictionary.json"), "w"))
        json.dump(self._discard, open(os.path.join(folder, "discard.json"), "w"))

    @staticmethod
    def load(folder):
        import json
        import os

        d = Dictionary()
        d._word2index = json.load(open(os.path.join(folder, "dictionary.json")))
        d._index2word = {v: k for k, v in d._word2index.items()}
        p = os.path.join(folder, "discard.json")
        d._discard = json.load(open(p)) if os.path.exists(p) else []
        return d


class SentenceSplitter(Transformer):
    """Paragraph -> sentences (a regex stand-in for the reference's OpenNLP sentence detector)."""

    _re = re.compile(r"(?<=[.!?])\s+")

    def apply(self, it):
        for text in it:
            yield [s for s in self._re.split(text.strip()) if s]


class SentenceTokenizer(Transformer):
    """Sentence -> lower-cased word tokens (a regex stand-in for the OpenNLP tokenizer)."""

    _re = re.compile(r"[A-Za-z0-9']+|[^\sA-Za-z0-9']")

    def apply(self, it):
        for s in it:
            if isinstance(s, (list, tuple)):
                yield [t for x in s for t in self._re.findall(x.lower())]
            else:
                yield self._re.findall(s.lower())


class SentenceBiPadding(Transformer):
    def __init__(self, start=SENTENCE_START, end=SENTENCE_END):
        self.start, self.end = start, end

    def apply(self, it):
        for s in it:
            yield f"{self.start} {s} {self.end}" if isinstance(s, str) else [self.start] + list(s) + [self.end]


class LabeledSentence:
    def __init__(self, data, label):
        self._data, self._label = list(data), list(label)

    def data(self):
        return self._data

    def label(self):
        return self._label

    def dataLength(self):
        return len(self._data)

    def labelLength(self):
        return len(self._label)

    def getData(self, i):
        return self._data[i]

    def getLabel(self, i):
        return self._label[i]


class TextToLabeledSentence(Transformer):
    """Token list -> LabeledSentence for next-word prediction: data = w[0:-1], label = w[1:] (indices)."""

    def __init__(self, dictionary):
        self.dictionary = dictionary

    def apply(self, it):
        for toks in it:
            idx = [float(self.dictionary.getIndex(w)) for w in toks]
            yield LabeledSentence(idx[:-1], idx[1:])


class LabeledSentenceToSample(Transformer):
    """LabeledSentence -> Sample: one-hot features [T, vocab] (``oneHot``) or index features, 1-based labels;
    optional fixed lengths pad with the end-of-sentence index."""

    def __init__(self, vocabLength, fixDataLength=None, fixLabelLength=None, oneHot=True):
        self.vocabLength, self.fixData, self.fixLabel, self.oneHot = vocabLength, fixDataLength, fixLabelLength, \
            oneHot

    def apply(self, it):
        for ls in it:
            data, label = list(ls.data()), list(ls.label())
            if self.fixData:
                pad = data[-1] if data else 0.0
                data = (data + [pad] * self.fixData)[:self.fixData]
            if self.fixLabel:
                pad = label[-1] if label else 0.0
                label = (label + [pad] * self.fixLabel)[:self.fixLabel]
            if self.oneHot:
                f = torch.zeros(len(data), self.vocabLength)
                f[torch.arange(len(data)), torch.tensor(data).long()] = 1.0
            else:
                f = torch.tensor(data) + 1.0
            yield Sample(f, torch.tensor(label) + 1.0)
