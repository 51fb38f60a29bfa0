"""Reference ``bigdl.dataset.sentence`` (P/dataset/sentence.py) without NLTK (not installed): sentences split after
``.``, ``!`` or ``?`` followed by white space, and words / punctuation marks are separate tokens — regular-expression
stand-ins for NLTK's Punkt splitter and word tokenizer (close on plain prose, not identical on abbreviations)."""
import re

_SENT = re.compile(r"(?<=[.!?])\s+")
_TOKEN = re.compile(r"\w+|[^\w\s]")


def read_localfile(fileName):
    with open(fileName) as f:
        return [line for line in f]


def sentences_split(line):
    return [s for s in _SENT.split(line.strip()) if s]


def sentences_bipadding(sent):
    return "SENTENCESTART " + sent + " SENTENCEEND"


def sentence_tokenizer(sentences):
    return _TOKEN.findall(sentences)


__all__ = ["read_localfile", "sentences_split", "sentences_bipadding", "sentence_tokenizer"]
