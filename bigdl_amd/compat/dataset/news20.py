"""Reference ``bigdl.dataset.news20`` (P/dataset/news20.py): 20 Newsgroups texts and GloVe vectors from a local
directory. Archives already present (``20news-18828.tar.gz``, ``glove.6B.zip``) are extracted; nothing is fetched
(no network in this environment)."""
import os
import tarfile
import zipfile

from .base import maybe_download

NEWS20_URL = "http://qwone.com/~jason/20Newsgroups/20news-18828.tar.gz"
GLOVE_URL = "http://nlp.stanford.edu/data/glove.6B.zip"
CLASS_NUM = 20


def download_news20(dest_dir):
    extracted_to = os.path.join(dest_dir, "20news-18828")
    if os.path.isdir(extracted_to):
        return extracted_to
    path = maybe_download("20news-18828.tar.gz", dest_dir, NEWS20_URL)
    with tarfile.open(path, "r:gz") as tar:
        tar.extractall(dest_dir, filter="data")
    return extracted_to


def download_glove_w2v(dest_dir):
    extracted_to = os.path.join(dest_dir, "glove.6B")
    if os.path.isdir(extracted_to):
        return extracted_to
    path = maybe_download("glove.6B.zip", dest_dir, GLOVE_URL)
    with zipfile.ZipFile(path) as z:
        z.extractall(extracted_to)
    return extracted_to


def get_news20(source_dir="./data/news20/"):
    """[(text, 1-based label)] over the class folders of 20news-18828 (files with numeric names)."""
    news_dir = download_news20(source_dir)
    texts = []
    label_id = 0
    for name in sorted(os.listdir(news_dir)):
        path = os.path.join(news_dir, name)
        label_id += 1
        if os.path.isdir(path):
            for fname in sorted(os.listdir(path)):
                if fname.isdigit():
                    with open(os.path.join(path, fname), encoding="latin-1") as f:
                        texts.append((f.read(), label_id))
    return texts


def get_glove_w2v(source_dir="./data/news20/", dim=100):
    """{word: [float] * dim} from glove.6B.<dim>d.txt."""
    w2v_dir = download_glove_w2v(source_dir)
    out = {}
    with open(os.path.join(w2v_dir, f"glove.6B.{dim}d.txt"), encoding="latin-1") as f:
        for line in f:
            parts = line.split(" ")
            out[parts[0]] = [float(v) for v in parts[1:]]
    return out


__all__ = ["CLASS_NUM", "download_news20", "download_glove_w2v", "get_news20", "get_glove_w2v"]
