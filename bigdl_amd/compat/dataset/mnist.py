"""``bigdl.dataset.mnist`` (reference P/dataset/mnist.py): IDX-file readers over a local directory (there is no
download here: the four ``*-ubyte.gz`` / ``*-ubyte`` files must already be in ``train_dir``)."""
import gzip
import os

import numpy as np

TRAIN_MEAN = 0.13066047740239506 * 255
TRAIN_STD = 0.3081078 * 255
TEST_MEAN = 0.13251460696903547 * 255
TEST_STD = 0.31048024 * 255

_FILES = {"train": ("train-images-idx3-ubyte", "train-labels-idx1-ubyte"),
          "test": ("t10k-images-idx3-ubyte", "t10k-labels-idx1-ubyte")}


def _open(path):
    if os.path.exists(path + ".gz"):
        return gzip.open(path + ".gz", "rb")
    if os.path.exists(path):
        return open(path, "rb")
    raise FileNotFoundError(f"{path}(.gz) not found (no network access: place the MNIST files there)")


def extract_images(f):
    data = f.read()
    magic, n, rows, cols = np.frombuffer(data[:16], dtype=">u4")
    if magic != 2051:
        raise ValueError(f"Invalid magic number {magic} in MNIST image file")
    return np.frombuffer(data[16:], dtype=np.uint8).reshape(int(n), int(rows), int(cols), 1)


def extract_labels(f):
    data = f.read()
    magic, n = np.frombuffer(data[:8], dtype=">u4")
    if magic != 2049:
        raise ValueError(f"Invalid magic number {magic} in MNIST label file")
    return np.frombuffer(data[8:], dtype=np.uint8)


def read_data_sets(train_dir, data_type="train"):
    """(images [n, 28, 28, 1] uint8, labels [n] uint8, 0-based)."""
    img, lab = _FILES[data_type]
    with _open(os.path.join(train_dir, img)) as f:
        images = extract_images(f)
    with _open(os.path.join(train_dir, lab)) as f:
        labels = extract_labels(f)
    return images, labels


def load_data(location="/tmp/mnist"):
    from .transformer import normalizer

    (train_images, train_labels) = read_data_sets(location, "train")
    (test_images, test_labels) = read_data_sets(location, "test")
    return (normalizer(train_images, TRAIN_MEAN, TRAIN_STD), train_labels + 1), \
        (normalizer(test_images, TRAIN_MEAN, TRAIN_STD), test_labels + 1)
