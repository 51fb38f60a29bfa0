"""MNIST (idx) and CIFAR-10 (binary batches) readers producing ByteRecords with 1-based labels
(reference S/models/lenet/Utils.scala load :81, S/models/vgg/Utils.scala loadTrain/loadTest/load :139-210).
Files are parsed with numpy views (no per-byte loops)."""
import os

import numpy as np

from .image import ByteRecord

TRAIN_MEAN_MNIST, TRAIN_STD_MNIST = 0.13066047740239506, 0.3081078
TEST_MEAN_MNIST, TEST_STD_MNIST = 0.13251460696903547, 0.31048024
CIFAR_TRAIN_MEAN = (0.4913996898739353, 0.4821584196221302, 0.44653092422369434)
CIFAR_TRAIN_STD = (0.24703223517429462, 0.2434851308749409, 0.26158784442034005)


def _u32(b, off):
    return int.from_bytes(b[off:off + 4], "big")


def load_mnist(featureFile, labelFile):
    fb = open(featureFile, "rb").read()
    lb = open(labelFile, "rb").read()
    assert _u32(lb, 0) == 2049 and _u32(fb, 0) == 2051, "bad MNIST magic numbers"
    n = _u32(lb, 4)
    assert n == _u32(fb, 4)
    rows, cols = _u32(fb, 8), _u32(fb, 12)
    imgs = np.frombuffer(fb, dtype=np.uint8, offset=16).reshape(n, rows * cols)
    labels = np.frombuffer(lb, dtype=np.uint8, offset=8)
    return [ByteRecord(imgs[i].tobytes(), float(labels[i]) + 1.0) for i in range(n)]


def write_mnist(featureFile, labelFile, images, labels):
    """Write uint8 [N, R, C] images and 0-based labels in idx format (test fixtures)."""
    n, r, c = images.shape
    with open(featureFile, "wb") as f:
        f.write((2051).to_bytes(4, "big") + n.to_bytes(4, "big") + r.to_bytes(4, "big") + c.to_bytes(4, "big"))
        f.write(np.asarray(images, dtype=np.uint8).tobytes())
    with open(labelFile, "wb") as f:
        f.write((2049).to_bytes(4, "big") + n.to_bytes(4, "big"))
        f.write(np.asarray(labels, dtype=np.uint8).tobytes())


def load_cifar_file(path, result):
    """One CIFAR-10 binary batch: records of 1 label byte + 3072 bytes planar RGB -> BGR interleaved records
    with the (width, height) int32 header of BGRImage.copy; labels 1-based."""
    raw = np.frombuffer(open(path, "rb").read(), dtype=np.uint8)
    rec = raw.reshape(-1, 3073)
    labels = rec[:, 0]
    planes = rec[:, 1:].reshape(-1, 3, 32, 32)
    bgr = planes[:, ::-1].transpose(0, 2, 3, 1)     # [N, 32, 32, 3] B, G, R
    hdr = (32).to_bytes(4, "big") + (32).to_bytes(4, "big")
    for i in range(rec.shape[0]):
        result.append(ByteRecord(hdr + np.ascontiguousarray(bgr[i]).tobytes(), float(labels[i]) + 1.0))
    return result


def load_cifar_train(folder):
    out = []
    for i in range(1, 6):
        load_cifar_file(os.path.join(folder, f"data_batch_{i}.bin"), out)
    return out


def load_cifar_test(folder):
    return load_cifar_file(os.path.join(folder, "test_batch.bin"), [])
