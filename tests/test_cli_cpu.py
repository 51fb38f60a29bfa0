"""Model-zoo CLI (models/{lenet,resnet,...}/Train|Test, LocalOptimizerPerf) on tiny local / synthetic data."""
import numpy as np

from bigdl_amd.dataset.mnist_cifar import write_mnist
from bigdl_amd.models.cli import main


def test_lenet_train_test_perf(tmp_path, capsys):
    rng = np.random.RandomState(0)
    imgs, labels = rng.randint(0, 255, (64, 28, 28)).astype(np.uint8), rng.randint(0, 10, 64)
    d = str(tmp_path)
    write_mnist(d + "/train-images-idx3-ubyte", d + "/train-labels-idx1-ubyte", imgs, labels)
    write_mnist(d + "/t10k-images-idx3-ubyte", d + "/t10k-labels-idx1-ubyte", imgs[:32], labels[:32])
    assert main(["train", "--model", "lenet5", "--data", d, "--maxEpoch", "1", "-b", "16",
                 "--modelPath", d + "/m.bigdl"]) == 0
    assert main(["test", "--model", "lenet5", "--data", d, "--modelPath", d + "/m.bigdl", "-b", "16"]) == 0
    assert "Top1Accuracy is" in capsys.readouterr().out
    assert main(["perf", "--model", "lenet5", "-b", "8", "-i", "2"]) == 0
    assert "records/second" in capsys.readouterr().out


def test_synthetic_training_for_sequence_and_autoencoder_models():
    assert main(["train", "--model", "rnn", "--synthetic", "16", "--maxEpoch", "1", "-b", "8", "--classNum", "20"]) == 0
    assert main(["train", "--model", "autoencoder", "--synthetic", "16", "--maxEpoch", "1", "-b", "8"]) == 0
