"""Example applications on the GPU engines: the model validator through the fused graph and int8 plans."""
import pytest

from bigdl_amd import examples

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("engine", ["dnn", "int8"])
def test_model_validator_gpu_engines(engine):
    m = examples.get("loadmodel")
    r = m.run(m.build_parser().parse_args(["--modelType", "caffe", "--model", "resnet50", "--classNum", "10",
                                           "--limit", "16", "--batchSize", "8", "--engine", engine]))
    assert r["images"] == 16 and 0.0 <= r["top1"] <= 1.0


def test_text_classifier_gpu():
    m = examples.get("textclassification")
    r = m.run(m.build_parser().parse_args(["--maxEpoch", "6", "--maxSequenceLength", "72", "--embeddingDim", "32",
                                           "--learningRate", "0.05"]))
    assert r["val_top1"] >= 0.8


def test_int8_example_gpu():
    m = examples.get("int8")
    r = m.run(m.build_parser().parse_args(["--imageSize", "32", "--valSize", "32", "--calibSize", "16"]))
    assert r["layers_with_scales"] > 10 and r["top1_agreement"] >= 0.8


@pytest.mark.parametrize("training", ["1", "0"])
def test_perf_example_gpu(training):
    m = examples.get("perf")
    r = m.run(m.build_parser().parse_args(["--model", "resnet50", "--batchSize", "8", "--iteration", "2",
                                           "--training", training, "--classNum", "10"]))
    assert r["images_per_s"] > 0


def test_lenet_local_gpu():
    m = examples.get("lenetlocal")
    r = m.run(m.build_parser().parse_args(["--maxEpoch", "2"]))
    assert r["top1"] >= 0.9
