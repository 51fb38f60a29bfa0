"""Example applications (bigdl_amd.examples, reference S/example/**) run end to end on small synthetic data."""
import pytest

from bigdl_amd import examples


def _run(name, argv):
    m = examples.get(name)
    return m.run(m.build_parser().parse_args(argv + ["--device", "cpu"] if "--device" in
                                             m.build_parser().format_help() else argv))


def test_text_classification_learns():
    r = _run("textclassification", ["--maxEpoch", "6", "--maxSequenceLength", "72", "--embeddingDim", "32",
                                     "--learningRate", "0.05"])
    assert r["val_top1"] >= 0.8


def test_ptb_lstm_language_model_perplexity_drops():
    r = _run("languagemodel", ["--vocabSize", "50", "--hiddenSize", "32", "--numSteps", "10", "--batchSize", "16",
                               "--maxEpoch", "3", "--syntheticWords", "6000"])
    assert r["val_perplexity"] < 0.5 * r["val_perplexity_before"]


def test_tree_lstm_sentiment_learns():
    r = _run("treelstm", ["--hiddenSize", "48", "--epoch", "8", "--p", "0.1", "--synthetic", "400"])
    assert r["root_accuracy"] >= 0.8


def test_udf_predictor_query():
    r = _run("udfpredictor", [])
    assert r["rows"] == 60 and r["accuracy"] >= 0.8 and 0 < r["query_rows"] < 60


def test_image_predictor_pipeline():
    r = _run("imagepredictor", [])
    assert r["images"] == 6 and all(1 <= p <= 10 for _, p in r["predictions"])


def test_tf_load_and_save_roundtrip():
    r = _run("tfloadandsave", [])
    assert r["max_abs_diff"] < 1e-5


@pytest.mark.parametrize("fmt", ["caffe", "bigdl", "torch"])
def test_model_validator_loads_every_format(fmt):
    r = _run("loadmodel", ["--modelType", fmt, "--model", "resnet50", "--classNum", "10", "--limit", "4",
                           "--batchSize", "2", "--engine", "blas"])
    assert r["images"] == 4 and 0.0 <= r["top5"] <= 1.0


def test_examples_cli_lists_examples(capsys):
    assert examples.main([]) == 2
    assert "textclassification" in capsys.readouterr().out


def test_lenet_local_train_test_predict():
    r = _run("lenetlocal", ["--maxEpoch", "2"])
    assert r["top1"] >= 0.9 and r["predicted"] == r["labels"]


@pytest.mark.parametrize("task,key,bound", [("logreg", "train_accuracy", 0.9), ("multilabel", "mse", 1e-3),
                                            ("lenet", "test_accuracy", 0.7)])
def test_ml_pipeline_tasks(task, key, bound):
    r = _run("mlpipeline", ["--task", task, "--maxEpoch", "5"])
    assert (r[key] >= bound) if key != "mse" else (r[key] <= bound)


def test_keras_lenet_trains():
    r = _run("keras", ["--maxEpoch", "3"])
    assert r["test_accuracy"] >= 0.9 and r["predict_shape"] == [8, 10]


def test_int8_scales_then_inference():
    r = _run("int8", ["--imageSize", "32", "--valSize", "16", "--calibSize", "8"])
    assert r["layers_with_scales"] > 10 and r["top1_agreement"] >= 0.8 and r["rel_output_error"] < 0.1


def test_tf_transfer_learning_trains_head_only():
    r = _run("tftransferlearning", ["--maxEpoch", "4"])
    assert r["extractor_frozen"] and r["test_accuracy"] >= 0.9


def test_image_transfer_learning():
    r = _run("imagetransferlearning", [])
    assert r["images"] == 16 and r["test_accuracy"] >= 0.75


@pytest.mark.parametrize("mode", ["imagenet", "coco"])
def test_seqfile_generators(mode):
    r = _run("seqfile", ["--mode", mode, "--blockSize", "2"])
    assert r["records"] == (12 if mode == "imagenet" else 3)
    if mode == "coco":
        assert r["annotations"] == 6


def test_perf_inference_cpu():
    r = _run("perf", ["--model", "resnet50", "--batchSize", "1", "--iteration", "1", "--training", "0",
                      "--classNum", "10"])
    assert r["images_per_s"] > 0
