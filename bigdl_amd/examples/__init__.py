"""Example applications (reference S/example/**): end-to-end programs built only on the public bigdl_amd API.

    python -m bigdl_amd.examples <name> [options]      (``--help`` per example)

    textclassification   TextClassifier: 20-newsgroup-style folders + GloVe -> TemporalConvolution classifier
                         (S/example/textclassification, S/example/utils/TextClassifier.scala)
    languagemodel        PTBWordLM: PTB-style corpus -> embedding + stacked LSTM word language model, perplexity
                         (S/example/languagemodel/PTBModel.scala, PTBWordLM.scala)
    treelstm             TreeLSTMSentiment: SST-style constituency trees -> BinaryTreeLSTM node sentiment
                         (S/example/treeLSTMSentiment)
    loadmodel            ModelValidator: load a BigDL / Caffe / Torch7 / TensorFlow model, optionally lower it to the
                         fused GPU engine or int8, validate Top-1 / Top-5 on an image folder (S/example/loadmodel)
    udfpredictor         DataframePredictor: a trained text model applied as a batched column UDF over a DataFrame,
                         then filtered like the reference's Spark SQL query (S/example/udfpredictor)
    imagepredictor       ImagePredictor: DLImageReader + DLClassifierModel over an image folder
                         (S/example/imageclassification)
    tfloadandsave        TensorFlow interop: save a model as a TF GraphDef, load it back and compare
                         (S/example/tensorflow/loadandsave)
    tftransferlearning   TensorFlow GraphDef as a frozen feature extractor + a newly trained head
                         (S/example/tensorflow/transferlearning)
    lenetlocal           LeNet-5 train / test / predict on MNIST idx files in one process (S/example/lenetLocal)
    mlpipeline           DLClassifier / DLEstimator DataFrame pipelines: LeNet, logistic regression, multi-label
                         linear regression (S/example/MLPipeline)
    imagetransferlearning  DataFrame image embeddings from a pre-trained net + DLClassifier
                         (S/example/dlframes/imageTransferLearning)
    keras                Keras-style LeNet: Sequential / compile / fit / evaluate / predict (S/example/keras)
    int8                 calibrated int8 scales (calcScales -> JSON) and int8 inference vs fp32
                         (S/example/mkldnn/int8/GenerateInt8Scales, ImageNetInference)
    seqfile              ImageNet / COCO Hadoop SequenceFile generators (S/models/utils/*SeqFileGenerator)
    perf                 ResNet-50 / VGG-16 / Inception training or fused-inference throughput (S/nn/mkldnn/Perf)

Every example runs on synthetic data when no data directory is given (no network access for datasets).
"""
import importlib
import sys

EXAMPLES = {
    "textclassification": "text_classifier",
    "languagemodel": "ptb_word_lm",
    "treelstm": "tree_lstm_sentiment",
    "loadmodel": "model_validator",
    "udfpredictor": "udf_predictor",
    "imagepredictor": "image_predictor",
    "tfloadandsave": "tf_load_and_save",
    "tftransferlearning": "tf_transfer_learning",
    "lenetlocal": "lenet_local",
    "mlpipeline": "ml_pipeline",
    "imagetransferlearning": "image_transfer_learning",
    "keras": "keras_lenet",
    "int8": "int8_inference",
    "seqfile": "seqfile_generator",
    "perf": "perf",
}


def get(name):
    return importlib.import_module(f"{__name__}.{EXAMPLES[name]}")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in EXAMPLES:
        print(__doc__)
        return 2
    return get(argv[0]).main(argv[1:])
