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
}


def get(name):
    return importlib.import_module(f"{__name__}.{EXAMPLES[name]}")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in EXAMPLES:
        print(__doc__)
        return 2
    return get(argv[0]).main(argv[1:])
