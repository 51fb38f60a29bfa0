"""bigdl_amd.interop — model import/export: Caffe, Torch7, TensorFlow, ONNX, Keras (reference S/utils/caffe,
S/utils/TorchFile.scala, S/utils/tf, P/contrib/onnx, P/keras)."""
