"""bigdl_amd.models — model zoo (reference S/models/**)."""
from .autoencoder import Autoencoder, AutoencoderGraph  # noqa: F401
from .inception import (Inception_Layer_v1, Inception_Layer_v2, Inception_v1, Inception_v1_NoAuxClassifier,  # noqa: F401
                        Inception_v1_NoAuxClassifierGraph, Inception_v2, Inception_v2_NoAuxClassifier)
from .lenet import LeNet5, LeNet5Graph  # noqa: F401
from .resnet import ResNet, ResNet50, ResNetGraph  # noqa: F401
from .rnn import PTBModel, SimpleRNN  # noqa: F401
from .vgg import Vgg_16, Vgg_16Graph, Vgg_19, Vgg_19Graph, VggForCifar10, VggForCifar10Graph  # noqa: F401
from .maskrcnn import MaskRCNN, MaskRCNNParams  # noqa: F401
