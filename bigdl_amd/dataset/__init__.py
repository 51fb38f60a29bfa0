"""bigdl_amd.dataset — datasets, samples, mini-batches and transformers (reference S/dataset/**)."""
from .core import *  # noqa: F401,F403
from .image import *  # noqa: F401,F403
from .mnist_cifar import load_cifar_test, load_cifar_train, load_mnist  # noqa: F401
from .text import (Dictionary, LabeledSentence, LabeledSentenceToSample, SentenceBiPadding,  # noqa: F401
                   SentenceSplitter, SentenceTokenizer, TextToLabeledSentence)
