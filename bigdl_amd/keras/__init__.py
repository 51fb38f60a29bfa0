"""Keras-1.2.2-style API (reference S/nn/keras/*, P/nn/keras/*): layers with shape inference, Sequential and
functional Model with compile / fit / evaluate / predict."""
from .engine import (Input, InputLayer, KerasIdentityWrapper, KerasLayer, KerasLayerWrapper, KerasModel,  # noqa: F401
                     Model, Sequential)
from .layers import *  # noqa: F401,F403
