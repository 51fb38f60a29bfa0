"""Reference ``bigdl.util.tf_utils`` (P/util/tf_utils.py). The functions that drive a live TensorFlow session
(``get_path``, ``convert``, ``export_checkpoint``, ``dump_model`` with ``sess``) need the ``tensorflow`` package,
which is not installed here: they raise ImportError with that reason. ``save_variable_bigdl`` and
``merge_checkpoint`` work on their own: variables are written in the engine's checkpoint format (safetensors,
read back by ``TensorflowLoader.checkpoints`` / ``Module.loadTF(..., binFile)``)."""
import os

import numpy as np
import torch


def _need_tf(what):
    try:
        import tensorflow  # noqa: F401
    except ImportError as e:
        raise ImportError(f"{what} needs the tensorflow package, which is not available in this environment") from e
    raise NotImplementedError(f"{what}: exporting from a live TensorFlow session is not supported; save the "
                              "GraphDef and use save_variable_bigdl for the variables")


def get_path(output_name, sess=None):
    _need_tf("get_path")


def convert(input_ops, output_ops, byte_order, bigdl_type):
    _need_tf("convert")


def export_checkpoint(checkpoint_path):
    _need_tf("export_checkpoint")


def dump_model(path, graph=None, sess=None, ckpt_file=None, bigdl_type="float"):
    _need_tf("dump_model")


def save_variable_bigdl(tensors, target_path, bigdl_type="float"):
    """{variable name: ndarray} -> a variable file ``Module.loadTF(..., binFile=target_path)`` reads."""
    from ...interop.tf_session import save_bin

    out = {}
    for name, v in tensors.items():
        if not isinstance(v, np.ndarray):
            raise TypeError(f"{name}: only numpy ndarrays can be saved (got {type(v).__name__})")
        out[name] = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32))
    save_bin(target_path, out)


def merge_checkpoint(input_graph, checkpoint, output_node_names, output_graph, sess=None):
    """Freeze ``input_graph`` (GraphDef file) with the variables of ``checkpoint`` (a save_variable_bigdl file):
    every VariableV2 / Variable node whose value is in the checkpoint becomes a Const, and the graph is cut to the
    ancestors of ``output_node_names``; written as binary GraphDef to ``output_graph``."""
    from ...interop.tensorflow import freeze_graph_with_variables
    from ...interop.tf_session import load_bin

    values = {k: v.numpy() for k, v in load_bin(checkpoint).items()}
    freeze_graph_with_variables(input_graph, values, output_node_names, output_graph)


__all__ = ["get_path", "convert", "export_checkpoint", "dump_model", "save_variable_bigdl", "merge_checkpoint"]
