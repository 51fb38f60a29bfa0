"""``bigdl.dataset.transformer`` (reference P/dataset/transformer.py)."""
from ..util.common import Sample  # noqa: F401


def normalizer(data, mean, std):
    """Normalize features by standard deviation; data is an ndarray."""
    return (data - mean) / std


__all__ = ["normalizer", "Sample"]
