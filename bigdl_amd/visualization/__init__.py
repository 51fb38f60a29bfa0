"""bigdl_amd.visualization — TensorBoard summaries (reference S/visualization/**)."""
from .summary import Summary, TrainSummary, ValidationSummary  # noqa: F401
from .tensorboard import FileReader, FileWriter, crc32c, masked_crc32c  # noqa: F401
