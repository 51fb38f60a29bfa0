"""bigdl_amd.transform.vision.image (reference S/transform/vision/image/**)."""
from .augmentation import *  # noqa: F401,F403
from .feature import *  # noqa: F401,F403
