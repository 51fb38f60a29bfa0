"""bigdl_amd.transform.vision.image (reference S/transform/vision/image/**)."""
from .augmentation import *  # noqa: F401,F403
from .feature import *  # noqa: F401,F403
from .roi import (BoundingBox, RandomSampler, RoiHFlip, RoiLabel, RoiNormalize, RoiProject,  # noqa: F401
                  RoiResize)


class SeqFileFolder:
    """Hadoop SequenceFiles of labelled BGR images as an ImageFrame (reference P/transform/vision/image.py
    SeqFileFolder.files_to_image_frame, S/dataset/DataSet.scala SeqFileFolder.filesToImageFrame): each record's
    key holds the label (or "name\nlabel"), its value the width / height header and the BGR pixels; features with
    a label above ``class_num`` are dropped, as in the reference."""

    @staticmethod
    def files_to_image_frame(url, class_num, partition_num=-1):
        import glob
        import os
        import struct

        import torch

        from ....dataset.seqfile import read_label, read_sequence_file
        from .feature import ImageFeature, LocalImageFrame

        feats = []
        for path in sorted(glob.glob(os.path.join(url, "*.seq"))):
            for key, value in read_sequence_file(path):
                label = float(read_label(key))
                if label > class_num:
                    continue
                w, h = struct.unpack_from(">ii", value, 0)
                f = ImageFeature(bytes=bytes(value[8:8 + w * h * 3]), label=torch.tensor([label]))
                f[ImageFeature.originalSize] = (h, w, 3)
                feats.append(f)
        return LocalImageFrame(feats)
