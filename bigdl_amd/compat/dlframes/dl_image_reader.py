"""Reference ``bigdl.dlframes.dl_image_reader`` (P/dlframes/dl_image_reader.py)."""
from ... import dlframes as _d


class DLImageReader:
    @staticmethod
    def readImages(path, sc=None, minParitions=1, bigdl_type="float"):
        return _d.DLImageReader.readImages(path, minParitions)


__all__ = ["DLImageReader"]
