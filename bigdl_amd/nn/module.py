"""``Module`` loaders / helpers (reference S/nn/Module.scala:32-166: load, loadModule, loadTorch, loadCaffe,
loadCaffeModel, loadTF, tensorflowCheckpoints, flatten :113-141, isCompact :143-166)."""
import torch


class Module:
    @staticmethod
    def loadModule(path, weightPath=None):
        from ..utils.serializer import load_module

        return load_module(path, weightPath)

    load = loadModule

    @staticmethod
    def loadTorch(path):
        from ..interop.torchfile import load_torch

        return load_torch(path)

    @staticmethod
    def loadCaffe(model, defPath, modelPath, matchAll=True, customizedConverters=None):
        from ..interop.caffe import load_caffe_into

        return load_caffe_into(model, defPath, modelPath, matchAll, customizedConverters)

    @staticmethod
    def loadCaffeModel(defPath, modelPath, customizedConverters=None):
        from ..interop.caffe import load_caffe

        return load_caffe(defPath, modelPath, customizedConverters)[0]

    @staticmethod
    def loadTF(path, inputs, outputs, byteOrder=None, binFile=None, generatedBackward=True):
        from ..interop.tensorflow import load_tf

        return load_tf(path, inputs, outputs, byteOrder, binFile, generatedBackward)

    @staticmethod
    def tensorflowCheckpoints(graphFile, binFile, byteOrder=None):
        """A TensorFlow Session whose variables come from ``binFile`` (reference Module.scala:108)."""
        from ..interop.tensorflow import TensorflowLoader

        return TensorflowLoader.checkpoints(graphFile, binFile, byteOrder)

    @staticmethod
    def loadONNX(path):
        from ..interop.onnx import load_onnx

        return load_onnx(path)

    @staticmethod
    def flatten(parameters):
        """Compact a list of tensors into one storage; returns the flat tensor (views rebound in place)."""
        total = sum(p.numel() for p in parameters)
        dev = parameters[0].device if parameters else "cpu"
        flat = torch.zeros(total, dtype=torch.float32, device=dev)
        off = 0
        for p in parameters:
            n = p.numel()
            flat[off:off + n].copy_(p.reshape(-1))
            p.data = flat[off:off + n].view(p.shape)
            off += n
        return flat

    @staticmethod
    def isCompact(parameters):
        if not parameters:
            return True
        st = parameters[0].untyped_storage().data_ptr()
        if any(p.untyped_storage().data_ptr() != st for p in parameters):
            return False
        off = parameters[0].storage_offset()
        for p in parameters:
            if p.storage_offset() != off:
                return False
            off += p.numel()
        return True
