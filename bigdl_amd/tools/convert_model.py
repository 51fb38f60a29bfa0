"""Model format converter (reference S/utils/ConvertModel.scala:25-133).

    python -m bigdl_amd.tools.convert_model --from caffe --to bigdl --prototxt net.prototxt \
        --input net.caffemodel --output net.bigdl [--quantize true]

--from  bigdl | caffe | torch | tensorflow | onnx | keras
--to    bigdl | caffe | torch | tensorflow | onnx
TensorFlow input needs --tf_inputs / --tf_outputs (comma-separated node names); Keras input is a JSON definition
(--input) plus an optional HDF5 weight file (--prototxt is reused as the weight path, like the reference reuses
it for Caffe). --quantize converts the loaded model to its int8 inference form before saving.
"""
import argparse
import sys


def load(fmt, inp, prototxt=None, tf_inputs=None, tf_outputs=None):
    from ..nn.module import Module

    if fmt == "bigdl":
        return Module.loadModule(inp)
    if fmt == "caffe":
        if not prototxt:
            raise SystemExit("--prototxt is required for --from caffe")
        return Module.loadCaffeModel(prototxt, inp)
    if fmt == "torch":
        return Module.loadTorch(inp)
    if fmt == "tensorflow":
        if not tf_inputs or not tf_outputs:
            raise SystemExit("--tf_inputs and --tf_outputs are required for --from tensorflow")
        return Module.loadTF(inp, tf_inputs.split(","), tf_outputs.split(","))
    if fmt == "onnx":
        return Module.loadONNX(inp)
    if fmt == "keras":
        from ..keras.converter import load_keras

        return load_keras(json_path=inp, hdf5_path=prototxt)
    raise SystemExit(f"unsupported source format {fmt}")


def save(model, fmt, out, overwrite=True, input_shape=None):
    if fmt == "bigdl":
        model.saveModule(out, overWrite=overwrite)
    elif fmt == "caffe":
        base = out[:-len(".caffemodel")] if out.endswith(".caffemodel") else out
        model.saveCaffe(base + ".prototxt", base + ".caffemodel", overwrite=overwrite)
    elif fmt == "torch":
        model.saveTorch(out, overWrite=overwrite)
    elif fmt == "onnx":
        from ..interop.onnx import save_onnx

        if not input_shape:
            raise SystemExit("--input_shape (e.g. 1,3,224,224) is required for --to onnx / tensorflow")
        save_onnx(model, input_shape, out)
    elif fmt == "tensorflow":
        if not input_shape:
            raise SystemExit("--input_shape (e.g. 1,3,224,224) is required for --to onnx / tensorflow")
        model.saveTF([("input", list(input_shape))], out)
    else:
        raise SystemExit(f"unsupported target format {fmt}")


def main(argv=None):
    ap = argparse.ArgumentParser(prog="convert_model", description=__doc__.split("\n")[0])
    ap.add_argument("--from", dest="src", required=True,
                    choices=["bigdl", "caffe", "torch", "tensorflow", "onnx", "keras"])
    ap.add_argument("--to", dest="dst", required=True, choices=["bigdl", "caffe", "torch", "tensorflow", "onnx"])
    ap.add_argument("--input", required=True)
    ap.add_argument("--output", required=True)
    ap.add_argument("--prototxt", default=None)
    ap.add_argument("--quantize", default="false")
    ap.add_argument("--tf_inputs", default=None)
    ap.add_argument("--tf_outputs", default=None)
    ap.add_argument("--input_shape", default=None, help="comma-separated shape for ONNX / TF export")
    a = ap.parse_args(argv)
    model = load(a.src, a.input, a.prototxt, a.tf_inputs, a.tf_outputs)
    if str(a.quantize).lower() in ("true", "1", "yes"):
        model = model.quantize()
    shape = [int(v) for v in a.input_shape.split(",")] if a.input_shape else None
    save(model, a.dst, a.output, input_shape=shape)
    print(f"converted {a.src}:{a.input} -> {a.dst}:{a.output}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
