"""HDF5 access for Keras weight files. The h5py package is not available in this environment; a native reader is
not implemented yet, so Keras weights must be passed as {layer_name: [arrays]} (see keras.converter)."""


def read_keras_weights(path):
    try:
        import h5py  # noqa: F401
    except ImportError as e:
        raise NotImplementedError("reading Keras HDF5 weight files needs h5py, which is not installed; pass the "
                                  "weights as a {layer_name: [numpy arrays]} dict instead") from e
    import h5py
    out = {}
    with h5py.File(path, "r") as f:
        g = f["model_weights"] if "model_weights" in f else f
        for name in [n.decode() if isinstance(n, bytes) else n for n in g.attrs["layer_names"]]:
            lg = g[name]
            wn = [n.decode() if isinstance(n, bytes) else n for n in lg.attrs["weight_names"]]
            out[name] = [lg[w][()] for w in wn]
    return out
