"""Reference ``bigdl.models`` package (P/models): model-zoo helpers."""
