"""Reference ``bigdl.contrib`` (P/contrib)."""
