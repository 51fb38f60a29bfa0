"""Reference ``bigdl.version`` (P/version.py): the API level this facade follows."""
__version__ = "0.10.0"
