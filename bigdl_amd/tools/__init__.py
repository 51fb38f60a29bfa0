"""Command-line tools (python -m bigdl_amd.tools.<name>)."""
