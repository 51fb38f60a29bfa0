"""Log routing (reference S/utils/LoggerFilter.scala:36-140): framework INFO logs to the console, third-party
INFO logs to a file (``bigdl.log`` in the working directory by default) so training output stays readable.

Controlled by the same switches as the reference's JVM properties, read from the environment:
BIGDL_LOGGERFILTER_DISABLE=true, BIGDL_LOGGERFILTER_LOGFILE=<path>, BIGDL_LOGGERFILTER_ENABLE_THIRDPARTY=false.
"""
import logging
import os

PATTERN = "%(asctime)s %(levelname)-5s %(name)s:%(lineno)d - %(message)s"
DATEFMT = "%Y-%m-%d %H:%M:%S"
THIRD_PARTY = ("torch", "urllib3", "matplotlib", "PIL", "filelock", "fsspec", "asyncio")


def _handler(h, level):
    h.setLevel(level)
    h.setFormatter(logging.Formatter(PATTERN, DATEFMT))
    return h


def redirectSparkInfoLogs(logPath=None):
    """Install the routing once; returns the log file path (or None when disabled)."""
    if os.environ.get("BIGDL_LOGGERFILTER_DISABLE", "false").lower() == "true":
        return None
    path = os.environ.get("BIGDL_LOGGERFILTER_LOGFILE", logPath or os.path.join(os.getcwd(), "bigdl.log"))
    if os.path.isdir(path):
        path = os.path.join(path, "bigdl.log")
    fh = _handler(logging.FileHandler(path), logging.INFO)
    enable = os.environ.get("BIGDL_LOGGERFILTER_ENABLE_THIRDPARTY", "true").lower() == "true"
    for name in THIRD_PARTY:
        lg = logging.getLogger(name)
        lg.handlers = [fh] if enable else []
        lg.setLevel(logging.INFO if enable else logging.ERROR)
        lg.propagate = False
    own = logging.getLogger("bigdl_amd")
    if not any(getattr(h, "_bigdl", False) for h in own.handlers):
        ch = _handler(logging.StreamHandler(), logging.INFO)
        ch._bigdl = True
        own.addHandler(ch)
        fh2 = _handler(logging.FileHandler(path), logging.INFO)
        fh2._bigdl = True
        own.addHandler(fh2)
    own.setLevel(logging.INFO)
    return path


__all__ = ["redirectSparkInfoLogs"]
