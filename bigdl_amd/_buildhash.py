"""Content hash of the native sources (csrc/*.hip, *.h, *.cpp) plus the compile flags. setup.py records it in
bigdl_amd/_build_info.json when it links bigdl_amd/_C; bigdl_amd.ops.native recomputes it at import and flags a
stale extension. Dependency-free on purpose (setup.py loads this file directly)."""
import glob
import hashlib
import os


def digest(paths, extra=""):
    h = hashlib.sha256(extra.encode())
    for p in sorted(paths):
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def source_digest(root, flags):
    csrc = os.path.join(root, "csrc")
    srcs = [p for ext in ("*.hip", "*.h", "*.cpp") for p in glob.glob(os.path.join(csrc, ext))]
    return digest(srcs, " ".join(flags))
