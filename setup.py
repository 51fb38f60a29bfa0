"""Build the bigdl_amd native extension in-tree for gfx950 (MI355X).

    python setup.py build_ext --inplace

1. every ``csrc/*.hip`` kernel file is compiled directly by ``hipcc --offload-arch=gfx950`` (no hipify
   pass, no CUDA sources: these are CDNA4 kernels written for HIP);
2. ``csrc/bindings.cpp`` (the only TU that includes torch headers) is compiled as a plain C++ torch
   extension and linked with those objects and libamdhip64 into ``bigdl_amd/_C.*.so``.

``__graft_entry__.build()`` runs this.
"""
import glob
import hashlib
import json
import os
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

from setuptools import setup
from torch.utils.cpp_extension import BuildExtension, CppExtension

HERE = os.path.dirname(os.path.abspath(__file__))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("BIGDL_AMD_ARCH", "gfx950")
OBJ_DIR = os.path.join(HERE, "build", "hipobj")
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fno-gpu-rdc",
             "-I" + os.path.join(HERE, "csrc"), "-Wno-unused-result"]


def _load_buildhash():
    import importlib.util

    spec = importlib.util.spec_from_file_location("_bigdl_buildhash", os.path.join(HERE, "bigdl_amd", "_buildhash.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


_BH = _load_buildhash()
_digest = _BH.digest


def source_digest():
    """Content hash of every native source and header plus the compile flags: what bigdl_amd/_build_info.json
    records and bigdl_amd.ops.native compares at import (stale-build check)."""
    return _BH.source_digest(HERE, HIP_FLAGS)


def _compile_one(src):
    # rebuilt unless the recorded content hash of (source, every header, flags) matches: an object is never reused
    # on timestamps alone (a stale build/hipobj from another tree or checkout would otherwise be linked unnoticed)
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
    want = _digest([src] + glob.glob(os.path.join(HERE, "csrc", "*.h")), " ".join(HIP_FLAGS))
    stamp = obj + ".sha256"
    if os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == want:
                return obj
    cmd = [HIPCC] + HIP_FLAGS + ["-c", src, "-o", obj]
    print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    with open(stamp, "w") as f:
        f.write(want)
    return obj


def compile_hip_objects():
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(HERE, "csrc", "*.hip")))
    jobs = int(os.environ.get("MAX_JOBS", "8"))
    with ThreadPoolExecutor(max_workers=max(1, min(jobs, 16))) as ex:
        return list(ex.map(_compile_one, srcs))


class HipBuildExt(BuildExtension):
    def build_extensions(self):
        objs = compile_hip_objects()
        for ext in self.extensions:
            ext.extra_objects = list(ext.extra_objects or []) + objs
        super().build_extensions()
        info = {"source_sha256": source_digest(), "arch": ARCH, "hip_flags": HIP_FLAGS,
                "objects": {os.path.basename(o): open(o + ".sha256").read().strip() for o in objs},
                "built_unix": int(time.time()), "mode": "setup.py build_ext"}
        with open(os.path.join(HERE, "bigdl_amd", "_build_info.json"), "w") as f:
            json.dump(info, f, indent=1)


ext = CppExtension(
    name="bigdl_amd._C",
    sources=[os.path.join("csrc", "bindings.cpp"), os.path.join("csrc", "host_runtime.cpp")],
    include_dirs=[os.path.join(HERE, "csrc"), os.path.join(ROCM, "include")],
    define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
    extra_compile_args=["-O3", "-std=c++17"],
    library_dirs=[os.path.join(ROCM, "lib")],
    libraries=["amdhip64"],
    extra_link_args=["-Wl,-rpath," + os.path.join(ROCM, "lib")],
)

if __name__ == "__main__":
    if len(sys.argv) == 1:
        sys.argv += ["build_ext", "--inplace"]
    setup(
        name="bigdl_amd",
        version="0.1.0",
        packages=["bigdl_amd"],
        ext_modules=[ext],
        cmdclass={"build_ext": HipBuildExt.with_options(use_ninja=True)},
    )
