"""Build libgpfit.so (HIP, gfx950) in-tree with hipcc.

The library is compiled straight from ``gladsgp_amd/csrc/*.hip`` into
``gladsgp_amd/libgpfit.so`` so it travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libgpfit.so")
SOURCES = ["gram.hip", "chol.hip", "predict.hip", "linalg.hip", "profile.hip", "blas.hip",
           "eig.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def _stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(PKG_DIR, "..", "include", "gpfit.h"))
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build_library(force: bool = False, verbose: bool = False) -> str:
    """Compile every HIP source for gfx950 into one shared library; return its path."""
    if not force and not _stale():
        return LIB_PATH
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    tmp = LIB_PATH + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-shared", "-fPIC",
           "-Wall", "-Wno-unused-function", "-o", tmp] + srcs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB_PATH)
    return LIB_PATH


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, verbose=True))
