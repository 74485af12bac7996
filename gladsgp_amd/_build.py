"""Build libgpfit.so (HIP, gfx950) in-tree with hipcc.

The library is compiled straight from ``gladsgp_amd/csrc/*.hip`` into
``gladsgp_amd/libgpfit.so`` so it travels with the repository snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_PATH = os.path.join(PKG_DIR, "libgpfit.so")
# Diagnostics variant (tools/dbg/pp_trace.py only, never loaded by the package): chol.hip with
# the persistent factorisation's timestamp trace compiled in (-DGPFIT_PP_TRACE).
TRACE_LIB_PATH = os.path.join(PKG_DIR, "libgpfit_trace.so")
SOURCES = ["gram.hip", "chol.hip", "predict.hip", "linalg.hip", "profile.hip", "blas.hip",
           "eig.hip", "comm.hip", "rng.hip", "mcmc.hip", "host_rng.hip", "field.hip"]
# Per-file extra flags.  chol.hip: MFMA accumulators in VGPRs (not AGPRs) so the update
# kernel, whose lookahead block calls the ~250-VGPR diagonal factor, keeps 2 waves/SIMD; and
# 16-byte LDS reads (ds_read_b128) for the factor's broadcast rows.
EXTRA = {"chol.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form",
                      "-Xclang", "-target-feature", "-Xclang", "+enable-ds128"]}
OBJ_DIR = os.path.join(PKG_DIR, "_obj")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
         "-Wno-unused-function"]


def _stale() -> bool:
    if not os.path.exists(LIB_PATH):
        return True
    t = os.path.getmtime(LIB_PATH)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(PKG_DIR, "..", "include", "gpfit.h"))
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build_library(force: bool = False, verbose: bool = False, trace: bool = False) -> str:
    """Compile every HIP source for gfx950 into one shared library; return its path.

    ``trace``: the diagnostics variant libgpfit_trace.so (chol.hip with -DGPFIT_PP_TRACE)."""
    out = TRACE_LIB_PATH if trace else LIB_PATH
    if not force and not trace and not _stale():
        return LIB_PATH
    os.makedirs(OBJ_DIR, exist_ok=True)

    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    headers.append(os.path.join(PKG_DIR, "..", "include", "gpfit.h"))
    t_hdr = max(os.path.getmtime(h) for h in headers if os.path.exists(h))

    def compile_one(src: str) -> str:
        tr = trace and src == "chol.hip"
        obj = os.path.join(OBJ_DIR, src.replace(".hip", "_trace.o" if tr else ".o"))
        if (not force and os.path.exists(obj) and
                os.path.getmtime(obj) > max(t_hdr, os.path.getmtime(os.path.join(CSRC, src)))):
            return obj                  # up to date: sources and headers older than the object
        cmd = ([HIPCC] + FLAGS + EXTRA.get(src, []) + (["-DGPFIT_PP_TRACE=1"] if tr else []) +
               ["-c", os.path.join(CSRC, src), "-o", obj])
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = out + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-ldl"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, out)
    return out


if __name__ == "__main__":
    print(build_library(force="--force" in sys.argv, verbose=True, trace="--trace" in sys.argv))
