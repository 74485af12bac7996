"""Where the fit's PCA seconds go (the `PCA (seconds)` column of timing.csv, src/model.py:206-214:
init_model = data upload + standardisation + randomized_svd + the .npy cache round trip).

Runs init_model at the fit workload's configuration (n = 512 runs, ny = 1,347,945 nodes,
float32 ensemble as fit_models loads it, r = 25 test vectors, q = 1) with every phase wrapped
in a host timer bracketed by torch.cuda.synchronize(), and times each gp_dgemm call that streams
the ensemble with HIP events (achieved GB/s against 8 TB/s: bytes = the X operand read once +
the small operands).  Prints one line per phase and a JSON summary.

    python tools/prof_pca.py [ny] [n] [--cold]

--cold skips the small warm-up run, so first-use costs (HIP context, code-object loads, the
caching allocator's first growth) land in the phases, as they do in bench.py --workload fit.
"""
import json
import os
import shutil
import sys
import tempfile
import time
from collections import defaultdict

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gladsgp_amd import blas, emulator, model as gmodel, svd as gsvd  # noqa: E402

cold = "--cold" in sys.argv
argv = [a for a in sys.argv[1:] if a != "--cold"]
ny = int(argv[0]) if len(argv) > 0 else 1347945
n = int(argv[1]) if len(argv) > 1 else 512
dev = torch.device("cuda", 0)
phases = defaultdict(float)
gemms = []


def timed(name, fn):
    def w(*a, **k):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn(*a, **k)
        torch.cuda.synchronize()
        phases[name] += time.perf_counter() - t0
        return r
    return w


_gemm = blas.gemm


def gemm_ev(transa, transb, A, B, alpha=1.0, beta=0.0, C=None):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    out = _gemm(transa, transb, A, B, alpha, beta, C)
    e1.record()
    torch.cuda.synchronize()
    m = A.cols if transa else A.rows
    k = A.rows if transa else A.cols
    nn = B.rows if transb else B.cols
    gemms.append({"op": f"gemm({int(transa)},{int(transb)}) {m}x{nn}x{k}",
                  "ms": e0.elapsed_time(e1),
                  # operand bytes as stored: gp_gemm_ex reads float32 operands as float32
                  "bytes": (4.0 if A.f32 else 8.0) * m * k + (4.0 if B.f32 else 8.0) * k * nn
                  + 8.0 * m * nn})
    return out


# phase wrappers (module attributes the package calls through)
emulator.SimData.__init__ = timed("upload (H2D + widen to fp64)", emulator.SimData.__init__)
emulator.EmulatorData.standardize_y = timed("standardise (gp_sim_stats + gp_standardize)",
                                            emulator.EmulatorData.standardize_y)
gsvd._legacy_normal_from = timed("Omega draw (svd.LegacyNormalDraw, host thread)",
                                 gsvd._legacy_normal_from)
gsvd.gemm = gemm_ev
gsvd.orthonormalize = timed("CholeskyQR3 (orthonormalize)", gsvd.orthonormalize)
gsvd.syevj = timed("Jacobi eig of B B^T (gp_syevj)", gsvd.syevj)
gmodel.randomized_svd = timed("randomized_svd total", gsvd.randomized_svd)
_save, _load = np.save, np.load
np.save = timed("np.save of U, S, Vh (cache)", _save)
np.load = timed("np.load of S, Vh (cache)", _load)

rng = np.random.default_rng(0)
t = rng.random((n, 8))
nm = 12
modes = (rng.standard_normal((nm, ny)) * (0.6 ** np.arange(nm))[:, None]).astype(np.float32)
coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, 8) + k) for k in range(nm)], 1)
Y = coef.astype(np.float32) @ modes
Y += 1e-3 * rng.standard_normal(Y.shape, dtype=np.float32)
tmp = tempfile.mkdtemp(prefix="gladsgp_pca_")
try:
    np.random.seed(0)
    # warm-up at a small size (first-call HIP / library costs out of the timed run)
    if not cold:
        gmodel.init_model(t[:64], Y[:64, :4096], "warm", 8, data_dir=tmp, device=dev,
                          recompute=True, verbose=False)
    phases.clear()
    gemms.clear()
    np.random.seed(0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gmodel.init_model(t.astype(np.float32), Y, "pca", 8, data_dir=tmp, device=dev,
                      recompute=True, verbose=False)
    torch.cuda.synchronize()
    total = time.perf_counter() - t0
finally:
    shutil.rmtree(tmp, ignore_errors=True)
    np.save, np.load = _save, _load

print(f"init_model (timing.csv PCA column) n={n} ny={ny}: {total:.3f} s")
acc = 0.0
for k, v in sorted(phases.items(), key=lambda kv: -kv[1]):
    print(f"  {k:48s} {v * 1e3:9.1f} ms")
g_ms = sum(g["ms"] for g in gemms)
print(f"  gp_dgemm calls inside randomized_svd: {len(gemms)}, {g_ms:.1f} ms in all")
for g in gemms:
    gbs = g["bytes"] / (g["ms"] * 1e-3) / 1e9
    print(f"    {g['op']:34s} {g['ms']:8.3f} ms  {g['bytes'] / 1e9:7.3f} GB  {gbs:8.1f} GB/s "
          f"({gbs / 8000:.3f} of 8 TB/s)")
print(json.dumps({"total_s": total, "phases_ms": {k: v * 1e3 for k, v in phases.items()},
                  "gemms": gemms}))
