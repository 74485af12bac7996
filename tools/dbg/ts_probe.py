"""Debug probe (not a test): what do the fit's ensemble-streaming products reach against plain
streaming reads of the same 5.5 GB on this box?  X = (512 x 1,347,945) fp64 rows padded to 128 B
(as emulator.standardize_y allocates y_std) and unpadded.  Times (median of 5, HIP events):
X.sum() (a read of X), gp_gemm_ex's tsk (X W: W fp64 column-major = the fit's Z, and W float32
row-major = the fit's Omega) and tsm (X^T Y, Q^T X).

    python tools/dbg/ts_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gladsgp_amd.blas import CM, gemm  # noqa: E402

dev = torch.device("cuda:0")
m, ny, r = 512, 1347945, 25
ld = (ny + 15) // 16 * 16
Xpad = torch.rand((m, ld), dtype=torch.float64, device=dev)[:, :ny]
GB = m * ny * 8 / 1e9


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts))


Wz = CM.empty(ny, r, dev)                               # the fit's Z: fp64 (ny x r), ld = ny
Wz.t.uniform_()
Om = CM.of_rowmajor(torch.rand((ny, r), device=dev, dtype=torch.float32))   # (r x ny), ld = r
Y = CM.empty(m, r, dev)
Y.t.uniform_()
rows = [("X.sum() (read X, padded)", t(lambda: Xpad.sum()))]
for name, X in (("padded", Xpad), ("unpadded", Xpad.contiguous())):
    Xc = CM.of_rowmajor(X)
    rows.append((f"tsk X Z      [{name}]", t(lambda: gemm(True, False, Xc, Wz))))
    rows.append((f"tsk X Omega  [{name}]", t(lambda: gemm(True, True, Xc, Om))))
    rows.append((f"tsm X^T Y    [{name}]", t(lambda: gemm(False, False, Xc, Y))))
    rows.append((f"tsm Q^T X^T  [{name}]", t(lambda: gemm(True, True, Y, Xc))))
    del Xc
for name, ms in rows:
    print(f"{name:28s} {ms:7.3f} ms  {GB / ms:6.2f} TB/s ({GB / ms / 8:.3f} of 8 TB/s)", flush=True)
