"""Debug probe (not a test): what do the fit's ensemble-streaming products reach against plain
streaming reads of the same 5.5 GB on this box?  X = (512 x 1,347,945) fp64 C-order, W =
(1,347,945 x 25).  Times (median of 5, HIP events): torch X.sum() (a read of X), torch X @ W
(hipBLAS dgemm), gp_gemm_ex's tsk (X W) and tsm (X^T Y, Y 512 x 25).

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
X = torch.rand((m, ny), dtype=torch.float64, device=dev)
W = torch.rand((ny, r), dtype=torch.float64, device=dev)
Y = torch.rand((m, r), dtype=torch.float64, device=dev)
GB = X.numel() * 8 / 1e9


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


Xc = CM.of_rowmajor(X)                 # (ny x m), ld = ny
Wt = W.t().contiguous()                # (25 x ny) C-order = column-major (ny x 25), ld = ny
Wc = CM(Wt, ny, r, ny)
Yt = Y.t().contiguous()
Yc = CM(Yt, m, r, m)
rows = []
rows.append(("X.sum() (read X)", t(lambda: X.sum())))
rows.append(("torch X @ W (hipBLAS)", t(lambda: X @ W)))
rows.append(("gp tsk X W  (gemm(1,0))", t(lambda: gemm(True, False, Xc, Wc))))
rows.append(("gp tsm X^T Y (gemm(0,0))", t(lambda: gemm(False, False, Xc, Yc))))
for name, ms in rows:
    print(f"{name:28s} {ms:7.3f} ms  {GB / ms:6.2f} TB/s ({GB / ms / 8:.3f} of 8 TB/s)", flush=True)
