"""Profile target: gram + potrf_inv at n (default 4096), `batch` problems, a few times.

    python tools/prof_potrf.py [n] [reps] [batch]

GPFIT_POTRF_SWEEP=1 in the environment: this tool sets gp_set_potrf_path(1) (the blocked sweep).
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import _capi, kernels  # noqa: E402

if os.environ.get("GPFIT_POTRF_SWEEP") == "1":
    _capi.lib().gp_set_potrf_path(1)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
batch = int(sys.argv[3]) if len(sys.argv) > 3 else 1
dev = torch.device("cuda:0")
X = torch.as_tensor(np.random.default_rng(0).random((n, 8)), device=dev)
beta = torch.as_tensor(np.stack([np.random.default_rng(10 + j).uniform(0.5, 5, 8)
                                 for j in range(batch)]), device=dev)
ones = torch.ones(batch, dtype=torch.float64, device=dev)
ts = []
for r in range(reps):
    G = kernels.gram(X, beta, ones, 1e-6 * ones, batch=batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ch = kernels.cholesky_inverse(G)
    torch.cuda.synchronize()
    ts.append(1e3 * (time.perf_counter() - t0))
    print(f"rep {r}: potrf_inv {ts[-1]:.3f} ms", flush=True)
ch.check()
print(f"n={n} batch={batch} min {min(ts):.3f} ms median {sorted(ts)[len(ts) // 2]:.3f} ms")
