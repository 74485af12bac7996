"""Profile target: gram + potrf_inv at n (default 4096) a few times."""
import sys, time
import numpy as np
import torch
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import kernels

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda:0")
X = torch.as_tensor(np.random.default_rng(0).random((n, 8)), device=dev)
beta = torch.as_tensor(np.random.default_rng(3).uniform(0.5, 5, 8), device=dev)
for r in range(reps):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    ch = kernels.cholesky_inverse(kernels.gram(X, beta, 1.0, 1e-6))
    torch.cuda.synchronize(); print(f"rep {r}: {1e3*(time.perf_counter()-t0):.3f} ms", flush=True)
ch.check()
