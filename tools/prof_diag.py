"""Profile target: potrf_inv at small n (n=64 -> only the diag kernel runs)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import kernels
dev = torch.device("cuda:0")
for n in (64, 128):
    X = torch.as_tensor(np.random.default_rng(0).random((n, 8)), device=dev)
    beta = torch.as_tensor(np.random.default_rng(3).uniform(0.5, 5, 8), device=dev)
    G = kernels.gram(X, beta, 1.0, 1e-6)
    for r in range(50):
        ch = kernels.cholesky_inverse(G.clone())
    torch.cuda.synchronize()
    ch.check()
print("done")
