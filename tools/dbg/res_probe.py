"""Probe for the prediction kernels at the C5 shape (64 GPs, n = 512, d = 8): gp_predict over
m test points, 3 calls (tools/pmc_res.sh runs it under rocprofv3 counter passes)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from gladsgp_amd import kernels  # noqa: E402

m = int(os.environ.get("RES_PROBE_M", "32768"))
n, B, d = 512, 64, 8
dev = torch.device("cuda:0")
rng = np.random.default_rng(3)
t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
X, Xs = t(rng.random((n, d))), t(rng.random((m, d)))
beta = t(rng.uniform(0.5, 5.0, (B, d)))
s, delta = t(rng.uniform(0.8, 1.5, B)), t(np.full(B, 1e-6))
W = t(rng.standard_normal((B, n)))
ch = kernels.cholesky_inverse(kernels.gram(X, beta, s, delta, batch=B))
ch.check()
for _ in range(3):
    mu, var = kernels.predict(ch, X, Xs, beta, s, s, W)
torch.cuda.synchronize()
print("ok", float(mu.abs().max()), float(var.min()))
