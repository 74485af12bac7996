"""Time gp_gram_ardse (full n x n Gram, d = 8) over n with HIP events: mean us per launch and
the HBM rate of its 8 n^2 B of stores.

    python tools/prof_gram.py [n ...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import kernels  # noqa: E402

dev = torch.device("cuda:0")
for n in [int(a) for a in sys.argv[1:]] or [1024, 2048, 4096, 8192]:
    X = torch.as_tensor(np.random.default_rng(0).random((n, 8)), device=dev)
    beta = torch.as_tensor(np.random.default_rng(3).uniform(0.5, 5, 8), device=dev)
    for _ in range(3):
        G = kernels.gram(X, beta, 1.0, 1e-6)
    reps = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        G = kernels.gram(X, beta, 1.0, 1e-6)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print(f"n={n:5d} full Gram {us:8.2f} us/launch  {8.0 * n * n / us / 1e3:7.1f} GB/s "
          f"(incl. the empty-tensor allocation per call)", flush=True)
