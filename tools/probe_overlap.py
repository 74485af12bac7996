"""Probe: how much does a concurrent TRMM (predict_solve on another stream) slow potrf_inv?
Decides whether TRMM row tiles can be overlapped with the factorisation."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import kernels  # noqa: E402

dev = torch.device("cuda:0")
n, m, d = 4096, 100000, 8
rng = np.random.default_rng(0)
X = torch.as_tensor(rng.random((n, d)), device=dev)
Xs = torch.as_tensor(np.random.default_rng(2).random((m, d)), device=dev)
beta = torch.as_tensor(np.random.default_rng(3).uniform(0.5, 5, d), device=dev).reshape(1, d)
w = torch.as_tensor(rng.standard_normal(n), device=dev)
G0 = kernels.gram(X, beta, 1.0, 1e-6)
ch = kernels.cholesky_inverse(G0.clone())
prep = kernels.predict_prepare(X, Xs, beta, 1.0)
torch.cuda.synchronize()


def timed_potrf(stream):
    G = G0.clone()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(stream):
        e0.record(stream)
        kernels.cholesky_inverse(G)
        e1.record(stream)
    return e0, e1


for label, pa, pb in (("alone", None, None), ("equal prio", 0, 0), ("potrf high prio", -1, 0)):
    res = []
    for rep in range(4):
        if pa is None:
            sa = torch.cuda.Stream(device=dev)
            e0, e1 = timed_potrf(sa)
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1))
            continue
        sa = torch.cuda.Stream(device=dev, priority=pa)
        sb = torch.cuda.Stream(device=dev, priority=pb)
        torch.cuda.synchronize()
        with torch.cuda.stream(sb):
            f0 = torch.cuda.Event(enable_timing=True)
            f1 = torch.cuda.Event(enable_timing=True)
            f0.record(sb)
            kernels.predict_solve(ch, prep, 1.0, w)
            f1.record(sb)
        e0, e1 = timed_potrf(sa)
        torch.cuda.synchronize()
        res.append((e0.elapsed_time(e1), f0.elapsed_time(f1)))
    print(label, res[1:])
