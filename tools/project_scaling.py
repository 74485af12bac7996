"""Projection (not a measurement) of the C3 strong-scaling step at N = 2, 4, 8 from one GPU:
the per-rank work of `bench.py --gpus N` (sharded.PipelinedPredictor with the split
sharded.calibrate_split picks) timed rank by rank on this GPU -- rank 0 factorises the next
GP (Gram + gp_potrf_inv) and predicts its c0 points, every other rank predicts its c1 points --
and the step taken as the slower of the two.  Not included: the L^-1 broadcast (67 MB over
xGMI, asynchronous, overlapped with the prediction), the (mean, var) gather (2 x 8 B per point)
and clock differences between GPUs.

    python tools/project_scaling.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import kernels  # noqa: E402
from gladsgp_amd.sharded import balanced_split  # noqa: E402

dev = torch.device("cuda:0")
n, m, d = 4096, 100000, 8
rng = np.random.default_rng(0)
X = torch.as_tensor(rng.random((n, d)), device=dev)
Xs = torch.as_tensor(rng.random((m, d)), device=dev)
beta = torch.as_tensor(rng.uniform(0.5, 5, (1, d)), device=dev)
w = torch.as_tensor(np.sin(rng.random(n) * 6), device=dev).reshape(1, n)
s, delta = 1.0, 1e-6
ws = kernels.PredictWorkspace()


def med(fn, reps=5):
    fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize(dev)
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[reps // 2]


ch = kernels.cholesky_inverse(kernels.gram(X, beta, s, delta))
t_fact = med(lambda: kernels.cholesky_inverse(kernels.gram(X, beta, s, delta)))
cache = {}


def T(p):
    if p <= 0:
        return 0.0
    if p not in cache:
        Xc = Xs[:p].contiguous()
        cache[p] = med(lambda: kernels.predict(ch, X, Xc, beta, s, s, w, workspace=ws), reps=3)
    return cache[p]


t1 = t_fact + T(m)
print(f"one GPU: factorisation {t_fact * 1e3:.3f} ms + prediction of {m} points "
      f"{T(m) * 1e3:.3f} ms = {t1 * 1e3:.3f} ms per GP ({m / t1 / 1e6:.3f} M pred/s, serial "
      "head; the bench's N = 1 step overlaps the cross-covariance with the factorisation)",
      flush=True)
for N in (2, 4, 8):
    counts = balanced_split(m, N, t_fact, T)
    r0 = t_fact + T(counts[0])
    rr = max(T(c) for c in counts[1:])
    step = max(r0, rr)
    print(f"N={N}: counts rank0 {counts[0]} / others {max(counts[1:])}; rank 0 {r0 * 1e3:.3f} ms, "
          f"others {rr * 1e3:.3f} ms -> projected step {step * 1e3:.3f} ms, "
          f"{m / step / 1e6:.2f} M pred/s, {t1 / step / N:.2f} of N x the serial one-GPU rate",
          flush=True)
