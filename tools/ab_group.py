"""A/B: factorisation group size for many-GP predictions at the reference's own shapes
(assess_all_models.py:471,481-489: 64 samples x p = 8, 4 test points per call; n = 256 / 512).

EmulatorPrediction factorises its (sample, PC) GPs in groups: one group of up to ~512 at these
sizes (the blocked sweep: the persistent kernel takes at most #CUs / 2 problems per launch) or
groups capped at the persistent kernel's limit.  Prints ms per EmulatorPrediction (median of
reps) for each group size."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import model as gm  # noqa: E402
from gladsgp_amd.emulator import EmulatorPrediction  # noqa: E402

dev = torch.device("cuda:0")
P = 8
for n, S in ((256, 64), (512, 64), (512, 128)):
    rng = np.random.default_rng(0)
    t = rng.random((n, 8))
    y = 1.0 + np.sin(2 * np.pi * t @ rng.uniform(0, 1, 8))[:, None] * rng.standard_normal(
        (1, 400)) + 0.05 * rng.standard_normal((n, 400))
    np.random.seed(0)
    data, model = gm.init_model(t, y, "ab", P, data_dir=f"/tmp/ab_group_{n}", device=dev,
                                verbose=False)
    r = np.random.default_rng(1)
    samples = {"betaU": r.uniform(0.2, 3.0, (S, 9 * P)), "lamUz": r.uniform(0.5, 3, (S, P)),
               "lamWs": r.uniform(200, 3000, (S, P)), "lamWOs": r.uniform(50, 500, (S, 1))}
    for m in (4, 1000):
        xp = np.random.default_rng(2).random((m, 8))
        ref = None
        for group in (None, 512, 256, 128, 96, 64, 32):
            ts = []
            for rep in range(6):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                pr = EmulatorPrediction(model=model, samples=samples, t_pred=xp, group=group)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            w = pr.w
            if ref is None:
                ref = w
            dm = float(np.max(np.abs(w - ref)))
            print(f"n={n} S={S} units={S * P} m={m} group={group}: "
                  f"{1e3 * np.median(ts[1:]):8.2f} ms (min {1e3 * min(ts[1:]):.2f}) "
                  f"max|dw| vs first {dm:.2e}", flush=True)
