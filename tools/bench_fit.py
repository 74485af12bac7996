"""Fit-side timing at the reference's fit configuration: n=512 runs, d=8, P PCs,
tune_step_sizes(100, 5) + do_mcmc(512) (src/model.py:234-235; the reference's own timing is
timing.csv: 1405.6 s MCMC for n=512, P=8 on CPU).  Synthetic field of C5's shape."""
import argparse
import json
import os
import sys
import time
import types

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gladsgp_amd import model as gmodel  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--ny", type=int, default=10000)
    ap.add_argument("--p", type=int, default=8)
    ap.add_argument("--burn", type=int, default=100)
    ap.add_argument("--levels", type=int, default=5)
    ap.add_argument("--nsamp", type=int, default=512)
    ap.add_argument("--out", default="gpurun_out/fit_bench")
    a = ap.parse_args()
    d = 8
    rng = np.random.default_rng(0)
    t = rng.random((a.n, d))
    modes = rng.standard_normal((12, a.ny)) * (0.6 ** np.arange(12))[:, None]
    coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, d) + k) for k in range(12)], 1)
    y = coef @ modes + 1e-3 * rng.standard_normal((a.n, a.ny))
    os.makedirs(a.out, exist_ok=True)
    np.savetxt(os.path.join(a.out, "X.csv"), t, delimiter=",",
               header=",".join(f"x{i}" for i in range(d)), comments="")
    np.save(os.path.join(a.out, "Y.npy"), y.T)
    cfg = types.SimpleNamespace(X_standard=os.path.join(a.out, "X.csv"),
                                Y_physical=os.path.join(a.out, "Y.npy"), data_dir=a.out,
                                exp="bench")
    dev = torch.device("cuda:0")
    t0 = time.perf_counter()
    models = gmodel.fit_models(cfg, [a.n], [a.p], dtype=np.float64, recompute=True, device=dev,
                               n_burn=a.burn, n_levels=a.levels, nsamp=a.nsamp, seed=0)
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
    tim = np.loadtxt(os.path.join(a.out, "models", "timing.csv"), delimiter=",")
    sweeps = a.burn * a.levels + a.nsamp
    m = models[0]
    acc = {k: np.round(np.mean(np.diff(m.samples[k], axis=0) != 0, axis=0), 3).tolist()
           for k in ("betaU", "lamUz", "lamWs", "lamWOs")}
    steps = {k: np.round(getattr(m.params, k).mcmcStepParam.reshape(-1), 4).tolist()
             for k in ("betaU", "lamUz", "lamWs", "lamWOs")}
    vals = {k: np.round(getattr(m.params, k).val.reshape(-1), 4).tolist()
            for k in ("lamUz", "lamWs", "lamWOs")}
    print(json.dumps({"n": a.n, "ny": a.ny, "P": a.p, "pca_s": float(tim[2]),
                      "mcmc_s": float(tim[3]), "total_s": tot, "sweeps": sweeps,
                      "ms_per_sweep": 1e3 * float(tim[3]) / sweeps,
                      "ref_mcmc_s_timing_csv": 1405.6 if (a.n, a.p) == (512, 8) else None,
                      "move_rate": acc, "tuned_steps": steps, "final_vals": vals,
                      "tune_accepts": {k: v.reshape(v.shape[0], -1).tolist()
                                       for k, v in m.tune_info["accepts"].items()
                                       if k != "betaU"}}))


if __name__ == "__main__":
    main()
