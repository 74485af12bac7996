"""Regenerate the committed golden fixtures (run in the build container, NOT on the GPU box).

    python tests/golden/make_golden.py [--reference /root/reference]

Writes only data (.npz / .json / .csv) into tests/golden/:

* ``synthetic_{train,test}_standard.csv`` — the reference's own design fixtures (512x8 and
  100x8, ``experiments/synthetic/expdesign/``; identical copies in
  ``examples/data/GlaDS_example/``), copied verbatim as data.
* ``nb02_known_answer.json`` — the MLE optimum printed by
  ``examples/02_univariate_GP_regression.ipynb`` (cell output at :70-72 of the raw JSON), the
  notebook inputs (:43), and the oracle's restatement of that fit (BFGS from [1, 0.5]) plus
  its 51-point posterior mean / sd at the optimum.
* ``svd_ref_64x500.npz`` — outputs of the reference's own ``src/svd.py`` ``randomized_svd``
  imported from the read-only reference tree, on a seeded float32 matrix with
  ``np.random.seed(123)`` (p=8, k=None, q=1) and (p=25, k=0, q=1), together with the Gaussian
  test matrices it drew, so the oracle restatement can be checked exactly.
* ``svd_ref_deficient.npz`` — the reference's ``randomized_svd`` on column-centred (hence
  rank <= n - 1) float32 ensembles of n = 16, 20, 25 runs with ``init_model``'s
  ``r = min(25, n, ny)``, k = 0, q = 1 (``src/model.py:84``; ``test_install.sh`` uses
  ``--nsim 16``), seeded, with the Gaussian test matrices it drew.
* ``svd_ref_pmax25.npz`` — the reference's ``randomized_svd`` called as ``init_model`` calls it
  (``randomized_svd(y_std, 25, k=0, q=1)``, Omega (ny, 25)) on n = 16 and 20 runs, with the raw
  ensemble, Omega and the global RNG's next value after the call.
* ``c2_golden.npz`` — oracle GP outputs on the real 512x8 design (C2 recipe) at
  256 test points: Gram spot values, logdet, mean, var, nll.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import gp_ref  # noqa: E402


def copy_designs(ref: str) -> None:
    src = os.path.join(ref, "experiments", "synthetic", "expdesign")
    for name in ("synthetic_train_standard.csv", "synthetic_test_standard.csv"):
        shutil.copyfile(os.path.join(src, name), os.path.join(HERE, name))


def notebook_known_answer(ref: str) -> None:
    nb = json.load(open(os.path.join(ref, "examples", "02_univariate_GP_regression.ipynb")))
    printed = None
    for cell in nb["cells"]:
        for out in cell.get("outputs", []):
            text = "".join(out.get("text", []))
            if "fun:" in text and "nit:" in text:
                printed = text
    assert printed is not None, "notebook output not found"
    fun = float(printed.split("fun:")[1].split()[0])
    xs = printed.split("x: [")[1].split("]")[0].split()
    nit = int(printed.split("nit:")[1].split()[0])
    x = np.linspace(1 / 8, 7 / 8, 5).reshape(-1, 1)
    y = x * np.sin(2 * np.pi * x)
    res = gp_ref.fit_gpmodule(x, y, x0=(1.0, 0.5), nugget=1e-3)
    theta = np.abs(res.x)
    s, beta, delta = gp_ref.gpmodule_theta_to_kernel(theta, 1e-3)
    xpred = np.linspace(0, 1, 51).reshape(-1, 1)
    mean, var = gp_ref.predict(x, xpred, y.ravel(), beta, s, delta, s_pred=s)
    out = {
        "source": "examples/02_univariate_GP_regression.ipynb (printed scipy result)",
        "printed_fun": fun, "printed_x": [float(v) for v in xs], "printed_nit": nit,
        "x_train": x.ravel().tolist(), "y_train": y.ravel().tolist(),
        "x_pred": xpred.ravel().tolist(), "nugget": 1e-3,
        "oracle_fun": float(res.fun), "oracle_theta": theta.tolist(),
        "oracle_mean": mean.tolist(), "oracle_var": var.tolist(),
    }
    json.dump(out, open(os.path.join(HERE, "nb02_known_answer.json"), "w"), indent=1)
    print("nb02: printed", fun, xs, "oracle", res.fun, theta)


def svd_reference(ref: str) -> None:
    spec = importlib.util.spec_from_file_location("ref_svd", os.path.join(ref, "src", "svd.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rng = np.random.default_rng(7)
    base = rng.standard_normal((64, 12)) @ rng.standard_normal((12, 500))
    X = (base + 0.05 * rng.standard_normal((64, 500))).astype(np.float32)
    out = {"X": X}
    for tag, (p, k) in {"p8": (8, None), "p25k0": (25, 0)}.items():
        np.random.seed(123)
        U, S, Vh = mod.randomized_svd(X, p, k=k, q=1)
        np.random.seed(123)
        kk = p if k is None else k
        omega = np.random.normal(size=(X.shape[1], p + kk)).astype(np.float32)
        out.update({f"{tag}_U": U, f"{tag}_S": S, f"{tag}_Vh": Vh, f"{tag}_omega": omega})
    np.savez_compressed(os.path.join(HERE, "svd_ref_64x500.npz"), **out)
    print("svd golden written")


def svd_reference_deficient(ref: str) -> None:
    spec = importlib.util.spec_from_file_location("ref_svd", os.path.join(ref, "src", "svd.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = {}
    ny = 400
    for n in (16, 20, 25):
        rng = np.random.default_rng(100 + n)
        t = rng.random((n, 4))
        modes = rng.standard_normal((8, ny)) * (0.7 ** np.arange(8))[:, None]
        coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, 4) + k) for k in range(8)], 1)
        y = (3.0 + coef @ modes + 1e-2 * rng.standard_normal((n, ny))).astype(np.float32)
        mu = np.mean(y, axis=0)                      # src/model.py:60-72
        sd = np.std(y, ddof=1, axis=0)
        sd[sd < 1e-6] = 1e-6
        y_std = (y - mu) / sd
        r = min(25, *y_std.shape)
        np.random.seed(1000 + n)
        U, S, Vh = mod.randomized_svd(y_std, r, k=0, q=1)
        np.random.seed(1000 + n)
        omega = np.random.normal(size=(ny, r)).astype(np.float32)
        out.update({f"n{n}_y_std": y_std, f"n{n}_U": U, f"n{n}_S": S, f"n{n}_Vh": Vh,
                    f"n{n}_omega": omega})
    np.savez_compressed(os.path.join(HERE, "svd_ref_deficient.npz"), **out)
    print("rank-deficient svd golden written")


def svd_reference_model_call(ref: str) -> None:
    """``svd_ref_pmax25.npz``: the reference's ``randomized_svd`` called exactly as
    ``init_model`` calls it (``src/model.py:81-84``: ``pmax = 25``, ``randomized_svd(y_std, 25,
    k=0, q=1)``) on column-centred float32 ensembles of n = 16 and 20 runs (fewer runs than
    pmax: Omega is drawn (ny, 25), numpy's reduced QR keeps min(n, 25) = n columns, so U is
    n x n, S n, Vh n x ny).  Stored: the raw float32 ensemble and design (so the build's own
    ``init_model`` runs on it), the float32 y_std the reference standardised (src/model.py:60-72),
    the drawn Omega, the reference's U / S / Vh, and the first ``np.random.random()`` after the
    call (the global RNG's advance)."""
    spec = importlib.util.spec_from_file_location("ref_svd", os.path.join(ref, "src", "svd.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    out = {}
    ny = 400
    for n in (16, 20):
        rng = np.random.default_rng(200 + n)
        t = rng.random((n, 8)).astype(np.float32)
        modes = rng.standard_normal((8, ny)) * (0.7 ** np.arange(8))[:, None]
        coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, 8) + k) for k in range(8)], 1)
        y = (3.0 + coef @ modes + 1e-2 * rng.standard_normal((n, ny))).astype(np.float32)
        mu = np.mean(y, axis=0)                      # src/model.py:60-72, in y's dtype
        sd = np.std(y, ddof=1, axis=0)
        sd[sd < 1e-6] = 1e-6
        y_std = (y - mu) / sd
        np.random.seed(2000 + n)
        U, S, Vh = mod.randomized_svd(y_std, 25, k=0, q=1)
        after = np.random.random()
        np.random.seed(2000 + n)
        omega = np.random.normal(size=(ny, 25)).astype(np.float32)
        assert U.shape == (n, n) and S.shape == (n,) and Vh.shape == (n, ny)
        out.update({f"n{n}_t": t, f"n{n}_y": y, f"n{n}_y_std": y_std, f"n{n}_omega": omega,
                    f"n{n}_U": U, f"n{n}_S": S, f"n{n}_Vh": Vh,
                    f"n{n}_next_random": np.float64(after), f"n{n}_seed": np.int64(2000 + n)})
    np.savez_compressed(os.path.join(HERE, "svd_ref_pmax25.npz"), **out)
    print("pmax=25 model-call svd golden written")


def c2_golden() -> None:
    X = np.loadtxt(os.path.join(HERE, "synthetic_train_standard.csv"), delimiter=",",
                   skiprows=1, comments=None)
    a = np.random.default_rng(1).uniform(0, 1, 8)
    y = np.sin(2 * np.pi * X @ a) + 0.1 * np.sum(X * X, axis=1)
    beta = np.random.default_rng(3).uniform(0.5, 5.0, 8)
    Xs = np.random.default_rng(2).random((256, 8))
    s, delta = 1.0, 1e-6
    G = gp_ref.gram_ardse(X, beta, s, delta)
    L, info = gp_ref.cholesky(G)
    logdet = 2 * np.sum(np.log(np.diag(L)))
    mean, var = gp_ref.predict(X, Xs, y, beta, s, delta)
    import scipy.linalg as sla
    z = sla.solve_triangular(L, y, lower=True)
    nll = 0.5 * z @ z + 0.5 * logdet
    idx = np.random.default_rng(5).integers(0, 512, size=(64, 2))
    np.savez_compressed(os.path.join(HERE, "c2_golden.npz"), X=X, y=y, beta=beta, Xs=Xs,
                        s=s, delta=delta, gram_idx=idx, gram_vals=G[idx[:, 0], idx[:, 1]],
                        logdet=logdet, mean=mean, var=var, nll=nll)
    print("c2 golden: logdet", logdet, "nll", nll)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    copy_designs(args.reference)
    notebook_known_answer(args.reference)
    svd_reference(args.reference)
    svd_reference_deficient(args.reference)
    svd_reference_model_call(args.reference)
    c2_golden()


if __name__ == "__main__":
    main()
