"""Drop-in for ``src/model.py``: ``init_model``, ``load_model``, ``fit_models``.

Same arguments, file layout and semantics as the reference (``src/model.py:20-245``), with
every array operation on the GPU through libgpfit:
  * output standardisation ``mu, sd(ddof=1) floored, y_std``          (model.py:56-73, A1)
  * PCA basis from ``randomized_svd(y_std, 25, k=0, q=1)``, cached as
    ``pca_{exp}_{U,S,Vh}.npy`` and always re-read from disk           (model.py:75-98, A2)
  * ``K = diag(S[:p]) Vh[:p] / sqrt(n)``, cast through float32 as the reference's
    ``create_K_basis(K.astype(np.float32))``                           (model.py:100-102, A3)
  * PC weights / LamSim of the SEPIA model and the truncation precision ``pc_prec`` with the
    ``lamWOs ~ Gamma(50, 50/pc_prec)`` prior                            (model.py:218-229, A4)
``fit_models`` then runs SEPIA's Metropolis fit (``tune_step_sizes`` / ``do_mcmc``,
model.py:234-235) on the GPU (gladsgp_amd.mcmc) and saves models + ``timing.csv``.
"""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from . import blas
from .blas import CM, gemm
from .emulator import EmulatorData, EmulatorModel
from .mcmc import SepiaParam
from .svd import LegacyNormalDraw, randomized_svd

PMAX = 25   # model.py:81


def _scale_rows_tensor(t: torch.Tensor, f: torch.Tensor) -> None:
    """t[j, :] *= f[j] for a C-order (p, ny) tensor (K = diag(f) Vh[:p], model.py:101).

    gp_rowscale scales rows of a column-major matrix; t^T stored C-order is exactly the
    column-major (p x ny) matrix, so scale that copy and write it back.
    """
    from . import _capi
    from .kernels import _stream
    p, ny = t.shape
    tt = t.transpose(0, 1).contiguous()          # (ny, p) C-order == column-major (p x ny)
    _capi.call("gp_rowscale", tt.data_ptr(), p, ny, p, f.data_ptr(), 0, _stream(t.device))
    t.copy_(tt.transpose(0, 1))


def init_model(t_std, y_sim, exp, p, data_dir="data/", sd_threshold=1e-6, recompute=False,
               device=None, float32_basis=True, omega=None, verbose=True):
    """Build EmulatorData / EmulatorModel with the PCA basis (src/model.py:20-107)."""
    y_ind_sim = np.linspace(0, 1, np.shape(y_sim)[1])
    os.makedirs(data_dir, exist_ok=True)
    pca_fpattern = os.path.join(data_dir, "pca_{}_{}.npy")
    have = all(os.path.exists(pca_fpattern.format(exp, a)) for a in ("U", "S", "Vh"))
    draw = None
    if (recompute or not have) and omega is None:
        # randomized_svd's test matrix as the reference draws it in init_model's
        # randomized_svd(y_std, 25, k=0) (src/svd.py:51, model.py:84): np.random.normal((ny, 25))
        # as float32, whatever n -- the same global-RNG stream and the same advance of it --
        # on a host thread while the ensemble is uploaded and standardised: numpy's own draw was
        # the PCA's largest single cost (347 of 694 ms at 512 x 1,347,945,
        # profiles/r04/prof_pca_a.log), hence the bit-identical vectorised + threaded host
        # generator.  numpy's state is read here and advanced at draw.result(), both on this
        # thread (svd.LegacyNormalDraw).
        draw = LegacyNormalDraw((np.shape(y_sim)[1], PMAX))
    data = EmulatorData(t_sim=t_std, y_sim=y_sim, y_ind_sim=y_ind_sim, device=device)
    data.standardize_y(sd_threshold=sd_threshold)           # mu, sd (ddof=1, floored), y_std
    sd_ = data.sim_data
    if recompute or not have:
        # fewer than 25 runs (or nodes): range(X Omega) is already all of range(X) with
        # min(n, ny) test vectors, so the first r columns of the reference's Omega give its
        # U, S, Vh (up to signs and rounding) without a rank-deficient B B^T
        r = min(PMAX, *sd_.y_std.shape)
        om = draw.result() if draw is not None else omega
        if draw is not None and r < PMAX:
            om = np.ascontiguousarray(om[:, :r])
        U, S, Vh = randomized_svd(sd_.y_std, r, k=0, q=1, omega=om)
        # the reference's y_std has y_sim's dtype (float32 in fit_models / load_model), and its
        # randomized_svd returns (and init_model caches) that dtype (src/svd.py:51-68,
        # model.py:87-89); the build computes in fp64 and casts the cached arrays alike
        ydt = y_sim.dtype if torch.is_tensor(y_sim) else np.asarray(y_sim).dtype
        f32 = ydt in (np.float32, torch.float32)
        cast = (lambda a: a.to(torch.float32)) if f32 else (lambda a: a)  # noqa: E731
        np.save(pca_fpattern.format(exp, "U"), cast(U[:, :PMAX]).cpu().numpy())
        np.save(pca_fpattern.format(exp, "S"), cast(S).cpu().numpy())
        np.save(pca_fpattern.format(exp, "Vh"), cast(Vh[:PMAX, :]).cpu().numpy())
    # always use the saved matrices (model.py:91-94)
    S = np.load(pca_fpattern.format(exp, "S"))
    Vh = np.load(pca_fpattern.format(exp, "Vh"))
    if verbose:
        S2 = S ** 2
        print("SVD proportion of variance:", (S2 / np.sum(S2))[:10])
    dev = data.device
    St = torch.as_tensor(S, dtype=torch.float64, device=dev)
    Vt = torch.as_tensor(Vh, dtype=torch.float64, device=dev)
    K = Vt[:p].contiguous().clone()
    f = (St[:p] / np.sqrt(sd_.n)).contiguous()
    _scale_rows_tensor(K, f)
    if float32_basis:                                       # create_K_basis(K.astype(float32))
        K = K.to(torch.float32).to(torch.float64)
    data.create_K_basis(K)
    if verbose:
        print("K.shape", tuple(K.shape))
    model = EmulatorModel(data)
    return data, model


def pc_precision(data: EmulatorData) -> float:
    """pc_prec = 1 / var(y_std - w K), w = y_std pinv(K) (src/model.py:219-224)."""
    from .emulator import pc_weights
    sd_ = data.sim_data
    W, _ = pc_weights(data)                                  # (n x P) column-major
    Kc = CM.of_rowmajor(sd_.K)                               # (ny x P) = K^T
    R = CM.of_rowmajor(sd_.y_std.clone())                    # (ny x n) = y_std^T
    gemm(False, True, Kc, W, alpha=-1.0, beta=1.0, C=R)      # y_std^T - K^T W^T
    n, ny = sd_.y_std.shape
    mv = blas.mean_var(R.t[:n, :ny], ddof=0)                 # np.var: ddof = 0
    return 1.0 / float(mv[1].item())


def load_model(train_config, m, p, dtype=np.float32, device=None):
    """src/model.py:109-150: design CSV + ensemble .npy -> init_model -> restore samples."""
    t_std = np.loadtxt(train_config.X_standard, delimiter=",", skiprows=1,
                       comments=None).astype(dtype)[:m]
    y_sim = np.load(train_config.Y_physical).T.astype(dtype)[:m]
    data_dir = os.path.join(train_config.data_dir, "models")
    os.makedirs(data_dir, exist_ok=True)
    model_name = "{}_n{:03d}_p{:02d}".format(train_config.exp, m, p)
    m_name = "{}_n{:03d}".format(train_config.exp, m)
    model_path = os.path.join(data_dir, model_name)
    data, model = init_model(t_std=t_std, y_sim=y_sim, exp=m_name, p=p, data_dir=data_dir,
                             recompute=False, device=device)
    print("Restoring from:", model_path)
    model.restore_model_info(model_path)
    return data, model


def fit_models(train_config, n_sims, n_pcs, dtype=np.float32, recompute=False, device=None,
               n_burn=100, n_levels=5, nsamp=512, seed=None):
    """src/model.py:152-245: for every (m, p), PCA + standardisation (init_model), the
    truncation precision pc_prec and its lamWOs prior Gamma(50, 50/pc_prec) with bounds
    [1, inf), start pc_prec, Uniform step 10 (model.py:218-231); then
    ``tune_step_sizes(100, 5)`` and ``do_mcmc(512)`` (model.py:234-235) on the GPU; saves
    each model and ``timing.csv`` (sims, PCs, PCA seconds, MCMC seconds) like the reference.
    ``n_burn``/``n_levels``/``nsamp`` default to the reference's values; ``seed`` seeds the
    sampler's uniforms (the reference uses numpy's global state).
    """
    t_std = np.loadtxt(train_config.X_standard, delimiter=",", skiprows=1,
                       comments=None).astype(dtype)
    y_sim = np.load(train_config.Y_physical).T.astype(dtype)
    data_dir = os.path.join(train_config.data_dir, "models")
    os.makedirs(data_dir, exist_ok=True)
    models, rows = [], []
    for m in n_sims:
        for p in n_pcs:
            t0 = time.perf_counter()
            data, model = init_model(t_std=t_std[:m], y_sim=y_sim[:m],
                                     exp="{}_n{:03d}".format(train_config.exp, m), p=p,
                                     data_dir=data_dir, recompute=recompute, device=device)
            torch.cuda.synchronize()
            dt_pca = time.perf_counter() - t0
            prec = pc_precision(data)
            print("PC PRECISION:", prec)
            gamma_a = 50.0
            model.params.lamWOs = SepiaParam(val=prec, name="lamWOs", val_shape=(1, 1),
                                             dist="Gamma", params=[gamma_a, gamma_a / prec],
                                             bounds=[1.0, np.inf], mcmcStepParam=10,
                                             mcmcStepType="Uniform")
            model.params.mcmcList = [model.params.betaU, model.params.lamUz,
                                     model.params.lamWs, model.params.lamWOs]
            if seed is not None:
                model.rng = np.random.default_rng(seed)
            t0 = time.perf_counter()
            model.tune_step_sizes(n_burn, n_levels)
            model.do_mcmc(nsamp)
            torch.cuda.synchronize()
            dt_mcmc = time.perf_counter() - t0
            model.save_model_info(os.path.join(data_dir,
                                               "{}_n{:03d}_p{:02d}".format(train_config.exp,
                                                                           m, p)))
            models.append(model)
            rows.append([m, p, dt_pca, dt_mcmc])
    np.savetxt(os.path.join(data_dir, "timing.csv"), np.array(rows, dtype=np.float64),
               delimiter=",", fmt="%.3f", header="sims,PCs,PCA (seconds),MCMC (seconds)")
    return models
