"""CPU oracle (TEST INFRASTRUCTURE ONLY) — numpy restatement of the sim-only GPMSA Metropolis fit.

Only ``tests/`` may import this module, as the checker of ``gladsgp_amd.mcmc``; the product
path never imports it.

Restates SEPIA's ``SepiaModel.do_mcmc`` as driven by ``src/model.py:225-235`` (SEPIA itself is
un-vendored, ``requirements-cc.txt:55``, and unavailable offline — SURVEY section 8c):

* per-PC log-likelihood  ``-1/2 log|Sigma_j| - 1/2 w_j^T Sigma_j^-1 w_j`` with
  ``Sigma_j = (1/lamUz_j) exp(-sum_k betaU[k+1,j] dt_k^2) + (1/lamWs_j + 1/(lamWOs LamSim_j)) I``
  (SURVEY A5/A7), via ``scipy.linalg.cholesky``;
* log priors: Beta(a, b) on ``rho = exp(-beta/4)`` (rho clipped at 0.999), Gamma(a, b) as
  (shape, rate);
* proposals ``x + step (u - 1/2)`` (``BetaRho``: the same move on rho), out-of-bounds ->
  reject; accept when ``log u < delta log posterior``;
* sweep order: betaU rows 0..d (row 0 = dummy x, prior only), lamUz, lamWs, lamWOs, with the
  same uniform layout as ``gladsgp_amd.mcmc.GPUSampler.sweep`` so both chains can be fed
  identical random numbers.

Parity status: the likelihood is the SURVEY A7 formula (pinned structurally by the reference's
``(S, (d+1) P)`` sample layout and the step-size defaults of ``03...ipynb:192-208``); SEPIA's
exact priors, proposal kernels and tuning constants are *unpinned* (no source, no fixtures).
"""
from __future__ import annotations

import numpy as np
import scipy.linalg as sla

from .gp_ref import gram_ardse

RHO_MAX = 0.999


def loglik_pcs(X, w, LamSim, betaU, lamUz, lamWs, lamWOs):
    """(P,) per-PC log-likelihoods; -inf where Sigma_j is not positive definite."""
    P = w.shape[0]
    out = np.empty(P)
    for j in range(P):
        s = 1.0 / lamUz[j]
        delta = 1.0 / lamWs[j] + 1.0 / (lamWOs * LamSim[j])
        G = gram_ardse(X, betaU[1:, j], s, delta)
        try:
            L = sla.cholesky(G, lower=True)
        except np.linalg.LinAlgError:
            out[j] = -np.inf
            continue
        z = sla.solve_triangular(L, w[j], lower=True)
        out[j] = -0.5 * z @ z - np.sum(np.log(np.diag(L)))
    return out


def log_prior(dist, params, x):
    a, b = params
    x = np.asarray(x, dtype=np.float64)
    if dist == "Gamma":
        return (a - 1.0) * np.log(x) - b * x
    if dist == "Beta":
        rho = np.minimum(np.exp(-x / 4.0), RHO_MAX)
        return (a - 1.0) * np.log(rho) + (b - 1.0) * np.log1p(-rho)
    raise ValueError(dist)


def propose(step_type, bounds, x, step, u):
    if step_type == "BetaRho":
        rho = np.exp(-x / 4.0) + step * (u - 0.5)
        ok = (rho > 0.0) & (rho <= 1.0)
        cand = -4.0 * np.log(np.where(ok, rho, 1.0))
    else:
        cand = x + step * (u - 0.5)
        ok = np.ones(np.shape(cand), bool)
    ok = ok & (cand >= bounds[0]) & (cand <= bounds[1])
    return np.where(ok, cand, x), ok


def run_chain(X, w, LamSim, spec, state, steps, U):
    """Run len(U) sweeps.  ``spec[name] = (dist, params, bounds, step_type)``; ``state`` dict
    with betaU (d+1, P), lamUz (P,), lamWs (P,), lamWOs float; ``steps`` like state; ``U`` the
    (sweeps, uniforms_per_sweep) uniforms.  Returns (final state, samples dict, accept counts).
    """
    st = {k: np.array(v, dtype=np.float64, copy=True) for k, v in state.items()}
    st["lamWOs"] = float(st["lamWOs"])
    d1, P = st["betaU"].shape
    ll = loglik_pcs(X, w, LamSim, st["betaU"], st["lamUz"], st["lamWs"], st["lamWOs"])
    rec = {k: [] for k in ("betaU", "lamUz", "lamWs", "lamWOs")}
    acc_n = {k: np.zeros_like(np.asarray(v, dtype=np.float64)) for k, v in st.items()}
    for u in U:
        o = 0
        dist, prm, bnd, stype = spec["betaU"]
        for k in range(d1):
            up, ua = u[o:o + P], u[o + P:o + 2 * P]
            o += 2 * P
            cur = st["betaU"][k].copy()
            cand, ok = propose(stype, bnd, cur, steps["betaU"][k], up)
            dlp = log_prior(dist, prm, cand) - log_prior(dist, prm, cur)
            if k == 0:
                acc = ok & (np.log(ua) < dlp)
                st["betaU"][0] = np.where(acc, cand, cur)
            else:
                trial = st["betaU"].copy()
                trial[k] = cand
                ll_new = loglik_pcs(X, w, LamSim, trial, st["lamUz"], st["lamWs"],
                                    st["lamWOs"])
                with np.errstate(invalid="ignore"):
                    acc = ok & (np.log(ua) < ll_new - ll + dlp)
                st["betaU"][k] = np.where(acc, cand, cur)
                ll = np.where(acc, ll_new, ll)
            acc_n["betaU"][k] += acc
        for name in ("lamUz", "lamWs"):
            dist, prm, bnd, stype = spec[name]
            up, ua = u[o:o + P], u[o + P:o + 2 * P]
            o += 2 * P
            cur = st[name].copy()
            cand, ok = propose(stype, bnd, cur, np.reshape(steps[name], P), up)
            args = {"lamUz": st["lamUz"], "lamWs": st["lamWs"]}
            args[name] = cand
            ll_new = loglik_pcs(X, w, LamSim, st["betaU"], args["lamUz"], args["lamWs"],
                                st["lamWOs"])
            with np.errstate(invalid="ignore"):
                acc = ok & (np.log(ua) < ll_new - ll + log_prior(dist, prm, cand)
                            - log_prior(dist, prm, cur))
            st[name] = np.where(acc, cand, cur)
            ll = np.where(acc, ll_new, ll)
            acc_n[name] += acc
        dist, prm, bnd, stype = spec["lamWOs"]
        up, ua = u[o], u[o + 1]
        o += 2
        cur = st["lamWOs"]
        cand, ok = propose(stype, bnd, np.array([cur]), np.reshape(steps["lamWOs"], 1),
                           np.array([up]))
        cand, ok = float(cand[0]), bool(ok[0])
        ll_new = loglik_pcs(X, w, LamSim, st["betaU"], st["lamUz"], st["lamWs"], cand)
        with np.errstate(invalid="ignore"):
            dl = np.sum(ll_new - ll) + float(log_prior(dist, prm, cand)
                                             - log_prior(dist, prm, cur))
        acc = ok and bool(np.log(ua) < dl)
        if acc:
            st["lamWOs"], ll = cand, ll_new
        acc_n["lamWOs"] += acc
        rec["betaU"].append(st["betaU"].reshape(-1).copy())
        rec["lamUz"].append(st["lamUz"].copy())
        rec["lamWs"].append(st["lamWs"].copy())
        rec["lamWOs"].append([st["lamWOs"]])
    return st, {k: np.array(v) for k, v in rec.items()}, acc_n
