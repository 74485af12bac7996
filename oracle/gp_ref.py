"""CPU oracle (TEST INFRASTRUCTURE ONLY) — numpy fp64 restatement of the GladsGP GP hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / reported CPU baseline.  The product path
(``gladsgp_amd``) never imports it: it runs the HIP kernels in ``libgpfit.so`` or fails.

What it restates (reference = timghill/GladsGP @ 2024_10_08, paths relative to its root):

* ARD squared-exponential Gram + jitter — ``examples/01_Gaussian_random_fields.ipynb:56-63,
  135-141`` (``sigma2*prod exp(-(dx/l)^2) + 1e-6 I``, i.e. ``beta = 1/l^2``) and GPmodule's
  ``squared_exponential`` as used by ``examples/02_univariate_GP_regression.ipynb:80``
  (``s = theta0^2, beta = 1/(2 theta1^2), delta = nugget^2``).  SEPIA's
  ``SepiaDistCov.compute_cov_mat(beta, lamz, lams)`` (un-vendored, ``requirements-cc.txt:55``)
  is the same form with ``s = 1/lamUz``, nugget ``1/lamWs`` (+ ``1/(lamWOs*LamSim)`` on the
  training diagonal).  Unified: ``G = s*exp(-sum_k beta_k (x_ik - x_jk)^2) + delta*I``.
* Jittered Cholesky — ``examples/01...ipynb:66,144`` (``scipy.linalg.cholesky(lower=True)``).
* Posterior mean / covariance — ``examples/02...ipynb:232-233``
  (``Kvec K^-1 y``, ``Kp - Kvec K^-1 Kvec^T``); here the marginal variance (diagonal) only,
  which is what SEPIA's ``storeMuSigma`` path exposes per point.
* MLE negative log-likelihood — GPmodule (un-vendored, ``requirements-cc.txt:20``):
  ``NLL = 1/2 y^T K^-1 y + 1/2 log|K|`` with no 2*pi term; pinned by the notebook's printed
  optimum ``fun = -3.989954265337257`` at ``x = [0.4093, 0.2270]`` (``02...ipynb:70-72``).
* Output standardisation and PCA basis — ``src/model.py:56-73`` (A1), ``:95-102`` (A3),
  ``:218-224`` (A4).
* Randomized SVD — ``src/svd.py:46-69`` (A2), with the Gaussian test matrix passed in so
  the restatement is deterministic.

Parity status: Gram/Cholesky/posterior formulas are pinned by the notebook-02 known answer
(``tests/golden/nb02_known_answer.json``); ``randomized_svd`` by outputs of the reference's
own ``src/svd.py`` (``tests/golden/svd_ref_64x500.npz``).  SEPIA's exact predictive code is
not available (un-vendored, no network): the per-(sample, PC) predictive mean/variance is the
GPMSA equation restated here, so SEPIA-specific parity is *partially unpinned* (see DESIGN.md).
"""
from __future__ import annotations

import numpy as np
import scipy.linalg as sla
import scipy.optimize as sopt

__all__ = [
    "gram_ardse", "cross_ardse", "cholesky", "predict", "nll_gpmodule", "fit_gpmodule",
    "gpmodule_theta_to_kernel", "standardize", "pca_basis", "pc_weights", "pc_precision",
    "randomized_svd", "sepia_gp_params", "sepia_predict_w", "reconstruct_y",
]


# ----------------------------------------------------------------------------------- kernels
def gram_ardse(X, beta, s, delta):
    """G = s*exp(-sum_k beta_k (x_ik-x_jk)^2) + delta*I  (examples/01...ipynb:135-141)."""
    X = np.asarray(X, dtype=np.float64)
    beta = np.asarray(beta, dtype=np.float64).reshape(-1)
    d2 = np.zeros((X.shape[0], X.shape[0]))
    for k in range(X.shape[1]):
        diff = X[:, k:k + 1] - X[:, k:k + 1].T
        d2 += beta[k] * diff * diff
    G = s * np.exp(-d2)
    G[np.diag_indices_from(G)] += delta
    return G


def cross_ardse(Xs, X, beta, s):
    """K*[i, j] = s*exp(-sum_k beta_k (xs_ik - x_jk)^2), shape (m, n) (02...ipynb:226 Kvec)."""
    Xs = np.asarray(Xs, dtype=np.float64)
    X = np.asarray(X, dtype=np.float64)
    beta = np.asarray(beta, dtype=np.float64).reshape(-1)
    d2 = np.zeros((Xs.shape[0], X.shape[0]))
    for k in range(X.shape[1]):
        diff = Xs[:, k:k + 1] - X[:, k:k + 1].T
        d2 += beta[k] * diff * diff
    return s * np.exp(-d2)


def cholesky(G):
    """Lower Cholesky factor and LAPACK-style info (0 ok, j>0: leading minor j not PD)."""
    try:
        return np.linalg.cholesky(G), 0
    except np.linalg.LinAlgError:
        # locate the first failing pivot (LAPACK potrf semantics) with an unblocked sweep
        A = np.array(G, dtype=np.float64, copy=True)
        n = A.shape[0]
        for j in range(n):
            v = A[j, j] - A[j, :j] @ A[j, :j]
            if not v > 0.0:
                return None, j + 1
            A[j, j] = np.sqrt(v)
            A[j + 1:, j] = (A[j + 1:, j] - A[j + 1:, :j] @ A[j, :j]) / A[j, j]
        return None, 0


def predict(X, Xs, w_hat, beta, s, delta, s_pred=None, chunk=10000):
    """Posterior mean and marginal variance of one GP (02...ipynb:232-233).

    mean = K* G^-1 w_hat ;  var = s_pred - diag(K* G^-1 K*^T),  G = gram(X) + delta I,
    s_pred defaults to s (noise-free prediction).  Cross-covariance is built in chunks of
    ``chunk`` test points (the bounded-memory loop of assess_all_models.py:481-500, but with
    one factorisation amortised over all points).
    """
    if s_pred is None:
        s_pred = s
    G = gram_ardse(X, beta, s, delta)
    L = np.linalg.cholesky(G)
    alpha = sla.cho_solve((L, True), np.asarray(w_hat, dtype=np.float64))
    m = Xs.shape[0]
    mean = np.empty(m)
    var = np.empty(m)
    for a in range(0, m, chunk):
        b = min(m, a + chunk)
        Ks = cross_ardse(Xs[a:b], X, beta, s)
        mean[a:b] = Ks @ alpha
        V = sla.solve_triangular(L, Ks.T, lower=True, check_finite=False)
        var[a:b] = s_pred - np.einsum("ij,ij->j", V, V)
    return mean, var


# -------------------------------------------------------------------- GPmodule MLE (config 1)
def gpmodule_theta_to_kernel(theta, nugget=1e-3):
    """GPmodule squared_exponential: K = theta0^2 exp(-dx^2/(2 theta1^2)) + nugget^2 I."""
    theta = np.asarray(theta, dtype=np.float64)
    s = theta[0] ** 2
    beta = np.full(1, 1.0 / (2.0 * theta[1] ** 2))
    return s, beta, nugget ** 2


def nll_gpmodule(theta, x, y, nugget=1e-3):
    """NLL = 1/2 y^T K^-1 y + 1/2 log|K| (no 2pi term) — reproduces 02...ipynb:70-72."""
    s, beta, delta = gpmodule_theta_to_kernel(theta, nugget)
    G = gram_ardse(np.asarray(x).reshape(len(x), -1), beta, s, delta)
    L, info = cholesky(G)
    if info:
        return np.inf
    yv = np.asarray(y, dtype=np.float64).reshape(-1)
    z = sla.solve_triangular(L, yv, lower=True)
    return 0.5 * z @ z + np.sum(np.log(np.diag(L)))


def fit_gpmodule(x, y, x0=(1.0, 0.5), nugget=1e-3):
    """GP(covariance=squared_exponential, cov_para={'nugget':1e-3}).fit(x, y, x0) (02:80-83)."""
    return sopt.minimize(nll_gpmodule, np.asarray(x0, dtype=np.float64), args=(x, y, nugget),
                         method="BFGS")


# ------------------------------------------------------------- src/model.py pre-processing
def standardize(y_sim, sd_threshold=1e-6):
    """src/model.py:60-72 — column mean, ddof=1 sd floored at sd_threshold, standardised Y."""
    y = np.asarray(y_sim, dtype=np.float64)
    mu = np.mean(y, axis=0)
    sd = np.std(y, ddof=1, axis=0)
    sd[sd < sd_threshold] = sd_threshold
    return mu, sd, (y - mu) / sd


def pca_basis(S, Vh, p, n):
    """src/model.py:101 — K = diag(S[:p]) Vh[:p] / sqrt(n)."""
    return np.diag(S[:p]) @ Vh[:p] / np.sqrt(n)


def pc_weights(y_std, K):
    """src/model.py:219 — w = y_std pinv(K)  (n, p); SEPIA's sim-only PC weights w_hat."""
    return np.dot(np.linalg.pinv(K).T, y_std.T).T


def pc_precision(y_std, K):
    """src/model.py:219-223 — 1/var(y_std - w K)."""
    w = pc_weights(y_std, K)
    return 1.0 / np.var(y_std - w @ K)


def randomized_svd(X, p, k=None, q=1, omega=None, rng=None):
    """src/svd.py:46-69 restated; ``omega`` (ny, p+k) may be given for determinism.

    dtype semantics follow the reference: Omega is float32 (:51) and numpy promotion decides
    the working precision, so a float32 X is factorised in float32, a float64 X in float64.
    """
    if k is None:
        k = p
    if omega is None:
        rng = np.random.default_rng(0) if rng is None else rng
        omega = rng.standard_normal((X.shape[1], p + k))
    omega = np.asarray(omega).astype(np.float32)
    Y = X @ omega
    for _ in range(q):
        Y = (X @ X.T) @ Y   # left-associative, as src/svd.py:56 (forms the n x n Gram)
    Q, _ = np.linalg.qr(Y, mode="reduced")
    B = Q.T @ X
    Ub, S, V = np.linalg.svd(B, full_matrices=False)
    U = Q @ Ub
    return U[:, :p], S[:p], V[:p, :]


# ------------------------------------------------------ SEPIA sim-only emulator (GPMSA form)
def sepia_gp_params(samples, LamSim, d, P, pred_nugget=True):
    """Per (sample, PC) kernel parameters from a SEPIA ``samples`` dict.

    betaU (S, (d+1)*P) reshapes C-order to (S, d+1, P), row 0 = dummy x (Delta = 0)
    (mcmc_diagnostics_advanced.py:57).  Sigma_j = exp(-sum beta Delta^2)/lamUz_j
    + (1/lamWs_j + 1/(lamWOs LamSim_j)) I on the training block; the prediction prior variance
    is 1/lamUz_j (+ 1/lamWs_j when ``pred_nugget``).
    Returns beta (S, P, d), s (S, P), delta (S, P), s_pred (S, P).
    """
    bu = np.asarray(samples["betaU"], dtype=np.float64)
    S = bu.shape[0]
    beta = bu.reshape(S, d + 1, P)[:, 1:, :].transpose(0, 2, 1).copy()
    lamUz = np.asarray(samples["lamUz"], dtype=np.float64).reshape(S, P)
    lamWs = np.asarray(samples["lamWs"], dtype=np.float64).reshape(S, P)
    lamWOs = np.asarray(samples["lamWOs"], dtype=np.float64).reshape(S, 1)
    LamSim = np.asarray(LamSim, dtype=np.float64).reshape(1, P)
    s = 1.0 / lamUz
    delta = 1.0 / lamWs + 1.0 / (lamWOs * LamSim)
    s_pred = s + (1.0 / lamWs if pred_nugget else 0.0)
    return beta, s, delta, s_pred


def sepia_predict_w(t_sim, t_pred, w_hat, samples, LamSim, pred_nugget=True):
    """Predictive mean and marginal variance of the PC weights, shapes (S, m, P) each."""
    t_sim = np.asarray(t_sim, dtype=np.float64)
    d = t_sim.shape[1]
    w_hat = np.asarray(w_hat, dtype=np.float64)
    P = w_hat.shape[1]
    beta, s, delta, s_pred = sepia_gp_params(samples, LamSim, d, P, pred_nugget)
    S = beta.shape[0]
    m = np.asarray(t_pred).shape[0]
    mean = np.empty((S, m, P))
    var = np.empty((S, m, P))
    for a in range(S):
        for j in range(P):
            mu, v = predict(t_sim, t_pred, w_hat[:, j], beta[a, j], s[a, j], delta[a, j],
                            s_pred[a, j])
            mean[a, :, j] = mu
            var[a, :, j] = v
    return mean, var


def reconstruct_y(w, K, mu, sd):
    """SepiaEmulatorPrediction.get_y(): y = (w K) sd + mu, shape (S, m, ny)."""
    return np.einsum("smp,py->smy", w, K) * sd + mu
