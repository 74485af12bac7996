"""Maximum-likelihood GP — drop-in for the GPmodule surface of BASELINE config 1.

Reference usage (``examples/02_univariate_GP_regression.ipynb`` cell 5, raw :80-85; GPmodule is
un-vendored, ``requirements-cc.txt:20``)::

    GPmodel = GPmodule.GP(covariance=GPmodule.squared_exponential, cov_para={'nugget': 1e-3})
    fit_maxl = GPmodel.fit(x, y, x0)        # x0 = [variance, length scale] start
    print(GPmodel.minimize_res)             # scipy OptimizeResult: fun -3.989954265337257
    ypred = GPmodel.predictor(xpred)
    epred = GPmodel.error(xpred)

and cell 9 uses ``GPmodel.covariance(x1, x2, theta)``, ``GPmodel.theta``, ``GPmodel.K`` and
``GPmodel.K_inv``.

Model (restated; pinned by the notebook's printed optimum, ``tests/golden/nb02_known_answer``):
``K(theta) = theta0^2 exp(-|dx|^2 / (2 theta1^2)) + nugget^2 I`` and the objective
``NLL(theta) = 1/2 y^T K^-1 y + 1/2 log|K|`` (no 2 pi term), minimised by BFGS from ``x0``.
Every objective evaluation runs on the GPU: Gram (gp_gram_ardse) -> Cholesky + L^-1
(gp_potrf_inv) -> quadratic form + logdet (gp_nll); scipy drives the optimisation on the host
(the reference does the same with numpy).  ``predictor`` / ``error`` are gp_predict's posterior
mean and sqrt(marginal variance) at the fitted theta (cell 9's formulas, diagonal only; the
prior variance at a prediction point is theta0^2 — whether GPmodule adds the nugget there is not
recorded anywhere in the reference: parity for ``error`` is unpinned at the 1e-6 level).
"""
from __future__ import annotations

import numpy as np
import scipy.optimize as sopt
import torch

from . import kernels

F64 = torch.float64


def _theta_to_kernel(theta, nugget):
    """(s, beta, delta) of the unified ARD-SE form for GPmodule's squared exponential."""
    theta = np.asarray(theta, dtype=np.float64).reshape(-1)
    return theta[0] ** 2, 1.0 / (2.0 * theta[1] ** 2), nugget ** 2


def squared_exponential(x1, x2, theta, nugget: float = 0.0, device=None):
    """theta0^2 exp(-|x1_i - x2_j|^2 / (2 theta1^2)) (+ nugget^2 on the diagonal when x1 is x2)
    as a numpy (n1, n2) matrix, built by the gp_cross_ardse kernel."""
    dev = _device(device)
    a = np.asarray(x1, dtype=np.float64)
    b = np.asarray(x2, dtype=np.float64)
    a = a.reshape(a.shape[0], -1)
    b = b.reshape(b.shape[0], -1)
    s, beta, delta = _theta_to_kernel(theta, nugget)
    d = a.shape[1]
    Kt = kernels.cross(torch.as_tensor(b, device=dev), torch.as_tensor(a, device=dev),
                       torch.full((1, d), beta, dtype=F64, device=dev), s)   # (1, n1, n2)
    K = Kt[0].cpu().numpy()
    if x1 is x2 and delta:
        K[np.diag_indices_from(K)] += delta
    return K


def _device(device):
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("gladsgp_amd.gpmodule runs on a HIP device (libgpfit); none found")
    return torch.device("cuda", torch.cuda.current_device())


class GP:
    """GPmodule.GP mirror (fit by maximum likelihood, predict at new points)."""

    def __init__(self, covariance=squared_exponential, cov_para=None, device=None):
        if covariance is not squared_exponential:
            raise NotImplementedError("only the squared-exponential covariance is on the GPU path")
        self.covariance_fn = covariance
        self.cov_para = dict(cov_para or {})
        self.nugget = float(self.cov_para.get("nugget", 0.0))
        self.device = _device(device)
        self.theta = None
        self.minimize_res = None
        self.nfev_gpu = 0

    # ------------------------------------------------------------------------------ kernels
    def covariance(self, x1, x2, theta):
        return squared_exponential(x1, x2, theta, self.nugget if x1 is x2 else 0.0,
                                   self.device)

    def _factor(self, theta):
        s, beta, delta = _theta_to_kernel(theta, self.nugget)
        d = self._X.shape[1]
        G = kernels.gram(self._X, torch.full((1, d), beta, dtype=F64, device=self.device), s,
                         delta)
        return kernels.cholesky_inverse(G), s, beta

    def negloglik(self, theta) -> float:
        """1/2 y^T K^-1 y + 1/2 log|K| at theta (inf where K is not positive definite)."""
        ch, _, _ = self._factor(theta)
        v = kernels.nll(ch, self._y)
        self.nfev_gpu += 1
        if int(ch.info[0]) != 0:
            return np.inf
        return float(v[0])

    # ---------------------------------------------------------------------------- surface
    def fit(self, x, y, x0, method: str = "BFGS", **minimize_kw):
        """Maximum-likelihood theta from start x0 (scipy BFGS over the GPU objective).
        Returns the fitted theta; the scipy result is ``self.minimize_res``."""
        x = np.asarray(x, dtype=np.float64)
        self._x = x.reshape(x.shape[0], -1)
        self._X = torch.as_tensor(self._x, device=self.device).contiguous()
        self._y_np = np.asarray(y, dtype=np.float64).reshape(-1)
        self._y = torch.as_tensor(self._y_np, device=self.device).reshape(1, -1)
        res = sopt.minimize(self.negloglik, np.asarray(x0, dtype=np.float64), method=method,
                            **minimize_kw)
        self.minimize_res = res
        self.theta = np.asarray(res.x, dtype=np.float64)
        ch, s, beta = self._factor(self.theta)
        ch.check()
        self._chol, self._s, self._beta = ch, s, beta
        return self.theta

    @property
    def K(self) -> np.ndarray:
        """Training covariance at the fitted theta, nugget^2 on the diagonal (numpy)."""
        return self.covariance(self._x, self._x, self.theta)

    @property
    def K_inv(self) -> np.ndarray:
        """K^-1 = L^-T L^-1 from the GPU factorisation (numpy; small-n diagnostics)."""
        Li = self._chol.Linv[0].cpu().numpy()
        return Li.T @ Li

    def _predict(self, xpred):
        xp = np.asarray(xpred, dtype=np.float64)
        xp = xp.reshape(xp.shape[0], -1)
        d = self._x.shape[1]
        beta = torch.full((1, d), self._beta, dtype=F64, device=self.device)
        mean, var = kernels.predict(self._chol, self._X,
                                    torch.as_tensor(xp, device=self.device), beta, self._s,
                                    self._s, self._y)
        return mean[0].cpu().numpy(), var[0].cpu().numpy()

    def predictor(self, xpred) -> np.ndarray:
        """Posterior mean K(xpred, x) K^-1 y at the fitted theta, shape (m,)."""
        return self._predict(xpred)[0]

    def error(self, xpred) -> np.ndarray:
        """Posterior standard error sqrt(diag(K(xp, xp) - K(xp, x) K^-1 K(x, xp))), shape (m,)."""
        return np.sqrt(np.maximum(self._predict(xpred)[1], 0.0))
