"""Multivariate GP emulator surface (the SEPIA objects the reference drives), on libgpfit.

Reference usage being replaced (SEPIA fork, un-vendored, ``requirements-cc.txt:55``):
  * ``SepiaData(t_sim, y_sim, y_ind_sim)`` + ``standardize_y`` + ``create_K_basis(K)``
    (``src/model.py:57-102``)                              -> :class:`EmulatorData`
  * ``SepiaModel(data)``, ``.get_samples(numsamples, nburn)``, ``.save_model_info`` /
    ``.restore_model_info`` (``src/model.py:106, 149, 238``; ``assess_all_models.py:471``)
                                                           -> :class:`EmulatorModel`
  * ``SepiaEmulatorPrediction(model=, samples=, t_pred=)`` with ``.w`` (S, m, P) and
    ``.get_y()`` (S, m, ny) (``time_predictions.py:76-79``, ``sensitivity_indices.py:85-88``,
    ``assess_all_models.py:489-492``)                      -> :class:`EmulatorPrediction`

The GPMSA sim-only model, per MCMC sample s and principal component j (one independent GP
each), with betaU (S, (d+1) P) reshaped C-order to (S, d+1, P), row 0 the dummy x
(``mcmc_diagnostics_advanced.py:57``):
  Sigma_j = (1/lamUz_j) exp(-sum_k beta_kj (t_ik - t_i'k)^2)
            + (1/lamWs_j + 1/(lamWOs LamSim_j)) I                       (training block)
  k*_j    = (1/lamUz_j) exp(-sum_k beta_kj (t*_k - t_ik)^2)              (cross-covariance)
  mean    = k*_j^T Sigma_j^-1 w_hat_j,  var = 1/lamUz_j [+ 1/lamWs_j] - k*_j^T Sigma_j^-1 k*_j
``pred_nugget`` selects whether 1/lamWs is part of the predictive prior variance (SEPIA's
exact choice is not verifiable offline — SURVEY §8c — so it is a flag, default on).

Differences from SEPIA, by design: by default ``.w`` is the posterior MEAN per (sample, PC)
and ``.var`` the marginal variance (SEPIA returns one joint random draw over the m_b x m_b
covariance of a call, which does not scale to m = 100k).  ``realize=True`` makes ``.w`` one
marginal draw per (sample, point, PC) instead (gp_realize, Philox4x32-10 on the device, seeded
by ``seed``), so the reference's quantile / coverage statistics over ``get_y()``
(assess_all_models.py:489-500) keep the GP's predictive spread; ``.mean`` always holds the
posterior mean.  ``.w`` is assignable, as the reference's callers do
(``preds.w = preds.w.astype(np.float32)``, time_predictions.py:78, assess_all_models.py:490,
513): ``get_y()`` then reconstructs from the assigned values and returns that dtype.  All
arithmetic runs in libgpfit (fp64); the (sample, PC) pairs are one batched Gram ->
Cholesky/L^-1 -> predict.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from . import blas, kernels
from . import dist as gdist
from . import mcmc, modelio
from .blas import CM, gemm
from .mcmc import ModelParams, SepiaParam  # noqa: F401  (re-exported for drop-in imports)

F64 = torch.float64


def _dev(device):
    if device is not None:
        return torch.device(device)
    if not torch.cuda.is_available():
        raise RuntimeError("the emulator runs on a HIP device (libgpfit); none found")
    return torch.device("cuda", torch.cuda.current_device())


def _np(x):
    return x.detach().cpu().numpy() if torch.is_tensor(x) else np.asarray(x)


def _to_host(t: torch.Tensor, dtype) -> np.ndarray:
    """Device tensor -> numpy in ``dtype``: narrowed on the device first (a float32 field crosses
    PCIe at half the bytes and skips a host conversion pass), copied into page-locked memory
    (one DMA, no pageable bounce; the returned array keeps its pinned block alive)."""
    tt = torch.float32 if np.dtype(dtype) == np.float32 else torch.float64
    src = t.to(tt).contiguous()
    host = torch.empty(src.shape, dtype=tt, pin_memory=True)
    host.copy_(src)
    return host.numpy()


def _to_device_f64(x, device) -> torch.Tensor:
    """float64 device copy of ``x``: host arrays cross PCIe in their own dtype (float32
    ensembles at half the bytes) and are widened on the device, not on the host."""
    if torch.is_tensor(x):
        return x.to(device=device, dtype=F64).contiguous()
    a = np.ascontiguousarray(np.asarray(x))
    if a.dtype not in (np.float32, np.float64):
        a = a.astype(np.float64)
    return torch.from_numpy(a).to(device).to(F64).contiguous()


class SimData:
    """Simulation block: design, raw and standardised outputs, PCA basis (SEPIA sim_data).

    ``t`` / ``y`` are host (numpy) arrays in the caller's dtype, as SEPIA's are — the
    reference's drivers run numpy on them (``np.std(model.data.sim_data.y, ddof=1, axis=0)``,
    time_predictions.py:65, assess_all_models.py:465); ``t_dev`` / ``y_dev`` are the float64
    device copies every kernel reads."""

    def __init__(self, t_sim, y_sim, y_ind_sim, device):
        self.device = device
        self.t_dev = _to_device_f64(t_sim, device)
        self.y_dev = _to_device_f64(y_sim, device)
        self._t_host = None if torch.is_tensor(t_sim) else np.asarray(t_sim)
        self._y_host = None if torch.is_tensor(y_sim) else np.asarray(y_sim)
        self.y_ind = np.asarray(y_ind_sim)
        self.y_mean = None
        self.y_sd = None
        self.y_std = None
        self.K = None          # (P, ny) basis

    @property
    def t(self) -> np.ndarray:
        if self._t_host is None:
            self._t_host = self.t_dev.cpu().numpy()
        return self._t_host

    @property
    def y(self) -> np.ndarray:
        if self._y_host is None:
            self._y_host = self.y_dev.cpu().numpy()
        return self._y_host

    @property
    def n(self) -> int:
        return self.t_dev.shape[0]


class EmulatorData:
    """Mirror of the SepiaData pieces src/model.py uses (sim-only, x = dummy)."""

    def __init__(self, t_sim, y_sim, y_ind_sim=None, device=None):
        device = _dev(device)
        y_ind_sim = np.linspace(0, 1, np.shape(y_sim)[1]) if y_ind_sim is None else y_ind_sim
        self.sim_data = SimData(t_sim, y_sim, y_ind_sim, device)
        self.device = device

    def standardize_y(self, y_mean=None, y_sd=None, sd_threshold=1e-6):
        """y_std = (y - mu)/sd with mu/sd from the ensemble when not given (model.py:60-73)."""
        sd_ = self.sim_data
        if y_mean is None or y_sd is None:
            mu, sd = blas.sim_stats(sd_.y_dev, sd_threshold)
        else:
            mu = torch.as_tensor(_np(y_mean), dtype=F64, device=self.device).contiguous()
            sd = torch.as_tensor(_np(y_sd), dtype=F64, device=self.device).contiguous()
        sd_.y_mean, sd_.y_sd = mu, sd
        # rows padded to a multiple of 16 doubles (128 B): every row of the ensemble starts
        # 16-B aligned, so the randomized SVD's ensemble-streaming products read it with 16-B
        # loads (blas.hip tsk16 / tsm16); y_std is a (n x ny) view of the padded buffer
        n, ny = sd_.y_dev.shape
        ld = (ny + 15) // 16 * 16
        out = torch.empty((n, ld), dtype=F64, device=sd_.y_dev.device)[:, :ny]
        sd_.y_std = blas.standardize(sd_.y_dev, mu, sd, out=out)

    def create_K_basis(self, K):
        """Set the PCA basis K (P x ny) — SEPIA create_K_basis (model.py:102)."""
        self.sim_data.K = (K.to(device=self.device, dtype=F64).contiguous() if torch.is_tensor(K)
                           else torch.as_tensor(np.asarray(K), dtype=F64,
                                                device=self.device).contiguous())


def pc_weights(data: EmulatorData):
    """w_hat = y_std pinv(K) (n x P) and LamSim = diag(K K^T) — model.py:219; SEPIA's w.

    pinv(K) = K^T (K K^T)^-1 for a full-row-rank basis: two MFMA GEMMs and the P x P
    Cholesky inverse (K K^T)^-1 = L^-T L^-1.
    """
    sd_ = data.sim_data
    K = CM.of_rowmajor(sd_.K)             # (ny x P) column-major view of K^T
    Ys = CM.of_rowmajor(sd_.y_std)        # (ny x n)
    P = sd_.K.shape[0]
    KKt = gemm(True, False, K, K)         # (P x P) = K K^T
    lam = torch.diagonal(KKt.logical()).contiguous().clone()
    YK = gemm(True, False, Ys, K)         # (n x P) = y_std K^T
    ch = kernels.cholesky_inverse(KKt.t[:P, :P].reshape(1, P, P).contiguous())
    ch.check()
    Linv = CM(ch.linv_buf[0], P, P, ch.linv_buf.shape[1])
    T = gemm(False, True, YK, Linv)       # (n x P) = y_std K^T L^-T
    W = gemm(False, False, T, Linv)       # (n x P) = y_std K^T L^-T L^-1
    return W, lam


class EmulatorModel:
    """Mirror of the SepiaModel surface the reference uses (sim-only)."""

    param_names = ("betaU", "lamUz", "lamWs", "lamWOs")

    def __init__(self, data: EmulatorData):
        self.data = data
        sd_ = data.sim_data
        if sd_.K is None or sd_.y_std is None:
            raise ValueError("EmulatorModel needs standardised y and a K basis")
        self.device = data.device
        self.w_hat_cm, lam = pc_weights(data)          # (n x P) column-major
        self.LamSim = lam
        self.n, self.d = sd_.t_dev.shape
        self.P = sd_.K.shape[0]
        # GPMSA default starting values, priors and steps (see gladsgp_amd.mcmc)
        self.params = ModelParams(self.d, self.P)
        self.samples = None
        self.rng = np.random.default_rng()

    # ---------------------------------------------------------------------------- sampling
    def _sampler(self) -> mcmc.GPUSampler:
        return mcmc.GPUSampler(self.data.sim_data.t_dev, self.w_hat.transpose(0, 1).contiguous(),
                               self.LamSim, self.params)

    def tune_step_sizes(self, n_burn, n_levels, prog=False, diagnostics=False,
                        update_vals=True):
        """SEPIA tune_step_sizes (src/model.py:234): per-element Metropolis step sizes from
        n_levels x n_burn sweeps on the GPU (algorithm: gladsgp_amd.mcmc module doc)."""
        sm = self._sampler()
        mcmc.tune_step_sizes(sm, int(n_burn), int(n_levels), self.rng)
        self.tune_info = sm.last_tune
        if diagnostics:
            for k, a in sm.last_tune["accepts"].items():
                print(f"tune {k}: acceptance per level (rows = step scale "
                      f"{sm.last_tune['scales'].tolist()}):\n{a / n_burn}")
        if update_vals:
            sm.write_back()

    def do_mcmc(self, nsamp, prog=False, do_propMH=True, no_init=False):
        """SEPIA do_mcmc (src/model.py:235): ``nsamp`` component-wise Metropolis sweeps on the
        GPU, appended to ``samples`` (betaU (N, (d+1) P), lamUz/lamWs (N, P), lamWOs (N, 1),
        logPost (N, 1)); the last state becomes the current parameter values."""
        sm = self._sampler()
        new = sm.run(int(nsamp), self.rng)
        sm.write_back()
        if self.samples is None:
            self.samples = new
        else:
            self.samples = {k: np.concatenate([self.samples[k], new[k]]) for k in new}

    @property
    def w_hat(self) -> torch.Tensor:
        """(n, P) PC weights of the training runs."""
        return self.w_hat_cm.logical()

    # ---------------------------------------------------------------------------------- I/O
    def set_samples(self, samples: dict):
        self.samples = {k: np.asarray(v, dtype=np.float64) for k, v in samples.items()}

    def get_samples(self, numsamples=None, nburn=0):
        """Posterior samples after ``nburn``, optionally ``numsamples`` evenly spaced."""
        if self.samples is None:
            raise ValueError("model has no MCMC samples (restore_model_info or set_samples)")
        tot = len(self.samples["lamUz"])
        idx = np.arange(nburn, tot)
        if numsamples is not None and numsamples < len(idx):
            idx = idx[np.linspace(0, len(idx) - 1, numsamples).astype(int)]
        return {k: v[idx] for k, v in self.samples.items()}

    def save_model_info(self, path):
        """Samples, current values and step sizes as ``path + '.npz'`` (plain arrays,
        gladsgp_amd.modelio)."""
        modelio.save_model_npz(path, self.samples,
                               {k: getattr(self.params, k).val for k in ModelParams.names},
                               {k: getattr(self.params, k).mcmcStepParam
                                for k in ModelParams.names})

    def restore_model_info(self, path):
        """Read ``path + '.npz'`` written by save_model_info or by
        tools/export_sepia_samples.py from a SEPIA fit (gladsgp_amd.modelio)."""
        samples, params, steps = modelio.load_model_npz(path)
        for k, v in params.items():
            self.params[k] = v
        for k, v in steps.items():
            p = getattr(self.params, k)
            p.mcmcStepParam = np.broadcast_to(v, p.val_shape).copy()
        self.samples = samples or None

    # ------------------------------------------------------------------------- likelihood
    def log_likelihood(self, params=None) -> float:
        """Sum over PCs of the Gaussian log-likelihood of w_hat_j (no 2pi term, no priors).

        Building block of SEPIA's logLik for the sim-only model (driven by do_mcmc,
        src/model.py:234-235): one batched Gram -> Cholesky -> nll over the P GPs.
        """
        pr = self.params.values() if params is None else params
        samples = {k: np.asarray(pr[k]).reshape(1, -1) for k in self.param_names}
        beta, s, delta, _ = gp_params(samples, _np(self.LamSim), self.d, self.P, False)
        X = self.data.sim_data.t_dev
        G = kernels.gram(X, torch.as_tensor(beta[0], device=self.device),
                         torch.as_tensor(s[0], device=self.device),
                         torch.as_tensor(delta[0], device=self.device), batch=self.P)
        ch = kernels.cholesky_inverse(G)
        ch.check()
        w = self.w_hat.transpose(0, 1).contiguous()           # (P, n)
        return -float(kernels.nll(ch, w).sum().item())


def gp_params(samples, LamSim, d, P, pred_nugget=True):
    """Per (sample, PC) kernel parameters: beta (S, P, d), s, delta, s_pred (S, P).

    Parameter marshalling only (host, O(S P d)): the covariance arithmetic is in libgpfit.
    """
    bu = np.asarray(samples["betaU"], dtype=np.float64)
    S = bu.shape[0]
    beta = bu.reshape(S, d + 1, P)[:, 1:, :].transpose(0, 2, 1).copy()
    lamUz = np.asarray(samples["lamUz"], dtype=np.float64).reshape(S, P)
    lamWs = np.asarray(samples["lamWs"], dtype=np.float64).reshape(S, P)
    lamWOs = np.asarray(samples["lamWOs"], dtype=np.float64).reshape(S, 1)
    lam = np.asarray(LamSim, dtype=np.float64).reshape(1, P)
    s = 1.0 / lamUz
    delta = 1.0 / lamWs + 1.0 / (lamWOs * lam)
    s_pred = s + (1.0 / lamWs if pred_nugget else 0.0)
    return beta, s, delta, s_pred


def predict_units(X, Xs, w_units, beta_u, s_u, delta_u, sp_u, budget_bytes=2 << 30,
                  m_chunk=0, group=None, fctx: kernels.FitPredictContext | None = None,
                  workspace: kernels.PredictWorkspace | None = None):
    """Posterior mean / variance of a list of GPs sharing X and Xs: returns (U, m) x 2.

    Units are processed in groups bounded by ``budget_bytes`` of Gram + L^-1 storage, and by
    ``group`` GPs per group when given; each group is one gp_fit_predict (batched Gram ->
    factorisation -> cross-covariance / TRMM / mean + variance), whose cross-covariance runs on
    ``fctx``'s own stream beside the factorisation when a context is given (bit-identical to
    gram -> potrf -> predict on one stream: tests/test_gpu_c4.py).
    """
    dev = X.device
    U = beta_u.shape[0]
    n = X.shape[0]
    m = Xs.shape[0]
    npad = kernels.padded_n(n)
    per = 8 * (n * n + npad * npad)
    g = max(1, int(budget_bytes // per))
    if group is not None:
        g = max(1, min(g, int(group)))
    mean = torch.empty((U, m), dtype=F64, device=dev)
    var = torch.empty((U, m), dtype=F64, device=dev)
    ws = workspace if workspace is not None else kernels.PredictWorkspace()
    for a in range(0, U, g):
        b = min(U, a + g)
        kernels.fit_predict(X, Xs, beta_u[a:b], s_u[a:b], delta_u[a:b], sp_u[a:b],
                            w_units[a:b], m_chunk=m_chunk, workspace=ws,
                            out=(mean[a:b], var[a:b]), ctx=fctx, check=True)
    return mean, var


class EmulatorPrediction:
    """Predictions of the P PC-GPs for each posterior sample at ``t_pred`` (m x d).

    ``ctx`` (a :class:`gladsgp_amd.dist.Context`) shards the work over ranks; rank 0 receives
    the gathered (S, m, P) results, other ranks hold ``None``:
      * units (S P) >= ranks: the (sample, PC) units are dealt round-robin (SURVEY §8e,
        multivariate emulator);
      * fewer units than ranks (the reference's scalar GPs: P = 1 with few samples,
        fit_scalar_models.py:477-481, mean_response.py:114-126) with m >= ranks: the test points
        are split instead, every rank predicting every unit on its contiguous block
        (``shard="points"``, SURVEY §8e single-output GP; see gladsgp_amd.sharded).
    ``shard`` forces "units" or "points".  ``group`` caps the GPs per batched factorisation.
    ``fctx`` / ``workspace``: a caller-owned gp_fit_predict context (cross-covariance beside the
    factorisation) and prediction workspace, reused across calls.
    """

    def __init__(self, model: EmulatorModel = None, samples: dict = None, t_pred=None,
                 pred_nugget: bool = True, ctx: gdist.Context | None = None,
                 budget_bytes: int = 2 << 30, m_chunk: int = 0, realize: bool = False,
                 seed: int | None = None, group: int | None = None, shard: str | None = None,
                 fctx: kernels.FitPredictContext | None = None,
                 workspace: kernels.PredictWorkspace | None = None):
        if model is None or samples is None or t_pred is None:
            raise ValueError("EmulatorPrediction needs model, samples and t_pred")
        self.model = model
        dev = model.device
        X = model.data.sim_data.t_dev
        Xs = (t_pred.to(device=dev, dtype=F64) if torch.is_tensor(t_pred) else
              torch.as_tensor(np.asarray(t_pred), dtype=F64, device=dev))
        Xs = Xs.reshape(-1, model.d).contiguous()
        beta, s, delta, sp = gp_params(samples, _np(model.LamSim), model.d, model.P,
                                       pred_nugget)
        S, P = s.shape
        self.S, self.m, self.P = S, Xs.shape[0], P
        self.lamWOs = np.asarray(samples["lamWOs"], dtype=np.float64).reshape(S)
        units = [(a, j) for a in range(S) for j in range(P)]
        dist_on = ctx is not None and ctx.distributed
        rank, world = (ctx.rank, ctx.world) if dist_on else (0, 1)
        if shard is None:
            shard = "points" if (dist_on and len(units) < world and self.m >= world) else "units"
        if shard not in ("units", "points"):
            raise ValueError(f"shard must be 'units' or 'points', got {shard!r}")
        self.shard = shard if dist_on else "units"
        w_hat = model.w_hat.transpose(0, 1).contiguous()       # (P, n)
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=F64, device=dev)  # noqa
        if self.shard == "points":
            # every unit on this rank's contiguous block of the test points
            lo, hi = gdist.shard_range(self.m, rank, world)
            sel_s = np.array([u[0] for u in units])
            sel_j = np.array([u[1] for u in units])
            jj = torch.as_tensor(sel_j, device=dev)
            mean_l, var_l = predict_units(X, Xs[lo:hi].contiguous(), w_hat[jj].contiguous(),
                                          t(beta[sel_s, sel_j]), t(s[sel_s, sel_j]),
                                          t(delta[sel_s, sel_j]), t(sp[sel_s, sel_j]),
                                          budget_bytes, m_chunk, group, fctx, workspace)
        else:
            mine = gdist.shard_units(len(units), rank, world)
            if mine:
                sel_s = np.array([units[u][0] for u in mine])
                sel_j = np.array([units[u][1] for u in mine])
                jj = torch.as_tensor(sel_j, device=dev)
                mean_l, var_l = predict_units(X, Xs, w_hat[jj].contiguous(),
                                              t(beta[sel_s, sel_j]), t(s[sel_s, sel_j]),
                                              t(delta[sel_s, sel_j]), t(sp[sel_s, sel_j]),
                                              budget_bytes, m_chunk, group, fctx, workspace)
            else:
                mean_l = torch.empty((0, self.m), dtype=F64, device=dev)
                var_l = torch.empty((0, self.m), dtype=F64, device=dev)
        self.ctx = ctx
        self.realized = bool(realize)
        self.seed = int(np.random.SeedSequence().entropy & (2 ** 63 - 1)) if seed is None \
            else int(seed)
        self._w_dtype = np.dtype(np.float64)
        if self.shard == "points":
            both = assemble_points(ctx, mean_l, var_l, self.m)
        else:
            both = assemble_units(ctx, mean_l, var_l, len(units))
        if both is None:
            self.mean_dev = self.w_dev = self.var_dev = None
            return
        mean_u, var_u = both
        # units are (s, j) in s-major order -> (S, P, m) -> (S, m, P)
        self.mean_dev = mean_u.reshape(S, P, self.m).permute(0, 2, 1).contiguous()
        self.var_dev = var_u.reshape(S, P, self.m).permute(0, 2, 1).contiguous()
        self.w_dev = (kernels.realize(self.mean_dev, self.var_dev, self.seed) if self.realized
                      else self.mean_dev)

    @property
    def w(self) -> np.ndarray:
        """(S, m, P) PC weights as the reference consumes ``.w`` (numpy): the posterior mean,
        or one marginal draw per entry with ``realize=True``, or whatever was assigned."""
        return None if self.w_dev is None else self.w_dev.cpu().numpy().astype(self._w_dtype,
                                                                              copy=False)

    @w.setter
    def w(self, value) -> None:
        """Assign the PC weights ``get_y()`` reconstructs from (the reference casts them with
        ``preds.w = preds.w.astype(np.float32)`` first): kept on the device as float64 copies of
        the assigned values; ``get_y()`` returns the assigned dtype."""
        a = np.asarray(value) if not torch.is_tensor(value) else value
        if tuple(a.shape) != (self.S, self.m, self.P):
            raise ValueError(f"w: expected shape {(self.S, self.m, self.P)}, got {tuple(a.shape)}")
        self._w_dtype = np.dtype(a.dtype if not torch.is_tensor(a) else
                                 torch.empty((), dtype=a.dtype).numpy().dtype)
        self.w_dev = _to_device_f64(a, self.model.device)

    @property
    def mean(self) -> np.ndarray:
        """(S, m, P) posterior mean of the PC weights."""
        return None if self.mean_dev is None else self.mean_dev.cpu().numpy()

    @property
    def var(self) -> np.ndarray:
        return None if self.var_dev is None else self.var_dev.cpu().numpy()

    def get_mu_sigma(self):
        return self.mean, self.var

    def sample_w(self, seed: int | None = None, offset: int = 1) -> np.ndarray:
        """A fresh marginal realisation per (sample, point, PC), mean + sqrt(var) N(0, 1), on
        the device (gp_realize; ``offset`` selects an independent stream for one seed)."""
        seed = self.seed if seed is None else int(seed)
        return kernels.realize(self.mean_dev, self.var_dev, seed, offset).cpu().numpy()

    def error_draws(self, rng=None, per_point: bool = True) -> np.ndarray:
        """Standardised residual error of the reference's predictions: one N(0, 1/sqrt(lamWOs_s))
        draw per posterior sample s (``time_predictions.py:84-87``) or per (sample, test point)
        (``per_point``, ``assess_all_models.py:493-497``), shape (S, m) / (S, 1).  The
        reference scales it by sd_y in physical units; get_y(add_error=True) does the same."""
        rng = np.random.default_rng() if rng is None else rng
        cols = self.m if per_point else 1
        return rng.standard_normal((self.S, cols)) / np.sqrt(self.lamWOs)[:, None]

    def get_y(self, std: bool = False, w=None, add_error: bool = False, rng=None,
              per_point: bool = True, ctx="inherit", gather: bool = True,
              to_host: bool = True):
        """Field reconstruction y = (w K) sd + mu, shape (S, m, ny) — SEPIA get_y().

        ``add_error`` adds the reference's PC-truncation error term (error_draws, times sd_y
        in physical units): y = (w K + e) sd + mu, one scalar e per (sample[, point]).

        Distributed (``ctx``, by default the prediction's; SURVEY §8e "field reconstruction"):
        rank 0's w (and error draws) are broadcast, rank r reconstructs the output columns
        ``shard_range(ny, r, N)`` with its slice of K, and with ``gather`` rank 0 receives the
        whole (S, m, ny) field (other ranks None); ``gather=False`` returns every rank's own
        (S, m, ny_r) column block (``self.y_cols`` holds its range).

        ``to_host=False`` returns the device tensor instead of numpy (no PCIe copy).  With at
        most gp_field_max_pcs() PCs the product, error term, back-transform and narrowing are
        one kernel (gp_field: every output element written once, in its final dtype).
        """
        sd_ = self.model.data.sim_data
        dev = self.model.device
        ctx = self.ctx if isinstance(ctx, str) else ctx
        dist_on = ctx is not None and ctx.distributed
        S, m, P = self.S, self.m, self.P
        if dist_on:
            flag = torch.tensor([1 if self._w_dtype == np.float32 else 0], device=dev)
            gdist.broadcast_(ctx, flag)
            f32 = bool(flag.item()) and w is None
            if ctx.rank == 0:
                wd = (self.w_dev if w is None else _to_device_f64(w, dev)).contiguous()
            else:
                wd = torch.empty((S, m, P), dtype=F64, device=dev)
            gdist.broadcast_(ctx, wd)
            ny = sd_.K.shape[1]
            c0, c1 = gdist.shard_range(ny, ctx.rank, ctx.world)
        else:
            f32 = w is None and self._w_dtype == np.float32
            wd = self.w_dev if w is None else _to_device_f64(w, dev)
            c0, c1 = 0, sd_.K.shape[1]
        out_dtype = np.float32 if f32 else np.float64
        self.y_cols = (c0, c1)
        e = None
        if add_error:
            cols = m if per_point else 1
            if not dist_on or ctx.rank == 0:
                e = torch.as_tensor(self.error_draws(rng, per_point), dtype=F64, device=dev)
            else:
                e = torch.empty((S, cols), dtype=F64, device=dev)
            if dist_on:
                gdist.broadcast_(ctx, e)
            e = (e.expand(S, m) if e.shape[1] == 1 else e).reshape(S * m).contiguous()
        mu = sd = None
        if not std:
            mu, sd = sd_.y_mean[c0:c1].contiguous(), sd_.y_sd[c0:c1].contiguous()
        w2 = wd.reshape(S * m, P).contiguous()
        if P <= blas.field_max_pcs():
            # one pass: y = (w K + e) sd + mu, written once in the output dtype (K's column
            # block read in place through its row stride)
            y = blas.field(w2, sd_.K[:, c0:c1], sd, mu, e, f32=f32)
        else:
            K = sd_.K if (c0, c1) == (0, sd_.K.shape[1]) else sd_.K[:, c0:c1].contiguous()
            Wc = CM.of_rowmajor(w2)                              # (P x S m)
            Kc = CM.of_rowmajor(K)                               # (ny_r x P)
            Yc = gemm(False, False, Kc, Wc)                      # (ny_r x S m) = (w K)^T
            y = Yc.t[: S * m, : c1 - c0]                         # (S m, ny_r) row-major
            if e is not None:
                y = y + e.reshape(S * m, 1)                      # one scalar per row
            if not std:
                y = blas.standardize(y.contiguous(), mu, sd, inverse=True)
        if dist_on and gather:
            counts = [gdist.shard_range(sd_.K.shape[1], r, ctx.world) for r in range(ctx.world)]
            y = gdist.gather_cols(ctx, y.contiguous(), [b - a for a, b in counts])
            if y is None:
                return None
        if not to_host:
            return y.reshape(S, m, -1)
        return _to_host(y.reshape(S, m, -1), out_dtype)


def assemble_units(ctx, mean_l: torch.Tensor, var_l: torch.Tensor, n_units: int):
    """Gather per-rank (mean, var) rows of round-robin-dealt units back into unit order.

    Single process: identity.  Distributed: one gather to rank 0 (RCCL on GPUs, gloo on CPU);
    returns None on the other ranks.
    """
    if ctx is None or not ctx.distributed:
        return mean_l, var_l
    world = ctx.world
    m = mean_l.shape[1]
    counts = [len(gdist.shard_units(n_units, r, world)) for r in range(world)]
    both = torch.stack([mean_l, var_l], dim=1) if mean_l.shape[0] else \
        torch.empty((0, 2, m), dtype=mean_l.dtype, device=mean_l.device)
    allb = gdist.gather_rows(ctx, both, counts)
    if allb is None:
        return None
    allb = unit_order(allb, n_units, world)
    return allb[:, 0], allb[:, 1]


def assemble_points(ctx, mean_l: torch.Tensor, var_l: torch.Tensor, m: int):
    """Gather every rank's (U, m_r) test-point block of all units to rank 0 as (U, m) x 2
    (one gather; None on the other ranks)."""
    if ctx is None or not ctx.distributed:
        return mean_l, var_l
    counts = [b - a for a, b in (gdist.shard_range(m, r, ctx.world) for r in range(ctx.world))]
    both = torch.stack([mean_l, var_l], dim=0).contiguous()   # (2, U, m_r)
    allb = gdist.gather_cols(ctx, both, counts)
    if allb is None:
        return None
    return allb[0], allb[1]


def unit_order(rank_major: torch.Tensor, n_units: int, world: int) -> torch.Tensor:
    """Rows gathered rank by rank (rank r's round-robin units shard_units(n_units, r, world) in
    order) -> rows in unit order."""
    order = np.concatenate([gdist.shard_units(n_units, r, world) for r in range(world)])
    inv = np.empty_like(order)
    inv[order] = np.arange(len(order))
    return rank_major[torch.as_tensor(inv, device=rank_major.device)]


# SEPIA-compatible alias for drop-in call sites
SepiaEmulatorPrediction = EmulatorPrediction


def default_data_dir():
    return os.path.join(os.getcwd(), "data")
