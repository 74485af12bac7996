"""The chained emulator surface of BASELINE config 5 on device-resident inputs.

One :meth:`FieldPipeline.run` is the whole north-star surface, in the reference's order:

1. standardise the ensemble: mu, sd (ddof = 1, floored), y_std = (y - mu) / sd
   (``src/model.py:60-72``, ``plot_PC_RMSE.py:86-89``);
2. ``randomized_svd(y_std, p, k=0, q=1)`` (``plot_PC_RMSE.py:90-91``; ``src/model.py:84`` with
   p = 25), the test matrix drawn once by the caller exactly as ``src/svd.py:51`` draws it;
3. the PC basis ``K = diag(S) Vh / sqrt(n)`` (``src/model.py:101``) and SEPIA's PC weights
   ``w_hat = y_std pinv(K)``, ``LamSim = diag(K K^T)`` (:class:`EmulatorModel`);
4. ``SepiaEmulatorPrediction(model=, samples=, t_pred=)``: the S x P independent PC GPs
   (Gram -> Cholesky / L^-1 -> cross-covariance / TRMM -> mean + variance, one batched
   gp_fit_predict; ``assess_all_models.py:487-489``);
5. ``preds.w = preds.w.astype(float32); preds.get_y()`` -- the field (``assess_all_models.py:
   490-492``, ``time_predictions.py:78-79``), left on the device (gp_field).

Every array stays on the device; the only host work is the hyperparameter marshalling of
step 4 and the small eigen / Cholesky checks (a handful of synchronisations per run).

Multi-GPU (``ctx`` with world > 1): every rank runs steps 1-3 redundantly on the
ensemble rank 0 broadcast at setup (a few ms at C5, bit-identical on identical GPUs), the
(sample, PC) GPs are dealt round-robin with one gather of (mean, var) to rank 0
(:class:`EmulatorPrediction`), and the field is reconstructed in ny-column blocks after one
broadcast of w, each rank keeping its own block (``get_y(gather=False)``).
"""
from __future__ import annotations

import numpy as np
import torch

from . import dist as gdist
from . import kernels
from .emulator import EmulatorData, EmulatorModel, EmulatorPrediction
from .model import _scale_rows_tensor
from .svd import randomized_svd

F64 = torch.float64


class FieldPipeline:
    """Device-resident inputs and reusable scratch of the C5 chain.

    ``t`` (n x d) design, ``y`` (n x ny) ensemble (float32 like the reference's fit dtype, or
    float64), ``omega`` (ny x p) the SVD's test matrix, ``samples`` a SEPIA-layout posterior
    sample dict, ``t_pred`` (m x d) test points -- host arrays or device tensors (copied to the
    device once, here)."""

    def __init__(self, t, y, omega, samples: dict, t_pred, p: int, device=None,
                 ctx: gdist.Context | None = None, m_chunk: int = 0, aux_chunks: int = 1,
                 field_f32: bool = True):
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        dev = self.device

        def up(a):
            if torch.is_tensor(a):
                return a.to(dev).contiguous()
            return torch.as_tensor(np.ascontiguousarray(a), device=dev)
        self.t = up(t).to(F64)
        self.y = up(y)
        self.omega = up(omega)
        self.t_pred = up(t_pred).to(F64)
        self.samples = {k: np.asarray(v, dtype=np.float64) for k, v in samples.items()}
        self.p = int(p)
        self.ctx = ctx
        self.m_chunk = int(m_chunk)
        self.field_f32 = bool(field_f32)
        self.fctx = kernels.FitPredictContext(dev, aux_chunks=aux_chunks)
        self.ws = kernels.PredictWorkspace()
        self.events = None

    def close(self) -> None:
        self.fctx.close()

    def _mark(self, name: str) -> None:
        if self.events is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.events.append((name, ev))

    def run(self) -> dict:
        """One pass of the chain; returns the device results (``y`` is this rank's field block:
        all of it on one GPU)."""
        n = self.t.shape[0]
        self._mark("start")
        data = EmulatorData(t_sim=self.t, y_sim=self.y, device=self.device)
        data.standardize_y()                                     # model.py:60-72
        self._mark("standardize")
        U, S, Vh = randomized_svd(data.sim_data.y_std, self.p, k=0, q=1, omega=self.omega)
        self._mark("svd")
        S64, Vh64 = S.to(F64), Vh.to(F64)
        K = Vh64.contiguous().clone()
        _scale_rows_tensor(K, (S64 / np.sqrt(n)).contiguous())   # model.py:101
        K = K.to(torch.float32).to(F64)                          # create_K_basis(K.astype(f32))
        data.create_K_basis(K)
        model = EmulatorModel(data)                              # w_hat, LamSim
        self._mark("basis")
        pred = EmulatorPrediction(model=model, samples=self.samples, t_pred=self.t_pred,
                                  ctx=self.ctx, m_chunk=self.m_chunk, fctx=self.fctx,
                                  workspace=self.ws)
        self._mark("predict")
        y = None
        if pred.w_dev is not None or (self.ctx is not None and self.ctx.distributed):
            if pred.w_dev is not None and self.field_f32:
                pred.w = pred.w_dev.to(torch.float32)            # preds.w.astype(np.float32)
            y = pred.get_y(gather=False, to_host=False)
        self._mark("get_y")
        return {"U": U, "S": S, "Vh": Vh, "K": K, "w_hat": model.w_hat, "LamSim": model.LamSim,
                "mean": pred.mean_dev, "var": pred.var_dev, "y": y,
                "y_cols": getattr(pred, "y_cols", None), "model": model, "pred": pred}


def synthetic_c5(n: int = 512, d: int = 8, ny: int = 10_000, m: int = 100_000, p: int = 64,
                 samples: int = 1, modes: int = 96, seed: int = 5):
    """SURVEY §8d C5 inputs, seeded: the reference's 512 x 8 training design (its own recipe,
    ``scipy.stats.qmc.Sobol(8, seed=20240318)``, which regenerates
    ``experiments/synthetic/expdesign/synthetic_train_standard.csv`` to 6e-7: tests/test_oracle.py),
    a float32 field ``Y (n x ny)`` = smooth functions of the design (sin(2 pi t a_k + k)) times
    ``modes`` fixed space modes with geometrically decaying weight (0.93^k: the leading ``p``
    singular values stay separated, so the PCs are determined, not noise) + 1e-3 noise, the
    SVD's test matrix drawn exactly as ``src/svd.py:51`` draws it after ``np.random.seed(0)``,
    ``samples`` SEPIA-layout posterior samples in GPMSA-typical ranges, and ``m`` test points
    ``default_rng(2).random((m, d))``.  Returns (t, Y, omega, samples, t_pred)."""
    from scipy.stats import qmc
    t = qmc.Sobol(d, seed=20240318, optimization=None).random(n) if n == 512 and d == 8 \
        else np.random.default_rng(0).random((n, d))
    rng = np.random.default_rng(seed)
    amp = 0.93 ** np.arange(modes)
    M = (rng.standard_normal((modes, ny)) * amp[:, None]).astype(np.float32)
    coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, d) + k) for k in range(modes)], 1)
    Y = coef.astype(np.float32) @ M
    Y += 1e-3 * rng.standard_normal(Y.shape, dtype=np.float32)
    state = np.random.get_state()
    np.random.seed(0)
    omega = np.random.normal(size=(ny, p)).astype(np.float32)     # src/svd.py:51
    np.random.set_state(state)
    srng = np.random.default_rng(seed + 1)
    smp = {"betaU": srng.uniform(0.2, 3.0, (samples, (d + 1) * p)),
           "lamUz": srng.uniform(0.5, 3.0, (samples, p)),
           "lamWs": srng.uniform(200.0, 3000.0, (samples, p)),
           "lamWOs": srng.uniform(50.0, 500.0, (samples, 1))}
    t_pred = np.random.default_rng(2).random((m, d))
    return t, Y, omega, smp, t_pred
