"""GPU: the reference's own call sequences run unchanged against the drop-in surface.

* ``time_predictions.py:76-87`` and ``assess_all_models.py:489-500``: build a prediction,
  ``preds.w = preds.w.astype(np.float32)``, ``preds.get_y()``, add the PC-truncation error
  draws, take quantiles — restated statement by statement below;
* the opt-in ``realize=True`` mode (one marginal draw per (sample, point, PC) on the device,
  gp_realize / Philox4x32-10) against the numpy restatement ``oracle/rng_ref``;
* the GPmodule MLE surface of BASELINE config 1 (``examples/02...ipynb`` cell 5): the notebook
  known answer (n = 5) and C1 (n = 64) against ``oracle.gp_ref.fit_gpmodule``.

Tolerances: float32-cast reconstructions rtol 1e-6 (the cast itself); realisations
1e-12 * scale (libm vs ocml log / sincos); MLE optimum |d fun| <= 1e-8 |fun|, theta 1e-4
relative (two BFGS runs over objectives that agree to ~1e-13); predictor / error 1e-8.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import gp_ref, rng_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def _ensemble(n=64, ny=700, d=6, seed=2):
    rng = np.random.default_rng(seed)
    t = rng.random((n, d))
    modes = rng.standard_normal((5, ny)) * (0.5 ** np.arange(5))[:, None]
    coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, d) + k) for k in range(5)], 1)
    y = (3.0 + coef @ modes + 1e-2 * rng.standard_normal((n, ny))).astype(np.float32)
    return t.astype(np.float32), y


def _samples(S, d, P, seed=1):
    rng = np.random.default_rng(seed)
    return {"betaU": rng.uniform(0.2, 3.0, (S, (d + 1) * P)),
            "lamUz": rng.uniform(0.5, 3.0, (S, P)),
            "lamWs": rng.uniform(200, 3000, (S, P)),
            "lamWOs": rng.uniform(50, 500, (S, 1))}


@pytest.fixture(scope="module")
def fitted(dev, tmp_path_factory):
    from gladsgp_amd import model as gm
    t, y = _ensemble()
    p = 4
    data, model = gm.init_model(t, y, "dropin", p, data_dir=str(tmp_path_factory.mktemp("d")),
                                device=dev, verbose=False)
    return t, y, data, model, p


def test_time_predictions_sequence(fitted):
    """time_predictions.py:55-87 restated: samples cast to float32, one test point at a time,
    preds.w cast to float32, get_y(), error draws per sample, y = emulator + error."""
    from gladsgp_amd.emulator import SepiaEmulatorPrediction
    t, y, data, model, p = fitted
    dtype = np.float32
    samples = _samples(5, t.shape[1], p)
    for key in samples.keys():                                   # :54-55
        samples[key] = samples[key].astype(dtype)
    n = model.data.sim_data.y.shape[1]                           # :63
    mu_y = np.mean(model.data.sim_data.y, axis=0)                # :64
    sd_y = np.std(model.data.sim_data.y, ddof=1, axis=0)         # :65
    sd_y[sd_y < 1e-6] = 1e-6
    assert n == y.shape[1] and model.data.sim_data.y.dtype == np.float32
    t_test_std = np.random.default_rng(3).random((3, t.shape[1])).astype(dtype)
    K = data.sim_data.K.cpu().numpy()
    mu = data.sim_data.y_mean.cpu().numpy()
    sd = data.sim_data.y_sd.cpu().numpy()
    np.testing.assert_allclose(mu_y, mu, rtol=1e-6)
    for i in range(t_test_std.shape[0]):
        xi = t_test_std[i:i + 1]
        preds = SepiaEmulatorPrediction(samples=samples, model=model, t_pred=xi)   # :76-77
        preds.w = preds.w.astype(dtype)                                          # :78
        emulator_preds = preds.get_y()                                           # :79
        error_preds = np.zeros(emulator_preds.shape, dtype=np.float32)           # :86-87
        for j in range(error_preds.shape[0]):
            error_preds[j] = sd_y * np.random.normal(
                scale=1 / np.sqrt(samples['lamWOs'][j])).astype(np.float32)
        y_preds = emulator_preds + error_preds                                   # :90
        assert emulator_preds.dtype == np.float32 and y_preds.shape == (5, 1, n)
        w32 = preds.w
        assert w32.dtype == np.float32
        y_ref = gp_ref.reconstruct_y(w32.astype(np.float64), K, mu, sd)
        np.testing.assert_allclose(emulator_preds, y_ref, rtol=1e-6,
                                   atol=1e-6 * np.abs(y_ref).max())
        # the cast values are what get_y reconstructs from (not the float64 mean)
        mean_r, _ = gp_ref.sepia_predict_w(t.astype(np.float64), xi.astype(np.float64),
                                           model.w_hat.cpu().numpy(),
                                           {k: v.astype(np.float64) for k, v in samples.items()},
                                           model.LamSim.cpu().numpy())
        np.testing.assert_allclose(w32, mean_r, rtol=1e-6, atol=1e-6 * np.abs(mean_r).max())


def test_assess_all_models_sequence_with_realisations(fitted):
    """assess_all_models.py:476-500 restated on a batch of 4 test points, with the opt-in
    realize mode so the quantile interval carries the GP's predictive spread."""
    from gladsgp_amd.emulator import SepiaEmulatorPrediction
    t, y, data, model, p = fitted
    dtype = np.float32
    quantile = 0.025
    samples = _samples(64, t.shape[1], p, seed=4)
    for key in samples.keys():
        samples[key] = samples[key].astype(dtype)
    sd_y = np.std(model.data.sim_data.y, ddof=1, axis=0)
    sd_y[sd_y < 1e-6] = 1e-6
    tj_pred = np.random.default_rng(5).random((4, t.shape[1]))
    for realize in (False, True):
        np.random.seed(0)                  # the same error draws for both intervals
        preds = SepiaEmulatorPrediction(t_pred=tj_pred, samples=samples, model=model,
                                        realize=realize, seed=1234)
        preds.w = preds.w.astype(np.float32)
        ypreds = preds.get_y()
        error_preds = np.zeros(ypreds.shape, dtype=np.float32)
        for l_pred in range(4):
            for l_sample in range(error_preds.shape[0]):
                err_sd = 1 / np.sqrt(samples['lamWOs'][l_sample])
                error_preds[l_sample][l_pred] = sd_y * np.random.normal(scale=err_sd)
        ypred_mean = np.mean(ypreds, axis=0)
        lq = np.quantile(ypreds + error_preds, quantile, axis=0)
        uq = np.quantile(ypreds + error_preds, 1 - quantile, axis=0)
        assert ypred_mean.shape == (4, y.shape[1]) and np.all(uq >= lq)
        if realize:
            # .w is mean + sqrt(var) z with z from Philox(seed) — exactly the restatement
            w_ref = rng_ref.realize(preds.mean, preds.var, 1234)
            np.testing.assert_allclose(preds.w, w_ref.astype(np.float32), rtol=1e-6,
                                       atol=1e-6 * np.abs(w_ref).max())
            width_real = np.mean(uq - lq)
        else:
            width_mean = np.mean(uq - lq)
    # with the predictive variance in the draws the interval cannot be narrower on average
    assert width_real >= width_mean * 0.999


def test_realize_matches_restatement(dev):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(0)
    N = 100_003
    mean = rng.standard_normal(N)
    var = rng.uniform(0, 2, N)
    var[::97] = -1e-16                     # tiny negative variances (rounding) clamp to 0
    out = kernels.realize(torch.as_tensor(mean, device=dev), torch.as_tensor(var, device=dev),
                          seed=2 ** 40 + 7, offset=5).cpu().numpy()
    ref = rng_ref.realize(mean, var, 2 ** 40 + 7, 5)
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-12 * np.abs(ref).max())
    z = (out - mean)[var > 0] / np.sqrt(var[var > 0])
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1) < 0.02
    assert np.all(out[::97] == mean[::97])
    # in place (out aliases mean)
    m_t = torch.as_tensor(mean, device=dev).clone()
    kernels.realize(m_t, torch.as_tensor(var, device=dev), seed=2 ** 40 + 7, offset=5, out=m_t)
    np.testing.assert_array_equal(m_t.cpu().numpy(), out)


def test_w_setter_validates_and_feeds_get_y(fitted):
    from gladsgp_amd.emulator import EmulatorPrediction
    t, y, data, model, p = fitted
    samples = _samples(2, t.shape[1], p)
    pred = EmulatorPrediction(model=model, samples=samples, t_pred=t[:3].astype(np.float64))
    with pytest.raises(ValueError):
        pred.w = np.zeros((2, 3, p + 1))
    w0 = np.zeros((2, 3, p))
    pred.w = w0
    y0 = pred.get_y()
    assert y0.dtype == np.float64
    np.testing.assert_allclose(y0, np.broadcast_to(data.sim_data.y_mean.cpu().numpy(),
                                                   y0.shape), rtol=1e-14, atol=1e-12)


def test_gpmodule_notebook_known_answer(dev, golden_dir):
    """examples/02 cell 5 on the GPU: fun = -3.989954265337257 at x = [0.4093, 0.2270]."""
    from gladsgp_amd import gpmodule as GPmodule
    ka = json.load(open(os.path.join(golden_dir, "nb02_known_answer.json")))
    x = np.vstack(np.linspace(1 / 8, 7 / 8, 5))
    xpred = np.vstack(np.linspace(0, 1, 51))
    f = lambda x: x * np.sin(2 * np.pi * x)  # noqa: E731
    y = f(x)
    GPmodel = GPmodule.GP(covariance=GPmodule.squared_exponential, cov_para={'nugget': 1e-3})
    x0 = np.array([1, 0.5])
    GPmodel.fit(x, y, x0)
    res = GPmodel.minimize_res
    assert res.success
    assert abs(res.fun - ka["printed_fun"]) <= 1e-7
    np.testing.assert_allclose(np.abs(res.x), ka["printed_x"], atol=1e-3)
    ypred = GPmodel.predictor(xpred)
    epred = GPmodel.error(xpred)
    assert ypred.shape == (51,) and epred.shape == (51,)
    s, beta, delta = gp_ref.gpmodule_theta_to_kernel(np.abs(res.x), 1e-3)
    mr, vr = gp_ref.predict(x, xpred, y.ravel(), beta, s, delta, s_pred=s)
    np.testing.assert_allclose(ypred, mr, rtol=0, atol=1e-8)
    np.testing.assert_allclose(epred, np.sqrt(np.maximum(vr, 0)), rtol=0, atol=1e-7)
    # cell 9: covariance(), K, K_inv at the fitted theta
    Kvec = GPmodel.covariance(xpred, x, GPmodel.theta)
    assert Kvec.shape == (51, 5) and GPmodel.K.shape == (5, 5)
    post_mean = Kvec @ GPmodel.K_inv @ y
    np.testing.assert_allclose(post_mean.ravel(), ypred, atol=1e-8)


def test_gpmodule_c1_fit(dev):
    """BASELINE config 1: x = linspace(1/8, 7/8, 64), y = x sin(2 pi x).

    At n = 64 with nugget 1e-3 the likelihood surface is ill-conditioned (kappa(K) ~ 1e8 near
    the optimum): BFGS's finite-difference gradients are noise-limited for numpy and GPU alike
    (both stop with 'precision loss' at different points), so the parity checks are
    (a) the objective on a theta grid, |dNLL| <= 1e-7 |NLL| (kappa eps), and (b) the same
    derivative-free optimiser (Nelder-Mead) on both objectives reaching the same optimum."""
    from gladsgp_amd import gpmodule as GPmodule
    x = np.vstack(np.linspace(1 / 8, 7 / 8, 64))
    y = x * np.sin(2 * np.pi * x)
    gp = GPmodule.GP(covariance=GPmodule.squared_exponential, cov_para={'nugget': 1e-3})
    gp.fit(x, y, np.array([1.0, 0.5]))          # the reference's call (BFGS): runs, finite
    assert np.isfinite(gp.minimize_res.fun) and gp.minimize_res.fun < 0
    for th0 in (0.3, 0.8, 1.5):
        for th1 in (0.05, 0.1, 0.2, 0.35):
            ref = gp_ref.nll_gpmodule(np.array([th0, th1]), x, y, 1e-3)
            got = gp.negloglik(np.array([th0, th1]))
            assert abs(got - ref) <= 1e-7 * max(1.0, abs(ref)), (th0, th1, got, ref)
    # fatol 1e-6 on |NLL| ~ 400: the objective itself is only kappa-eps (~1e-8 relative) exact,
    # so a simplex whose values must agree to 1e-9 absolute can stall on rounding noise
    opts = dict(xatol=1e-6, fatol=1e-6, maxiter=4000)
    gp.fit(x, y, np.array([1.0, 0.5]), method="Nelder-Mead", options=opts)
    import scipy.optimize as sopt
    ref = sopt.minimize(gp_ref.nll_gpmodule, np.array([1.0, 0.5]), args=(x, y, 1e-3),
                        method="Nelder-Mead", options=opts)
    assert gp.minimize_res.success and ref.success
    assert abs(gp.minimize_res.fun - ref.fun) <= 1e-7 * abs(ref.fun)
    np.testing.assert_allclose(np.abs(gp.theta), np.abs(ref.x), rtol=1e-3)
    xpred = np.vstack(np.linspace(0, 1, 101))
    s, beta, delta = gp_ref.gpmodule_theta_to_kernel(np.abs(gp.theta), 1e-3)
    mr, vr = gp_ref.predict(x, xpred, y.ravel(), beta, s, delta, s_pred=s)
    np.testing.assert_allclose(gp.predictor(xpred), mr, rtol=0, atol=1e-7)
    np.testing.assert_allclose(gp.error(xpred) ** 2, np.maximum(vr, 0), rtol=0, atol=1e-8)
