"""Host-side pieces of the Metropolis fit: step-size logistic regression, parameter surface,
and the oracle's likelihood restatement (no GPU)."""
import math

import numpy as np
import pytest
from scipy import stats

from gladsgp_amd import mcmc
from oracle import gp_ref, mcmc_ref


def test_logistic_step_recovers_target():
    # acceptance p(step) = sigmoid(b0 + b1 log step): the fit must return the 1/e step
    b0, b1 = 1.0, -1.5
    steps = 0.3 * 2.0 ** np.linspace(-2, 2, 5)
    p = 1.0 / (1.0 + np.exp(-(b0 + b1 * np.log(steps))))
    trials = 100000
    acc = np.round(p * trials)
    got = mcmc.logistic_step(np.log(steps), acc, trials, pseudo=0.0)
    want = math.exp((mcmc.TARGET_LOGIT - b0) / b1)
    assert abs(got / want - 1) < 1e-3     # the two unit-weight anchors barely move a 1e5 fit


def test_logistic_step_degenerate_levels():
    steps = np.log(np.array([0.1, 0.2, 0.4]))
    # everything accepted at every level: the anchors extrapolate beyond the ladder
    got = mcmc.logistic_step(steps, np.array([100, 100, 100]), 100)
    assert np.isfinite(got) and got > 0.4
    # nothing accepted: extrapolate below it
    got = mcmc.logistic_step(steps, np.array([0, 0, 0]), 100)
    assert np.isfinite(got) and got < 0.1
    # acceptance rising steeply with the step (wrong sign) -> a ladder value
    got = mcmc.logistic_step(steps, np.array([0, 50, 100]), 100)
    assert np.isclose(np.log(got), steps).any()


def test_model_params_surface():
    pr = mcmc.ModelParams(d=3, P=2)
    assert pr.betaU.val.shape == (4, 2) and pr.lamWOs.val.shape == (1, 1)
    # default step sizes pinned by examples/03...ipynb:192-208
    assert np.all(pr.betaU.mcmcStepParam == 0.1) and np.all(pr.lamUz.mcmcStepParam == 5)
    assert np.all(pr.lamWs.mcmcStepParam == 100) and np.all(pr.lamWOs.mcmcStepParam == 100)
    # the reference's override (src/model.py:225-229)
    pr.lamWOs = mcmc.SepiaParam(val=42.0, name="lamWOs", val_shape=(1, 1), dist="Gamma",
                                params=[50, 50 / 42.0], bounds=[1.0, np.inf],
                                mcmcStepParam=10, mcmcStepType="Uniform")
    assert pr["lamWOs"][0, 0] == 42.0 and pr.lamWOs.bounds == (1.0, np.inf)
    pr["lamUz"] = [[2.0, 3.0]]
    assert pr.values()["lamUz"].tolist() == [[2.0, 3.0]]
    with pytest.raises(ValueError):
        mcmc.SepiaParam(1.0, "x", (1, 1), dist="Cauchy")


def test_oracle_loglik_is_gaussian_logpdf():
    rng = np.random.default_rng(0)
    n, d, P = 40, 3, 2
    X = rng.random((n, d))
    w = rng.standard_normal((P, n))
    lam = np.array([3.0, 7.0])
    betaU = rng.uniform(0.5, 3, (d + 1, P))
    lamUz, lamWs, lamWOs = np.array([1.5, 0.7]), np.array([300.0, 900.0]), 120.0
    ll = mcmc_ref.loglik_pcs(X, w, lam, betaU, lamUz, lamWs, lamWOs)
    for j in range(P):
        G = gp_ref.gram_ardse(X, betaU[1:, j], 1 / lamUz[j], 1 / lamWs[j] + 1 / (lamWOs * lam[j]))
        ref = stats.multivariate_normal(np.zeros(n), G).logpdf(w[j]) + 0.5 * n * np.log(2 * np.pi)
        assert abs(ll[j] - ref) < 1e-9 * max(1.0, abs(ref))


def test_oracle_chain_moves_and_respects_bounds():
    rng = np.random.default_rng(1)
    n, d, P = 24, 2, 2
    X = rng.random((n, d))
    w = rng.standard_normal((P, n))
    lam = np.array([2.0, 5.0])
    pr = mcmc.ModelParams(d, P)
    spec = {k: (getattr(pr, k).dist, getattr(pr, k).params, getattr(pr, k).bounds,
                getattr(pr, k).mcmcStepType) for k in pr.names}
    state = {"betaU": pr.betaU.val, "lamUz": pr.lamUz.val[0], "lamWs": pr.lamWs.val[0],
             "lamWOs": pr.lamWOs.val[0, 0]}
    steps = {k: getattr(pr, k).mcmcStepParam for k in pr.names}
    U = rng.random((60, mcmc.uniforms_per_sweep(d, P)))
    st, rec, acc = mcmc_ref.run_chain(X, w, lam, spec, state, steps, U)
    assert rec["betaU"].shape == (60, (d + 1) * P) and rec["lamWOs"].shape == (60, 1)
    assert np.all(rec["lamUz"] >= 0.3) and np.all((rec["lamWs"] >= 60) & (rec["lamWs"] <= 1e5))
    assert np.all(rec["betaU"] >= 0)
    assert acc["lamUz"].sum() > 0 and acc["betaU"].sum() > 0


def test_restore_accepts_sepia_shaped_samples(tmp_path):
    """restore_model_info flattens SEPIA's (S,) + val_shape sample arrays (npz export)."""
    from gladsgp_amd.emulator import EmulatorModel
    S, d, P = 5, 3, 2
    rng = np.random.default_rng(0)
    bu = rng.random((S, d + 1, P))
    f = tmp_path / "m.npz"
    np.savez(f, samples_betaU=bu, samples_lamUz=rng.random((S, 1, P)),
             samples_lamWs=rng.random((S, 1, P)), samples_lamWOs=rng.random(S))
    m = EmulatorModel.__new__(EmulatorModel)       # I/O only: no data / device needed
    m.params = mcmc.ModelParams(d, P)
    m.restore_model_info(str(f))
    assert m.samples["betaU"].shape == (S, (d + 1) * P)
    np.testing.assert_array_equal(m.samples["betaU"].reshape(S, d + 1, P), bu)
    assert m.samples["lamUz"].shape == (S, P) and m.samples["lamWOs"].shape == (S, 1)
