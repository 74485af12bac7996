"""GPU Metropolis fit (gladsgp_amd.mcmc, gp_loglik) against the oracle restatement
(oracle/mcmc_ref.py) fed the same uniforms, and the fit_models -> load_model round trip."""
import os
import types

import numpy as np
import pytest
import torch

from gladsgp_amd import kernels, mcmc
from oracle import gp_ref, mcmc_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def _t(a, dev):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=dev)


def _problem(n, d, P, seed):
    rng = np.random.default_rng(seed)
    X = rng.random((n, d))
    lam = rng.uniform(1.0, 10.0, P)
    w = np.empty((P, n))
    for j in range(P):   # PC weights drawn from a GP so the chain has structure to find
        G = gp_ref.gram_ardse(X, rng.uniform(0.5, 4.0, d), 1.0, 1e-3)
        w[j] = np.linalg.cholesky(G) @ rng.standard_normal(n)
    return X, w, lam


@pytest.mark.parametrize("n,P", [(64, 3), (200, 5), (257, 2)])
def test_loglik_matches_oracle(dev, n, P):
    d = 4
    X, w, lam = _problem(n, d, P, seed=n)
    rng = np.random.default_rng(7)
    betaU = rng.uniform(0.2, 5.0, (d + 1, P))
    lamUz = rng.uniform(0.5, 3.0, P)
    lamWs = rng.uniform(100, 5000, P)
    lamWOs = 300.0
    ref = mcmc_ref.loglik_pcs(X, w, lam, betaU, lamUz, lamWs, lamWOs)
    ws = kernels.LoglikWorkspace(n, P, dev)
    beta = _t(betaU[1:].T, dev)
    s = _t(1.0 / lamUz, dev)
    delta = _t(1.0 / lamWs + 1.0 / (lamWOs * lam), dev)
    got = kernels.loglik(_t(X, dev), beta, s, delta, _t(w, dev), ws).cpu().numpy()
    tol = 1e-9 * np.maximum(1.0, np.abs(ref))
    assert np.all(np.abs(got - ref) <= tol), (got, ref)
    assert np.all(ws.info.cpu().numpy() == 0)


def test_loglik_non_pd_is_minus_inf(dev):
    n, d, P = 96, 2, 3
    X, w, lam = _problem(n, d, P, seed=3)
    beta = _t(np.full((P, d), 0.5), dev)
    s = _t([1.0, 1.0, 1.0], dev)
    delta = _t([1e-3, -5.0, 1e-3], dev)         # problem 1 is indefinite
    ws = kernels.LoglikWorkspace(n, P, dev)
    got = kernels.loglik(_t(X, dev), beta, s, delta, _t(w, dev), ws).cpu().numpy()
    assert np.isfinite(got[0]) and np.isfinite(got[2]) and got[1] == -np.inf
    assert ws.info.cpu().numpy()[1] > 0


def _spec(pr):
    return {k: (getattr(pr, k).dist, getattr(pr, k).params, getattr(pr, k).bounds,
                getattr(pr, k).mcmcStepType) for k in pr.names}


@pytest.mark.parametrize("n,d,P,steps_scale,graph,spec", [(48, 2, 3, 1.0, False, 1),
                                                          (48, 2, 3, 1.0, True, 1),
                                                          (48, 2, 3, 1.0, False, 2),
                                                          (48, 2, 3, 1.0, True, 3),
                                                          (130, 3, 2, 0.3, True, 2),
                                                          (130, 3, 2, 0.3, False, 3)])
def test_chain_matches_oracle(dev, n, d, P, steps_scale, graph, spec):
    """The oracle runs one update at a time; the sampler's speculative groups (spec updates per
    batched gp_loglik, 2^spec - 1 parameter states) must give the same chain."""
    X, w, lam = _problem(n, d, P, seed=11 + n)
    pr = mcmc.ModelParams(d, P)
    for k in pr.names:
        getattr(pr, k).mcmcStepParam = getattr(pr, k).mcmcStepParam * steps_scale
    sampler = mcmc.GPUSampler(_t(X, dev), _t(w, dev), _t(lam, dev), pr, use_graph=graph,
                              spec=spec)
    nsw = 25
    rec = sampler.run(nsw, np.random.default_rng(5))
    U = np.random.default_rng(5).random((nsw, mcmc.uniforms_per_sweep(d, P)))
    state = {"betaU": pr.betaU.val, "lamUz": pr.lamUz.val[0], "lamWs": pr.lamWs.val[0],
             "lamWOs": pr.lamWOs.val[0, 0]}
    steps = {k: getattr(pr, k).mcmcStepParam for k in pr.names}
    _, ref, acc = mcmc_ref.run_chain(X, w, lam, _spec(pr), state, steps, U)
    for k in ("betaU", "lamUz", "lamWs", "lamWOs"):
        np.testing.assert_allclose(rec[k], ref[k], rtol=1e-9, atol=1e-12, err_msg=k)
    assert acc["betaU"][1:].sum() > 0            # the chain actually moved
    assert np.all(np.isfinite(rec["logPost"]))


def test_tune_and_sample(dev):
    n, d, P = 80, 3, 2
    X, w, lam = _problem(n, d, P, seed=21)
    pr = mcmc.ModelParams(d, P)
    sampler = mcmc.GPUSampler(_t(X, dev), _t(w, dev), _t(lam, dev), pr)
    rng = np.random.default_rng(0)
    mcmc.tune_step_sizes(sampler, 20, 3, rng)
    for k in pr.names:
        stp = getattr(pr, k).mcmcStepParam
        assert np.all(np.isfinite(stp)) and np.all(stp > 0), k
    assert sampler.last_tune["accepts"]["lamUz"].shape == (3, P)
    rec = sampler.run(40, rng)
    assert rec["betaU"].shape == (40, (d + 1) * P)
    assert np.all(np.isfinite(rec["logPost"]))


def test_fit_models_roundtrip(dev, tmp_path):
    from gladsgp_amd import model as gmodel
    from gladsgp_amd.emulator import SepiaEmulatorPrediction
    rng = np.random.default_rng(4)
    n, ny, d = 40, 300, 3
    t = rng.random((n, d))
    modes = rng.standard_normal((4, ny))
    y = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, d) + k) for k in range(4)], 1) @ modes
    y = y + 1e-2 * rng.standard_normal((n, ny))
    xcsv = tmp_path / "X_std.csv"
    np.savetxt(xcsv, t, delimiter=",", header=",".join(f"x{i}" for i in range(d)), comments="")
    ynpy = tmp_path / "Y.npy"
    np.save(ynpy, y.T)                           # the reference stores (ny, n)
    cfg = types.SimpleNamespace(X_standard=str(xcsv), Y_physical=str(ynpy),
                                data_dir=str(tmp_path), exp="toy")
    models = gmodel.fit_models(cfg, [n], [3], dtype=np.float64, device=dev, n_burn=10,
                               n_levels=3, nsamp=16, seed=1)
    assert len(models) == 1
    assert models[0].samples["lamUz"].shape == (16, 3)
    tim = np.loadtxt(tmp_path / "models" / "timing.csv", delimiter=",")
    assert tim.shape == (4,) and tim[0] == n and tim[1] == 3
    data, mdl = gmodel.load_model(cfg, n, 3, dtype=np.float64, device=dev)
    np.testing.assert_array_equal(mdl.samples["betaU"], models[0].samples["betaU"])
    np.testing.assert_array_equal(mdl.params.lamWs.mcmcStepParam,
                                  models[0].params.lamWs.mcmcStepParam)
    samples = mdl.get_samples(numsamples=4, nburn=4)
    pred = SepiaEmulatorPrediction(model=mdl, samples=samples, t_pred=rng.random((7, d)))
    assert pred.w.shape == (4, 7, 3) and np.all(np.isfinite(pred.var))
    assert pred.get_y().shape == (4, 7, ny)


def test_speculative_groups_same_chain(dev):
    """spec = 1 .. 4 (up to 15 parameter states x P GPs per gp_loglik) give the same chain: the
    batch a likelihood is evaluated in does not change its value."""
    n, d, P = 96, 3, 4
    X, w, lam = _problem(n, d, P, seed=31)
    recs = []
    for spec in (1, 2, 3, 4):
        pr = mcmc.ModelParams(d, P)
        sampler = mcmc.GPUSampler(_t(X, dev), _t(w, dev), _t(lam, dev), pr, spec=spec)
        recs.append(sampler.run(30, np.random.default_rng(9)))
    for r in recs[1:]:
        for k in ("betaU", "lamUz", "lamWs", "lamWOs", "logPost"):
            np.testing.assert_allclose(r[k], recs[0][k], rtol=1e-12, atol=1e-12, err_msg=k)


@pytest.mark.parametrize("spec,graph", [(1, False), (2, True), (4, False)])
def test_fused_sweep_equals_tensor_sweep(dev, spec, graph):
    """gp_mcmc_group_prep / _decide (csrc/mcmc.hip) against the tensor-op sweep they replace:
    the same proposals, decisions and counters (op-for-op arithmetic, no FMA contraction)."""
    n, d, P = 72, 4, 5
    X, w, lam = _problem(n, d, P, seed=41)
    recs, cnts = [], []
    for fused in (False, True):
        pr = mcmc.ModelParams(d, P)
        sampler = mcmc.GPUSampler(_t(X, dev), _t(w, dev), _t(lam, dev), pr, use_graph=graph,
                                  spec=spec, fused=fused)
        assert sampler.fused == fused
        recs.append(sampler.run(30, np.random.default_rng(13)))
        cnts.append(sampler.counts())
    for k in ("betaU", "lamUz", "lamWs", "lamWOs"):
        np.testing.assert_array_equal(recs[1][k], recs[0][k], err_msg=k)
    np.testing.assert_allclose(recs[1]["logPost"], recs[0]["logPost"], rtol=1e-13, atol=0)
    for k in cnts[0]:
        np.testing.assert_array_equal(cnts[1][k], cnts[0][k], err_msg=str(k))


@pytest.mark.parametrize("block", [16, 5])
def test_block_graph_equals_eager(dev, block):
    """run() replays `block` sweeps per graph (uniform rows and record rows in static blocks)
    and runs the remainder one sweep at a time: the chain, the records and the counters equal
    the eager (no graph) sweep's bit for bit, recording or not."""
    n, d, P = 64, 3, 4
    X, w, lam = _problem(n, d, P, seed=51)
    recs, cnts = [], []
    for graph in (False, True):
        pr = mcmc.ModelParams(d, P)
        sampler = mcmc.GPUSampler(_t(X, dev), _t(w, dev), _t(lam, dev), pr, use_graph=graph)
        sampler.block = block
        rng = np.random.default_rng(17)
        sampler.run(block + 3, rng, record=False)              # a block + singles, unrecorded
        recs.append(sampler.run(2 * block + 7, rng, block=block + 4))
        cnts.append(sampler.counts())
    assert len(recs[1]["lamUz"]) == 2 * block + 7
    for k in ("betaU", "lamUz", "lamWs", "lamWOs", "logPost"):
        np.testing.assert_array_equal(recs[1][k], recs[0][k], err_msg=k)
    for k in cnts[0]:
        np.testing.assert_array_equal(cnts[1][k], cnts[0][k], err_msg=str(k))


def test_merged_group_step_equals_two_launches(dev, monkeypatch):
    """gp_mcmc_group_step (a group's decisions + the next group's proposals in one launch)
    gives the chain, records and counters of gp_mcmc_group_decide + gp_mcmc_group_prep."""
    n, d, P = 64, 3, 4
    X, w, lam = _problem(n, d, P, seed=61)
    recs, cnts = [], []
    for merge in ("0", "1"):
        monkeypatch.setenv("GPFIT_MCMC_MERGE", merge)
        pr = mcmc.ModelParams(d, P)
        sampler = mcmc.GPUSampler(_t(X, dev), _t(w, dev), _t(lam, dev), pr, spec=2)
        assert sampler._merge == (merge == "1")
        recs.append(sampler.run(21, np.random.default_rng(23)))
        cnts.append(sampler.counts())
    for k in ("betaU", "lamUz", "lamWs", "lamWOs", "logPost"):
        np.testing.assert_array_equal(recs[1][k], recs[0][k], err_msg=k)
    for k in cnts[0]:
        np.testing.assert_array_equal(cnts[1][k], cnts[0][k], err_msg=str(k))


@pytest.mark.parametrize("n,P", [(512, 24), (512, 8), (700, 8), (130, 1), (1000, 3), (64, 2)])
def test_loglik_in_chain_matches_oracle_and_linv_path(dev, n, P):
    """gp_loglik on the persistent factorisation's in-chain mode (the chain solves z = L^-1 w by
    forward substitution over its diagonal inverses, the DP tasks add sum_k L_jk z_k, the last
    workgroup writes ll; no L^-1 tasks, trmv or reduction) against the oracle, and against the
    L^-1 path (gp_set_potrf_path(1): blocked sweep + L^-1 + trmv + reduction).  (512, 24) is the
    fit's speculative group at timing.csv:9; 700 a ragged last tile; 8 and 24 the per-XCD
    queues."""
    from gladsgp_amd import _capi
    d = 8
    X, w, lam = _problem(n, d, P, seed=n + P)
    rng = np.random.default_rng(P)
    betaU = rng.uniform(0.2, 3.0, (d + 1, P))
    lamUz = rng.uniform(0.5, 3.0, P)
    lamWs = rng.uniform(200, 3000, P)
    lamWOs = 120.0
    ref = mcmc_ref.loglik_pcs(X, w, lam, betaU, lamUz, lamWs, lamWOs)
    args = (_t(X, dev), _t(betaU[1:].T, dev), _t(1.0 / lamUz, dev),
            _t(1.0 / lamWs + 1.0 / (lamWOs * lam), dev), _t(w, dev))
    ws = kernels.LoglikWorkspace(n, P, dev)
    got = kernels.loglik(*args, ws).cpu().numpy()
    ws.check_status()
    assert np.all(ws.info.cpu().numpy() == 0)
    prev = _capi.lib().gp_set_potrf_path(1)
    try:
        ws1 = kernels.LoglikWorkspace(n, P, dev)
        alt = kernels.loglik(*args, ws1).cpu().numpy()
    finally:
        _capi.lib().gp_set_potrf_path(prev)
    tol = 1e-9 * np.maximum(1.0, np.abs(ref))
    assert np.all(np.abs(got - ref) <= tol), (got - ref)
    assert np.all(np.abs(got - alt) <= 1e-11 * np.maximum(1.0, np.abs(alt))), (got - alt)
    # repeated calls on one workspace: bit-identical (deterministic partial-sum order)
    again = kernels.loglik(*args, ws).cpu().numpy()
    assert np.array_equal(again, got)
