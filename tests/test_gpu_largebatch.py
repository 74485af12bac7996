"""GPU parity at the reference's own prediction shapes: many (sample, PC) GPs per call.

The reference predicts with 64 or 128 posterior samples x p = 8 PCs (assess_all_models.py:471,
plot_test_error.py:486, train_config.py:75) from m = 256 or 512 training runs
(train_config.py:9, the n = 512 models of timing.csv), in batches of 4 test points
(assess_all_models.py:481-489): 512-1024 independent GPs at n = 256-512 per
SepiaEmulatorPrediction.  EmulatorPrediction factorises them in groups far larger than the
persistent kernel's two-workgroups-per-problem limit, so these tests cover the group split and
both factorisation paths (persistent groups and the blocked sweep) against the oracle.

Tolerances: |dmean| <= 1e-9 max(1, |mean|), |dvar| <= 1e-9 (s ~ 0.3-2).
"""

import numpy as np
import pytest
import torch

from oracle import gp_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def _t(x, dev):
    return torch.as_tensor(np.asarray(x, dtype=np.float64), device=dev)


def _ensemble(n, ny=400, d=8, seed=0):
    rng = np.random.default_rng(seed)
    t = rng.random((n, d))
    modes = rng.standard_normal((10, ny)) * (0.6 ** np.arange(10))[:, None]
    coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, d) + k) for k in range(10)], 1)
    return t, 1.0 + coef @ modes + 1e-3 * rng.standard_normal((n, ny))


def _samples(S, d, P, seed=1):
    rng = np.random.default_rng(seed)
    return {"betaU": rng.uniform(0.2, 3.0, (S, (d + 1) * P)),
            "lamUz": rng.uniform(0.5, 3.0, (S, P)),
            "lamWs": rng.uniform(200, 3000, (S, P)),
            "lamWOs": rng.uniform(50, 500, (S, 1))}


def _check_units(pred, t, t_pred, w_hat, lam, samples, units):
    d, P = t.shape[1], w_hat.shape[1]
    beta, s, delta, s_pred = gp_ref.sepia_gp_params(samples, lam, d, P)
    worst = [0.0, 0.0]
    for a, j in units:
        mu, var = gp_ref.predict(t, t_pred, w_hat[:, j], beta[a, j], s[a, j], delta[a, j],
                                 s_pred[a, j])
        dm = np.max(np.abs(pred.w[a, :, j] - mu))
        dv = np.max(np.abs(pred.var[a, :, j] - var))
        assert dm <= 1e-9 * max(1.0, np.max(np.abs(mu))), (a, j, dm)
        assert dv <= 1e-9, (a, j, dv)
        worst = [max(worst[0], dm), max(worst[1], dv)]
    return worst


@pytest.mark.parametrize("n,S,group", [(256, 64, None), (512, 128, None), (512, 64, 512),
                                       (256, 64, 96)])
def test_reference_prediction_shapes(dev, tmp_path, n, S, group):
    """S x 8 units (512 or 1024 GPs), 4 test points per call; ``group``: GPs factorised per
    launch (None = the library's choice; 512 forces the blocked sweep, 96 persistent groups
    with a ragged last group)."""
    from gladsgp_amd import model as gm
    from gladsgp_amd.emulator import EmulatorPrediction
    P = 8
    t, y = _ensemble(n)
    np.random.seed(0)
    data, model = gm.init_model(t, y, "lb", P, data_dir=str(tmp_path), device=dev,
                                verbose=False)
    samples = _samples(S, t.shape[1], P)
    t_pred = np.random.default_rng(4).random((4, t.shape[1]))
    pred = EmulatorPrediction(model=model, samples=samples, t_pred=t_pred, group=group)
    assert pred.w.shape == (S, 4, P)
    w_hat = model.w_hat.cpu().numpy()
    lam = model.LamSim.cpu().numpy()
    units = [(0, 0), (S - 1, P - 1), (S // 2, 3), (1, 5), (S // 2 - 1, P - 1), (S - 2, 0)]
    _check_units(pred, t, t_pred, w_hat, lam, samples, units)
    assert np.all(pred.var > 0)


@pytest.fixture
def force_sweep():
    """gp_set_potrf_path(1) (the ABI's test hook) for the test, restored afterwards."""
    from gladsgp_amd import _capi
    prev = _capi.lib().gp_set_potrf_path(1)
    yield
    _capi.lib().gp_set_potrf_path(prev)


@pytest.mark.parametrize("sweep", [False, True])
def test_cholesky_inverse_batch_256_n512(dev, sweep, request):
    """One cholesky_inverse of 256 n = 512 Grams (beyond the persistent kernel's batch limit:
    the blocked sweep), and the same with gp_set_potrf_path(1) forcing the sweep at a batch the
    persistent kernel would take (128)."""
    from gladsgp_amd import kernels
    B = 256 if not sweep else 128
    if sweep:
        request.getfixturevalue("force_sweep")
    n = 512
    rng = np.random.default_rng(31)
    X = rng.random((n, 8))
    betas = rng.uniform(0.5, 5, (B, 8))
    s = rng.uniform(0.5, 2.0, B)
    delta = rng.uniform(1e-4, 1e-2, B)
    G = kernels.gram(_t(X, dev), _t(betas, dev), _t(s, dev), _t(delta, dev))
    ch = kernels.cholesky_inverse(G)
    assert ch.info.cpu().tolist() == [0] * B
    for b in (0, 1, 63, B // 2 - 1, B // 2, B - 1):
        Gb = gp_ref.gram_ardse(X, betas[b], s[b], delta[b])
        Lref = np.linalg.cholesky(Gb)
        L = ch.L[b].cpu().numpy()
        Li = ch.Linv[b].cpu().numpy()
        assert np.linalg.norm(L @ L.T - Gb) / np.linalg.norm(Gb) <= 1e-13
        assert np.max(np.abs(L - Lref)) <= 1e-10 * np.max(np.abs(Lref))
        assert np.max(np.abs(Li @ L - np.eye(n))) <= 1e-9
        np.testing.assert_allclose(float(ch.logdet[b]), 2 * np.sum(np.log(np.diag(Lref))),
                                   rtol=0, atol=1e-9 * n)


def test_sweep_multi_tile_matches_persistent(dev):
    """The sweep and the persistent kernel agree at a multi-tile shape with ragged tiles."""
    from gladsgp_amd import kernels
    rng = np.random.default_rng(17)
    n, B = 1000, 6
    X = rng.random((n, 8))
    betas = rng.uniform(0.5, 5, (B, 8))
    G = kernels.gram(_t(X, dev), _t(betas, dev), 1.0, 1e-4)
    from gladsgp_amd import _capi
    a = kernels.cholesky_inverse(G.clone())
    prev = _capi.lib().gp_set_potrf_path(1)
    try:
        b = kernels.cholesky_inverse(G.clone())
        torch.cuda.synchronize()
    finally:
        assert _capi.lib().gp_set_potrf_path(prev) == 1
    for c in (a, b):
        assert c.info.cpu().tolist() == [0] * B
    La, Lb = a.L.cpu().numpy(), b.L.cpu().numpy()
    for k in range(B):
        assert np.max(np.abs(La[k] - Lb[k])) <= 1e-11 * np.max(np.abs(La[k]))


@pytest.mark.parametrize("n,B", [(512, 24), (1024, 32), (1000, 16)])
def test_xcd_queues_match_shared_queue(dev, n, B):
    """Batches of 8k run the persistent factorisation from per-XCD task queues
    (gp_set_potrf_path(0)); every tile keeps its K order, so L, L^-1 and logdet are bit-identical
    to the one-shared-queue launch (path 2).  A non-PD problem aborts only itself (info at its
    failing column), whichever queue it sits in."""
    from gladsgp_amd import _capi, kernels
    rng = np.random.default_rng(23)
    X = rng.random((n, 8))
    betas = rng.uniform(0.5, 5, (B, 8))
    G = kernels.gram(_t(X, dev), _t(betas, dev), 1.0, 1e-5)
    bad = 8 + 3                                      # queue 3 of the per-XCD launch
    G[bad, 700 % n, 700 % n] = -1.0
    a = kernels.cholesky_inverse(G.clone())
    prev = _capi.lib().gp_set_potrf_path(2)
    try:
        b = kernels.cholesky_inverse(G.clone())
        torch.cuda.synchronize()
    finally:
        assert _capi.lib().gp_set_potrf_path(prev) == 2
    ia, ib = a.info.cpu().tolist(), b.info.cpu().tolist()
    assert ia == ib
    assert ia[bad] > 0 and [v for k, v in enumerate(ia) if k != bad] == [0] * (B - 1)
    ok = [k for k in range(B) if k != bad]
    assert torch.equal(a.L[ok], b.L[ok])
    assert torch.equal(a.Linv[ok], b.Linv[ok])
    assert torch.equal(a.logdet[ok], b.logdet[ok])
    Gb = gp_ref.gram_ardse(X, betas[0], 1.0, 1e-5)
    L = a.L[0].cpu().numpy()
    assert np.linalg.norm(L @ L.T - Gb) / np.linalg.norm(Gb) <= 1e-13
