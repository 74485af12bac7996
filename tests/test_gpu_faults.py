"""GPU: the factorisation's internal-error path is loud, and inputs that are not finite reach
info.

* gp_set_poll_budget(-1) makes every later persistent factorisation start with its problems
  given up, deterministically (no timing involved): info = -1 for every problem, reported by the
  last workgroup to leave the launch (after every chain and XT task has returned);
  Cholesky.check / fit_predict(check=True) raise FactorizationInternalError (never "not
  positive definite"); gp_loglik returns NaN (never the -inf of a rejected proposal) and raises
  its sticky status word, which the Metropolis sampler reads once per run and raises on.
* produced tiles are read with sc1 loads unless no 128-B line spans two tiles: lda % 16 != 0
  (n = 1000, 2100 with lda = n) at batch > 1 against LAPACK (chol.hip pp_term).
* a NaN / Inf hyperparameter or design value makes the Gram's diagonal NaN (exp_neg keeps NaN),
  so the factorisation reports info > 0 instead of factorising a finite delta * I.
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


@pytest.fixture
def aborted():
    """Every factorisation enqueued inside the block starts given up (info = -1)."""
    from gladsgp_amd import _capi
    lib = _capi.lib()
    prev = lib.gp_set_poll_budget(-1)
    try:
        yield
    finally:
        torch.cuda.synchronize()
        lib.gp_set_poll_budget(prev if prev > 0 else 0)


def _t(x, dev):
    return torch.as_tensor(np.asarray(x, dtype=np.float64), device=dev)


def _grams(n, B, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.random((n, 8))
    return X, [gp_ref.gram_ardse(X, rng.uniform(0.5, 5, 8), 1.0, 1e-4) for _ in range(B)]


def test_internal_error_reported_as_info_minus_one(dev, aborted):
    from gladsgp_amd import kernels
    _, Gs = _grams(1024, 3)
    ch = kernels.cholesky_inverse(_t(np.stack(Gs), dev).contiguous())
    assert ch.info.cpu().tolist() == [-1, -1, -1]
    with pytest.raises(kernels.FactorizationInternalError):
        ch.check()


def test_internal_error_through_the_c_abi(dev, aborted):
    """gp_potrf_inv (the allocating form) and gp_potrf: info = -1 via the C ABI itself."""
    from gladsgp_amd import _capi, kernels
    n = 700
    _, Gs = _grams(n, 2, seed=3)
    A = _t(np.stack(Gs), dev).contiguous()
    npad = kernels.padded_n(n)
    Linv = torch.empty((2, npad, npad), dtype=torch.float64, device=dev)
    info = torch.full((2,), 99, dtype=torch.int32, device=dev)
    logdet = torch.empty(2, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    _capi.call("gp_potrf_inv", A.data_ptr(), n, n, n * n, Linv.data_ptr(), npad, npad * npad, 2,
               info.data_ptr(), logdet.data_ptr(), st)
    assert info.cpu().tolist() == [-1, -1]
    A2 = _t(np.stack(Gs), dev).contiguous()
    info.fill_(99)
    _capi.call("gp_potrf", A2.data_ptr(), n, n, n * n, 2, info.data_ptr(), logdet.data_ptr(), st)
    assert info.cpu().tolist() == [-1, -1]


def test_fit_predict_raises_internal_error(dev, aborted):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(5)
    X, Xs = rng.random((512, 8)), rng.random((300, 8))
    w = np.sin(X @ rng.uniform(0, 1, 8))
    with kernels.FitPredictContext(dev) as fctx:
        with pytest.raises(kernels.FactorizationInternalError):
            kernels.fit_predict(_t(X, dev), _t(Xs, dev), _t(rng.uniform(0.5, 5, 8), dev), 1.0,
                                1e-6, 1.0, _t(w, dev), ctx=fctx)


def test_loglik_internal_error_is_nan_and_sticky(dev):
    from gladsgp_amd import _capi, kernels
    lib = _capi.lib()
    rng = np.random.default_rng(6)
    n, P, d = 320, 3, 8
    X = _t(rng.random((n, d)), dev).contiguous()
    beta = _t(rng.uniform(0.5, 4, (P, d)), dev).contiguous()
    s = _t(np.full(P, 1.1), dev)
    delta = _t(np.full(P, 1e-3), dev)
    w = _t(rng.standard_normal((P, n)), dev).contiguous()
    ws = kernels.LoglikWorkspace(n, P, dev)
    ll_ok = kernels.loglik(X, beta, s, delta, w, ws).cpu().numpy()
    assert np.all(np.isfinite(ll_ok))
    ws.check_status()                      # clean
    prev = lib.gp_set_poll_budget(-1)
    try:
        ll_bad = kernels.loglik(X, beta, s, delta, w, ws).cpu().numpy()
    finally:
        torch.cuda.synchronize()
        lib.gp_set_poll_budget(prev if prev > 0 else 0)
    assert np.all(np.isnan(ll_bad)), ll_bad           # never -inf (a silent rejection)
    assert ws.info.cpu().tolist() == [-1] * P
    with pytest.raises(kernels.FactorizationInternalError):
        ws.check_status()                  # raises once, then reset
    ws.check_status()
    # a non-positive-definite proposal stays a rejection (-inf), not an error
    bad = delta.clone()
    bad[1] = -5.0
    ll_np = kernels.loglik(X, beta, s, bad, w, ws).cpu().numpy()
    assert ll_np[1] == -np.inf and np.isfinite(ll_np[0]) and np.isfinite(ll_np[2])
    ws.check_status()


@pytest.mark.parametrize("graph", [False, True])
def test_sampler_raises_on_internal_error(dev, graph):
    """Eager sweeps, and a captured sweep graph (the default): kernel arguments, the preset
    abort included, are frozen when the graph is captured, so the graph case captures after
    gp_set_poll_budget(-1)."""
    from gladsgp_amd import _capi, kernels, mcmc
    lib = _capi.lib()
    rng = np.random.default_rng(7)
    n, P, d = 200, 2, 4
    X = _t(rng.random((n, d)), dev)
    w = _t(rng.standard_normal((P, n)), dev)
    sm = mcmc.GPUSampler(X, w, _t(np.full(P, 3.0), dev), mcmc.ModelParams(d, P),
                         use_graph=graph)
    if not graph:
        sm.run(2, np.random.default_rng(0), record=False)      # healthy
    prev = lib.gp_set_poll_budget(-1)
    try:
        with pytest.raises(kernels.FactorizationInternalError):
            sm.run(2, np.random.default_rng(1), record=True)
    finally:
        torch.cuda.synchronize()
        lib.gp_set_poll_budget(prev if prev > 0 else 0)


@pytest.mark.parametrize("n,B", [(1000, 8), (2100, 4), (1100, 12)])
def test_unaligned_lda_batched_matches_lapack(dev, n, B):
    """lda = n with n % 16 != 0: tile columns share cache lines with their neighbours, so every
    produced tile must be read with sc1 loads (PPArgs::plain = 0)."""
    from gladsgp_amd import kernels
    assert n % 16 != 0
    rng = np.random.default_rng(n + B)
    Gs = [gp_ref.gram_ardse(rng.random((n, 8)), rng.uniform(0.5, 5, 8), 1.0, 1e-4)
          for _ in range(B)]
    ch = kernels.cholesky_inverse(_t(np.stack(Gs), dev).contiguous())
    assert ch.info.cpu().tolist() == [0] * B
    L_all = ch.L.cpu().numpy()
    Li_all = ch.Linv.cpu().numpy()
    for b in range(B):
        Lref = np.linalg.cholesky(Gs[b])
        L = L_all[b]
        assert np.linalg.norm(L @ L.T - Gs[b]) / np.linalg.norm(Gs[b]) <= 1e-13
        assert np.max(np.abs(L - Lref)) <= 1e-10 * np.max(np.abs(Lref))
        assert np.max(np.abs(Li_all[b] @ L - np.eye(n))) <= 1e-9


@pytest.mark.parametrize("what", ["beta_nan", "beta_inf", "x_nan"])
def test_non_finite_inputs_reach_info(dev, what):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(12)
    n, d = 300, 8
    X = rng.random((n, d))
    beta = rng.uniform(0.5, 5, d)
    if what == "beta_nan":
        beta[3] = np.nan
    elif what == "beta_inf":
        beta[0] = np.inf
    else:
        X[150, 2] = np.nan
    G = kernels.gram(_t(X, dev), _t(beta, dev), 1.0, 1e-6)
    ch = kernels.cholesky_inverse(G)
    assert int(ch.info[0]) != 0
    # gp_loglik: a rejection (-inf), the likelihood of a matrix that is not positive definite
    ws = kernels.LoglikWorkspace(n, 1, dev)
    ll = kernels.loglik(_t(X, dev).contiguous(), _t(beta, dev).reshape(1, d).contiguous(),
                        _t([1.0], dev), _t([1e-6], dev), _t(np.ones((1, n)), dev), ws)
    assert float(ll[0]) == -np.inf
