"""Host logic of gladsgp_amd.mcmc.GPUSampler on the CPU: the sweep's speculative groups
(``spec`` updates per batched likelihood call, 2^spec - 1 parameter states) against the oracle
chain (oracle/mcmc_ref.py, one update at a time) fed the same uniforms.

Only the likelihood is swapped: ``kernels.loglik`` (the HIP gp_loglik) is replaced inside this
test by a torch CPU stand-in with the same contract, so the selection of each update's
likelihood from the outcomes of the group's earlier updates, the per-GP / shared (lamWOs)
decisions and the uniform layout are checked without a GPU.  The product path has no such
fallback; the GPU twin of this test is tests/test_gpu_mcmc.py.
"""
import numpy as np
import pytest
import torch

from gladsgp_amd import kernels, mcmc
from oracle import gp_ref, mcmc_ref

F64 = torch.float64


def _cpu_loglik(X, beta, s, delta, w, ws, out=None):
    """gp_loglik's contract on the CPU: ll_b = -1/2 w_b^T G_b^-1 w_b - 1/2 log|G_b|, -inf where
    G_b is not positive definite."""
    B = beta.shape[0]
    d2 = (X[None, :, None, :] - X[None, None, :, :]) ** 2          # (1, n, n, d)
    G = s.view(B, 1, 1) * torch.exp(-(d2 * beta.view(B, 1, 1, -1)).sum(-1))
    G = G + delta.view(B, 1, 1) * torch.eye(X.shape[0], dtype=F64)
    L, info = torch.linalg.cholesky_ex(G)
    z = torch.linalg.solve_triangular(L, w.unsqueeze(-1), upper=False).squeeze(-1)
    ll = -0.5 * (z * z).sum(-1) - torch.log(torch.diagonal(L, dim1=-2, dim2=-1)).sum(-1)
    ll = torch.where(info == 0, ll, torch.full_like(ll, -np.inf))
    if out is None:
        return ll
    out.copy_(ll)
    return out


class _Ws:
    def __init__(self, n, batch, device):
        self.n, self.batch = n, batch

    def check_status(self, reset=True):
        pass


@pytest.fixture
def cpu_loglik(monkeypatch):
    monkeypatch.setattr(kernels, "loglik", _cpu_loglik)
    monkeypatch.setattr(kernels, "LoglikWorkspace", _Ws)


def _problem(n, d, P, seed):
    rng = np.random.default_rng(seed)
    X = rng.random((n, d))
    lam = rng.uniform(1.0, 10.0, P)
    w = np.empty((P, n))
    for j in range(P):
        G = gp_ref.gram_ardse(X, rng.uniform(0.5, 4.0, d), 1.0, 1e-3)
        w[j] = np.linalg.cholesky(G) @ rng.standard_normal(n)
    return X, w, lam


@pytest.mark.parametrize("spec", [1, 2, 3, 5])
def test_speculative_sweep_matches_oracle(cpu_loglik, spec):
    n, d, P, nsw = 20, 3, 3, 30
    X, w, lam = _problem(n, d, P, seed=4)
    pr = mcmc.ModelParams(d, P)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64))  # noqa: E731
    sampler = mcmc.GPUSampler(t(X), t(w), t(lam), pr, spec=spec)
    assert not sampler.use_graph
    # groups of `spec` consecutive likelihood-changing updates: d betaU rows, lamUz, lamWs, lamWOs
    assert [len(g) for g in sampler.groups][:-1] == [spec] * (len(sampler.groups) - 1)
    assert sum(len(g) for g in sampler.groups) == d + 3
    rec = sampler.run(nsw, np.random.default_rng(5))
    U = np.random.default_rng(5).random((nsw, mcmc.uniforms_per_sweep(d, P)))
    state = {"betaU": pr.betaU.val, "lamUz": pr.lamUz.val[0], "lamWs": pr.lamWs.val[0],
             "lamWOs": pr.lamWOs.val[0, 0]}
    steps = {k: getattr(pr, k).mcmcStepParam for k in pr.names}
    specs = {k: (getattr(pr, k).dist, getattr(pr, k).params, getattr(pr, k).bounds,
                 getattr(pr, k).mcmcStepType) for k in pr.names}
    _, ref, acc = mcmc_ref.run_chain(X, w, lam, specs, state, steps, U)
    for k in ("betaU", "lamUz", "lamWs", "lamWOs"):
        np.testing.assert_allclose(rec[k], ref[k], rtol=1e-9, atol=1e-12, err_msg=k)
    # both outcomes occur inside groups, so the speculative selection is exercised
    cnt = sampler.counts()
    assert 0 < cnt["lamUz"].sum() < nsw * P
    assert 0 < sum(cnt[("betaU", k)].sum() for k in range(1, d + 1)) < nsw * P * d


def test_spec_must_be_positive(cpu_loglik):
    X = torch.zeros((4, 2), dtype=F64)
    with pytest.raises(ValueError):
        mcmc.GPUSampler(X, torch.zeros((2, 4), dtype=F64), torch.ones(2, dtype=F64),
                        mcmc.ModelParams(2, 2), spec=0)


def test_default_spec_cost_model():
    """default_spec: spec 3 at the fit's n = 512, P = 8 (11 updates; r06al measured 1.054 vs
    1.278 ms per sweep at spec 2), less speculation once the batch is work-bound, always within
    the fused kernels' group limit."""
    from gladsgp_amd import _capi
    assert mcmc.default_spec(512, 8, 11) == 3
    assert mcmc.default_spec(512, 64, 11) < 3
    assert mcmc.default_spec(2048, 8, 11) == 1
    for n in (16, 512, 1024, 4096):
        for P in (1, 8, 25, 64):
            assert 1 <= mcmc.default_spec(n, P, 11) <= _capi.MCMC_MAX_GROUP
