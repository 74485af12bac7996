"""GPU parity of the column-resident prediction kernel (predict.hip trmm_res_kernel, round 6).

Every prediction with npad <= 512 runs it: with the cross-covariance produced inside the kernel
(d <= 8: gp_predict, gp_fit_predict) or read from a materialised chunk (gp_predict_solve after
gp_predict_cross, and d > 8).  Checked here:
* against the oracle (gp_ref.predict) on a sample spread over every chunk, at the prediction
  tolerance of tests/test_gpu_kernels.py (|dmean| <= 1e-8 max|mean|, |dvar| <= 1e-9 s);
* bit for bit across entry points (predict, fit_predict, predict_cross + predict_solve), across
  chunkings and across prefixes of the test set: the fused and the slab K* are the same values
  and every sum keeps its order;
* ragged shapes: n = 1, 5, 127-129, 300, 384, 511, 512 (npad 128-512), m not a multiple of the
  32-point panel, batches 1-3, d = 1, 3, 8 (fused) and 12 (slab);
* the tile-packed L^-1 (the sharded single-GP payload) gives the padded layout's bits.
"""
import numpy as np
import pytest
import torch

from oracle import gp_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from gladsgp_amd import kernels  # noqa: F401
    return torch.device("cuda:0")


def _problem(n, m, B, d, seed):
    rng = np.random.default_rng(seed)
    X = rng.random((n, d))
    Xs = rng.random((m, d))
    betas = rng.uniform(0.5, 5.0, (B, d)) * (8.0 / d)
    W = np.sin(X @ rng.uniform(0, 1, (d, B))).T.copy()      # (B, n)
    s = rng.uniform(0.8, 1.5, B)
    delta = rng.uniform(1e-6, 1e-4, B)
    return X, Xs, betas, W, s, delta


def _oracle_check(X, Xs, W, betas, s, delta, mean, var, idx):
    for b in range(W.shape[0]):
        mr, vr = gp_ref.predict(X, Xs[idx], W[b], betas[b], s[b], delta[b], s_pred=s[b])
        assert np.max(np.abs(mean[b, idx] - mr)) <= 1e-8 * max(1.0, np.max(np.abs(mr))), b
        assert np.max(np.abs(var[b, idx] - vr)) <= 1e-9 * s[b], b


@pytest.mark.parametrize("n,m,B,d", [
    (1, 70, 1, 8),
    (5, 777, 2, 8),
    (127, 1000, 1, 3),
    (128, 4100, 3, 8),
    (129, 2049, 2, 1),
    (300, 9000, 2, 8),      # two 8192-point chunks for a batch, the second ragged
    (384, 3001, 1, 8),
    (511, 5000, 3, 8),
    (512, 17000, 1, 8),     # one GP: a 16384-point chunk + a ragged tail
    (333, 5000, 2, 12),     # d > 8: the cross-covariance from a chunk (slab mode)
])
def test_res_matches_oracle_and_is_bitwise_across_paths(dev, n, m, B, d):
    from gladsgp_amd import kernels
    X, Xs, betas, W, s, delta = _problem(n, m, B, d, 1000 * n + m + B + d)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    Xd, Xsd, bd, Wd, sd, dd = t(X), t(Xs), t(betas), t(W), t(s), t(delta)
    mean_f, var_f, ch = kernels.fit_predict(Xd, Xsd, bd, sd, dd, sd, Wd)
    ref_m, ref_v = mean_f.cpu().numpy(), var_f.cpu().numpy()
    idx = np.unique(np.concatenate([np.arange(0, m, max(1, m // 250)),
                                    np.arange(max(0, m - 40), m)]))
    _oracle_check(X, Xs, W, betas, s, delta, ref_m, ref_v, idx)
    res = {"predict": kernels.predict(ch, Xd, Xsd, bd, sd, sd, Wd)}
    for mc in (128, 1280):
        res[f"predict m_chunk={mc}"] = kernels.predict(ch, Xd, Xsd, bd, sd, sd, Wd, m_chunk=mc)
        res[f"fit_predict m_chunk={mc}"] = kernels.fit_predict(Xd, Xsd, bd, sd, dd, sd, Wd,
                                                               m_chunk=mc)[:2]
    prep = kernels.predict_prepare(Xd, Xsd, bd, sd, batch=B, m_chunk=1024)
    res["predict_solve"] = kernels.predict_solve(ch, prep, sd, Wd)
    with kernels.FitPredictContext(dev) as fctx:
        res["fit_predict ctx"] = kernels.fit_predict(Xd, Xsd, bd, sd, dd, sd, Wd, ctx=fctx)[:2]
        torch.cuda.synchronize()
    for name, (mu, var) in res.items():
        assert np.array_equal(mu.cpu().numpy(), ref_m), name
        assert np.array_equal(var.cpu().numpy(), ref_v), name
    pre = max(1, m // 3)
    mu, var = kernels.predict(ch, Xd, Xsd[:pre].contiguous(), bd, sd, sd, Wd)
    assert np.array_equal(mu.cpu().numpy(), ref_m[:, :pre])
    assert np.array_equal(var.cpu().numpy(), ref_v[:, :pre])


@pytest.mark.parametrize("n,B,d", [(200, 1, 8), (512, 2, 8), (300, 2, 12)])
def test_res_packed_linv_bitwise(dev, n, B, d):
    """The tile-packed L^-1 gives the padded layout's bits, fused (d <= 8) and from
    materialised chunks (d > 8)."""
    from gladsgp_amd import kernels
    X, Xs, betas, W, s, delta = _problem(n, 4000, B, d, 5 * n + B)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    Xd, Xsd, bd, Wd, sd, dd = t(X), t(Xs), t(betas), t(W), t(s), t(delta)
    ch = kernels.cholesky_inverse(kernels.gram(Xd, bd, sd, dd, batch=B))
    ch.check()
    ref_m, ref_v = kernels.predict(ch, Xd, Xsd, bd, sd, sd, Wd)
    pk = kernels.PackedLinv(n, kernels.pack_linv(ch), ch.info)
    for mc in (0, 1280):
        mu, var = kernels.predict(pk, Xd, Xsd, bd, sd, sd, Wd, m_chunk=mc)
        assert torch.equal(mu, ref_m) and torch.equal(var, ref_v), mc


def test_res_nonfinite_hyperparameters_propagate(dev):
    """A NaN length-scale reaches the outputs of its own GP only (the fused K* keeps
    cross_kp's NaN propagation; rows past n stay exact zeros)."""
    from gladsgp_amd import kernels
    n, m, B, d = 200, 3000, 2, 8
    X, Xs, betas, W, s, delta = _problem(n, m, B, d, 99)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    Xd, Xsd, bd, Wd, sd, dd = t(X), t(Xs), t(betas), t(W), t(s), t(delta)
    ch = kernels.cholesky_inverse(kernels.gram(Xd, bd, sd, dd, batch=B))
    ch.check()
    good_m, good_v = kernels.predict(ch, Xd, Xsd, bd, sd, sd, Wd)
    bad = bd.clone()
    bad[1, 3] = float("nan")
    mu, var = kernels.predict(ch, Xd, Xsd, bad, sd, sd, Wd)
    assert torch.equal(mu[0], good_m[0]) and torch.equal(var[0], good_v[0])
    assert torch.isnan(mu[1]).all() and torch.isnan(var[1]).all()


def test_predict_path_hook(dev):
    """gp_set_predict_path: 2 (the column-resident kernel from materialised chunks) gives the
    fused path's bits; 1 (cross-covariance chunks + the pair TRMM) agrees to rounding."""
    from gladsgp_amd import _capi, kernels
    n, m, B, d = 300, 3000, 2, 8
    X, Xs, betas, W, s, delta = _problem(n, m, B, d, 17)
    t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
    Xd, Xsd, bd, Wd, sd, dd = t(X), t(Xs), t(betas), t(W), t(s), t(delta)
    lib = _capi.lib()
    prev = lib.gp_set_predict_path(0)
    try:
        ref = kernels.fit_predict(Xd, Xsd, bd, sd, dd, sd, Wd)[:2]
        lib.gp_set_predict_path(2)
        slab = kernels.fit_predict(Xd, Xsd, bd, sd, dd, sd, Wd)[:2]
        lib.gp_set_predict_path(1)
        pair = kernels.fit_predict(Xd, Xsd, bd, sd, dd, sd, Wd)[:2]
    finally:
        assert lib.gp_set_predict_path(prev) in (0, 1, 2)
    assert torch.equal(slab[0], ref[0]) and torch.equal(slab[1], ref[1])
    assert float((pair[0] - ref[0]).abs().max()) <= 1e-10 * max(1.0, float(ref[0].abs().max()))
    assert float((pair[1] - ref[1]).abs().max()) <= 1e-12 * float(sd.max())


def test_res_boundary_513_uses_pair_path_and_matches_oracle(dev):
    """npad 512 -> 640 at n = 513: the row-pair path; both sides of the boundary agree with the
    oracle at the prediction tolerance."""
    from gladsgp_amd import kernels
    for n in (512, 513):
        X, Xs, betas, W, s, delta = _problem(n, 2500, 2, 8, n)
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
        mean, var, _ = kernels.fit_predict(t(X), t(Xs), t(betas), t(s), t(delta), t(s), t(W))
        idx = np.arange(0, 2500, 7)
        _oracle_check(X, Xs, W, betas, s, delta, mean.cpu().numpy(), var.cpu().numpy(), idx)
