"""GPU parity of the fit-side kernels: GEMM (incl. split-K), ensemble statistics /
standardisation (src/model.py:60-72), Jacobi eigensolver, and randomized_svd (src/svd.py)
against numpy and the oracle restatement."""
import os

import numpy as np
import pytest
import torch

from oracle import gp_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def _t(a, dev):
    return torch.as_tensor(np.asarray(a, dtype=np.float64), device=dev)


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (70, 33, 129), (128, 64, 64), (17, 5, 60000)])
def test_gemm(dev, ta, tb, m, n, k):
    from gladsgp_amd.blas import CM, gemm
    rng = np.random.default_rng(m + n + k + ta * 2 + tb)
    A = rng.standard_normal((k, m) if ta else (m, k))
    B = rng.standard_normal((n, k) if tb else (k, n))
    C0 = rng.standard_normal((m, n))
    # column-major buffers: a (rows x cols) matrix M is stored as M^T in C order
    Ac = CM(_t(A.T.copy(), dev), A.shape[0], A.shape[1], A.shape[0])
    Bc = CM(_t(B.T.copy(), dev), B.shape[0], B.shape[1], B.shape[0])
    Cc = CM(_t(C0.T.copy(), dev), m, n, m)
    gemm(bool(ta), bool(tb), Ac, Bc, alpha=0.7, beta=-1.3, C=Cc)
    ref = 0.7 * ((A.T if ta else A) @ (B.T if tb else B)) - 1.3 * C0
    got = Cc.logical().cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-12 * np.sqrt(k) * np.abs(ref).max())


def test_sim_stats_and_standardize(dev):
    from gladsgp_amd import blas
    rng = np.random.default_rng(0)
    Y = rng.standard_normal((37, 1000)) * rng.uniform(0, 3, 1000) + rng.standard_normal(1000)
    Y[:, 5] = 2.5                      # constant location: sd floored (src/model.py:62-64)
    mu_r, sd_r, ystd_r = gp_ref.standardize(Y, 1e-6)
    Yd = _t(Y, dev)
    mu, sd = blas.sim_stats(Yd, 1e-6)
    np.testing.assert_allclose(mu.cpu().numpy(), mu_r, rtol=1e-14, atol=1e-14)
    np.testing.assert_allclose(sd.cpu().numpy(), sd_r, rtol=1e-13)
    assert float(sd[5]) == 1e-6
    ystd = blas.standardize(Yd, mu, sd)
    np.testing.assert_allclose(ystd.cpu().numpy(), ystd_r, rtol=1e-12, atol=1e-12)
    back = blas.standardize(ystd, mu, sd, inverse=True)
    np.testing.assert_allclose(back.cpu().numpy(), Y, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("r", [1, 2, 7, 25, 64, 100])
def test_syevj(dev, r):
    from gladsgp_amd.blas import CM, syevj
    rng = np.random.default_rng(r)
    M = rng.standard_normal((r, r + 3))
    A = M @ M.T
    w_ref, _ = np.linalg.eigh(A)
    Ac = CM(_t(A, dev).contiguous(), r, r, r)
    W, V, sw = syevj(Ac)
    W = W.cpu().numpy()
    V = V.logical().cpu().numpy()
    np.testing.assert_allclose(W, w_ref[::-1], rtol=1e-11, atol=1e-11 * w_ref.max())
    np.testing.assert_allclose(V.T @ V, np.eye(r), atol=1e-12)
    np.testing.assert_allclose(V @ np.diag(W) @ V.T, A, atol=1e-10 * np.abs(A).max())
    assert int(sw[0]) < 30


def test_randomized_svd_vs_reference_golden(dev, golden_dir):
    """Reference src/svd.py outputs (float32, seeded) vs GPU fp64 with the same Omega."""
    from gladsgp_amd.svd import randomized_svd
    g = np.load(os.path.join(golden_dir, "svd_ref_64x500.npz"))
    X = g["X"]
    for tag, (p, k) in {"p8": (8, None), "p25k0": (25, 0)}.items():
        U, S, Vh = randomized_svd(X, p, k=k, q=1, omega=g[f"{tag}_omega"], device=dev)
        assert U.shape == (64, p) and S.shape == (p,) and Vh.shape == (p, 500)
        # fp64 oracle restatement with the same Omega: tight
        Uo, So, Vo = gp_ref.randomized_svd(X.astype(np.float64), p, k=k, q=1,
                                           omega=g[f"{tag}_omega"])
        np.testing.assert_allclose(S, So, rtol=1e-9)
        sgn = np.sign(np.sum(U * Uo, axis=0))
        ns = min(p, 12)   # signal subspace; noise-level vectors are not identifiable
        np.testing.assert_allclose((U * sgn)[:, :ns], Uo[:, :ns], atol=1e-8)
        np.testing.assert_allclose((Vh * sgn[:, None])[:ns], Vo[:ns], atol=1e-8)
        # reference (float32) singular values of the signal part
        np.testing.assert_allclose(S[:ns], g[f"{tag}_S"][:ns], rtol=1e-4)
        np.testing.assert_allclose(U.T @ U, np.eye(p), atol=1e-10)


def test_randomized_svd_field(dev):
    """C5-like ensemble (512 x 10k smooth field + noise): top PCs match an exact SVD."""
    from gladsgp_amd.svd import randomized_svd
    rng = np.random.default_rng(5)
    n, ny, rank = 512, 10000, 20
    modes = rng.standard_normal((rank, ny)) * (0.6 ** np.arange(rank))[:, None]
    Y = rng.standard_normal((n, rank)) @ modes + 1e-3 * rng.standard_normal((n, ny))
    np.random.seed(0)
    U, S, Vh = randomized_svd(Y, 25, k=0, q=1, device=dev)
    S_ex = np.linalg.svd(Y, compute_uv=False)
    np.testing.assert_allclose(S[:10], S_ex[:10], rtol=1e-6)
    # reconstruction of the rank-20 part
    err = np.linalg.norm(Y - (U * S) @ Vh) / np.linalg.norm(Y)
    assert err < 1e-2
    # same Omega as the reference would draw after np.random.seed(0)
    np.random.seed(0)
    om = np.random.normal(size=(ny, 25)).astype(np.float32)
    _, So, _ = gp_ref.randomized_svd(Y, 25, k=0, q=1, omega=om)
    # singular values come from eig(B B^T): absolute error ~ eps S_max^2 / S_i (stated model)
    tol = 1e-9 * So + 1e-12 * So[0] ** 2 / So
    assert np.all(np.abs(S - So) <= tol)
