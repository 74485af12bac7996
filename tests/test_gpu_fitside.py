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
@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (70, 33, 129), (128, 64, 64), (17, 5, 60000),
                                   (512, 25, 70001), (20001, 25, 300), (25, 20001, 300),
                                   # tsm / tsm_t with the narrow side below one 16-wide MFMA
                                   # column tile (blas.hip's clamped column indices)
                                   (20001, 7, 300), (7, 20001, 300), (20001, 1, 300),
                                   (15, 20001, 300),
                                   # K = 16: one K-group, the prologue must not prefetch a second
                                   (16, 20001, 16), (20001, 16, 16),
                                   # tsk with a last K-slice of 8 (tsk_shape at m = 512: 288-long
                                   # slices, 69992 = 243 * 288 + 8)
                                   (512, 7, 69992)])
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


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("m,n,k", [(70, 33, 129), (512, 25, 40000), (3, 200, 7),
                                   # the tall-skinny kernels (blas.hip ts_kind): tsk (long K,
                                   # ta = 1), tsm (K <= 1024, the big side C's rows / C^T's)
                                   (512, 25, 70001), (700, 7, 65537), (20001, 25, 300),
                                   (25, 20001, 300), (32, 9000, 512),
                                   # even leading dimensions: the fp64 tsk runs take the
                                   # 16-B tsk16 form, the float32 runs the 8-B one
                                   (512, 25, 70000), (20000, 25, 300),
                                   # narrow side < 16 (tsm, tsm_t), K = 16, a last tsk slice of
                                   # 8 (69992) or 16 (70000 above) k
                                   (20001, 7, 300), (7, 20001, 300), (20001, 15, 300),
                                   (1, 20001, 300), (16, 20001, 16), (20001, 16, 16),
                                   (512, 25, 69992), (512, 7, 70000)])
def test_gemm_float32_operands_bit_identical(dev, ta, tb, m, n, k):
    """gp_gemm_ex with a float32 A and/or B (widened on load) equals gp_gemm_ex / gp_dgemm on
    fp64 copies of the same values bit for bit, split-K shapes included (512 x 25 x 40000 is
    the fit's X Omega shape at a shorter field)."""
    from gladsgp_amd.blas import CM, gemm
    rng = np.random.default_rng(7 * m + n + k + ta * 2 + tb)
    A = rng.standard_normal((k, m) if ta else (m, k)).astype(np.float32)
    B = rng.standard_normal((n, k) if tb else (k, n)).astype(np.float32)
    C0 = rng.standard_normal((m, n))

    def cm(M, dt):
        return CM(torch.as_tensor(M.T.copy(), device=dev).to(dt), M.shape[0], M.shape[1],
                  M.shape[0])

    res = {}
    for fa, fb in ((0, 0), (1, 0), (0, 1), (1, 1)):
        Cc = CM(_t(C0.T.copy(), dev), m, n, m)
        gemm(bool(ta), bool(tb), cm(A, torch.float32 if fa else torch.float64),
             cm(B, torch.float32 if fb else torch.float64), alpha=0.7, beta=-1.3, C=Cc)
        res[(fa, fb)] = Cc.logical().cpu().numpy()
    for key in ((1, 0), (0, 1), (1, 1)):
        assert np.array_equal(res[key], res[(0, 0)]), key
    ref = 0.7 * ((A.T if ta else A).astype(np.float64) @ (B.T if tb else B)) - 1.3 * C0
    np.testing.assert_allclose(res[(0, 0)], ref, rtol=1e-12,
                               atol=1e-12 * np.sqrt(k) * np.abs(ref).max())


@pytest.mark.parametrize("kind", ["tsk", "tsm", "tsm_t"])
@pytest.mark.parametrize("big,runs", [(70001, None), (20001, None), (20001, 16), (70000, 16)])
def test_tall_skinny_padded_ld_matches_unpadded(dev, kind, big, runs):
    """The ensemble's padded row stride (emulator.standardize_y) selects the 16-B tsk form
    (blas.hip tsk16); every tall-skinny product on the padded ensemble equals the one on an
    unpadded copy bit for bit, odd lengths (a 16-B pair straddling the row end, zeroed)
    included, and numpy within 1e-12."""
    from gladsgp_amd.blas import CM, gemm
    if kind == "tsk" and big < 65536:
        pytest.skip("tsk needs K >= 65536")
    rng = np.random.default_rng(big + len(kind) + (runs or 0))
    # runs = 16: the reference's test_install.sh ensemble (--nsim 16), K = 16 for tsm / tsm_t
    r = 25
    if runs is None:
        runs = 300 if kind != "tsk" else 512
    X = rng.standard_normal((runs, big))                 # C-order ensemble: runs x locations
    ld = (big + 15) // 16 * 16
    pad = torch.full((runs, ld), float("nan"), dtype=torch.float64, device=dev)
    pad[:, :big] = _t(X, dev)
    Xp = CM(pad, big, runs, ld)                          # (locations x runs), padded
    Xu = CM(_t(X, dev), big, runs, big)
    if kind == "tsk":                                    # (runs x r) = X W
        W = rng.standard_normal((big, r))
        Wc = CM(_t(W.T.copy(), dev), big, r, big)
        outs = [gemm(True, False, M, Wc).logical().cpu().numpy() for M in (Xp, Xu)]
        ref = X @ W
    elif kind == "tsm":                                  # (locations x r) = X^T Y
        Y = rng.standard_normal((runs, r))
        Yc = CM(_t(Y.T.copy(), dev), runs, r, runs)
        outs = [gemm(False, False, M, Yc).logical().cpu().numpy() for M in (Xp, Xu)]
        ref = X.T @ Y
    else:                                                # (r x locations) = Q^T X
        Q = rng.standard_normal((runs, r))
        Qc = CM(_t(Q.T.copy(), dev), runs, r, runs)
        outs = [gemm(True, True, Qc, M).logical().cpu().numpy() for M in (Xp, Xu)]
        ref = Q.T @ X
    assert np.array_equal(outs[0], outs[1])
    np.testing.assert_allclose(outs[0], ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())


def test_randomized_svd_float32_input_reads_no_fp64_copy(dev):
    """randomized_svd on a float32 ensemble (the reference's fit dtype) keeps it float32 on the
    device: its outputs equal the fp64-input run's outputs cast to float32, bit for bit."""
    from gladsgp_amd.svd import randomized_svd
    rng = np.random.default_rng(11)
    n, ny, r = 40, 6000, 12
    t = rng.random((n, 3))
    X = (np.sin(t @ rng.standard_normal((3, ny))) + 0.01 * rng.standard_normal((n, ny)))
    X32 = X.astype(np.float32)
    om = rng.standard_normal((ny, r)).astype(np.float32)
    X32d = torch.as_tensor(X32, device=dev)
    a = randomized_svd(X32d, r, k=0, q=1, omega=om)
    b = randomized_svd(X32d.to(torch.float64), r, k=0, q=1, omega=om)
    assert all(x.dtype == torch.float32 for x in a) and all(y.dtype == torch.float64 for y in b)
    for x, y in zip(a, b):
        assert torch.equal(x, y.to(torch.float32))


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
        # float32 input -> float32 outputs, as src/svd.py:51-68 returns for a float32 X
        U32, S32, Vh32 = randomized_svd(X.astype(np.float32), p, k=k, q=1,
                                        omega=g[f"{tag}_omega"], device=dev)
        assert U32.dtype == S32.dtype == Vh32.dtype == np.float32
        U, S, Vh = randomized_svd(X.astype(np.float64), p, k=k, q=1, omega=g[f"{tag}_omega"],
                                  device=dev)
        assert U.dtype == np.float64
        assert U.shape == (64, p) and S.shape == (p,) and Vh.shape == (p, 500)
        np.testing.assert_array_equal(S32, S.astype(np.float32))
        np.testing.assert_array_equal(U32, U.astype(np.float32))
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


@pytest.mark.parametrize("n", [16, 20, 25])
def test_randomized_svd_rank_deficient_vs_reference(dev, golden_dir, n):
    """init_model's r = min(25, n, ny) on a column-centred ensemble of n <= 25 runs (rank
    <= n - 1: a CholeskyQR pass hits a zero pivot): the reference's own src/svd.py outputs
    (tests/golden/svd_ref_deficient.npz) vs the GPU with the same Omega."""
    from gladsgp_amd.svd import randomized_svd
    g = np.load(os.path.join(golden_dir, "svd_ref_deficient.npz"))
    y_std = g[f"n{n}_y_std"]
    r = min(25, *y_std.shape)
    # fp64 input: fp64 outputs, compared tightly (a float32 input returns float32, as the
    # reference's src/svd.py does: test_randomized_svd_vs_reference_golden)
    U, S, Vh = randomized_svd(y_std.astype(np.float64), r, k=0, q=1, omega=g[f"n{n}_omega"],
                              device=dev)
    assert U.shape == (n, r) and S.shape == (r,) and Vh.shape == (r, y_std.shape[1])
    assert np.all(np.isfinite(U)) and np.all(np.isfinite(S)) and np.all(np.isfinite(Vh))
    np.testing.assert_allclose(U.T @ U, np.eye(r), atol=1e-10)
    S_ref = g[f"n{n}_S"]
    # the n - 1 nonzero singular values (float32 reference), the last one numerically zero
    np.testing.assert_allclose(S[: n - 1], S_ref[: n - 1], rtol=2e-4, atol=1e-4 * S_ref[0])
    assert S[-1] <= 1e-6 * S[0]
    # exact SVD of the (rank n-1) input: the GPU's fp64 values are tight
    S_ex = np.linalg.svd(y_std.astype(np.float64), compute_uv=False)
    np.testing.assert_allclose(S[: n - 1], S_ex[: n - 1], rtol=1e-8)
    # leading, well-separated singular vectors agree with the reference up to sign
    U_ref, Vh_ref = g[f"n{n}_U"], g[f"n{n}_Vh"]
    for i in range(3):
        if (S_ref[i] - S_ref[i + 1]) > 1e-2 * S_ref[0]:
            sg = np.sign(U[:, i] @ U_ref[:, i])
            np.testing.assert_allclose(sg * U[:, i], U_ref[:, i], atol=1e-3)
            np.testing.assert_allclose(sg * Vh[i], Vh_ref[i], atol=1e-3)
    # reconstruction of the input from the rank-r factors
    err = np.linalg.norm(y_std - (U * S) @ Vh) / np.linalg.norm(y_std)
    assert err < 1e-6


def test_init_model_small_ensemble(dev, tmp_path):
    """init_model at the reference's test_install.sh size (--nsim 16): no failure, finite
    basis, PC weights of the GPU basis match the oracle."""
    from gladsgp_amd import model as gm
    rng = np.random.default_rng(16)
    t = rng.random((16, 8))
    y = (2.0 + np.sin(2 * np.pi * t @ rng.uniform(0, 1, 8))[:, None]
         * rng.standard_normal((1, 300)) + 0.1 * rng.standard_normal((16, 300)))
    data, model = gm.init_model(t.astype(np.float32), y.astype(np.float32), "tiny", 5,
                                data_dir=str(tmp_path), device=dev, verbose=False)
    K = data.sim_data.K.cpu().numpy()
    assert K.shape == (5, 300) and np.all(np.isfinite(K))
    ystd = data.sim_data.y_std.cpu().numpy()
    np.testing.assert_allclose(model.w_hat.cpu().numpy(), gp_ref.pc_weights(ystd, K),
                               atol=1e-7)


@pytest.mark.parametrize("p,k", [(100, None), (150, 0)])
def test_randomized_svd_large_rank(dev, p, k):
    """p + k beyond the old 128 cap (the reference's default k=None doubles p; plot_PC_RMSE.py
    uses p = min(100, n)): 200 x 3000 input, against numpy with the same Omega."""
    from gladsgp_amd.svd import randomized_svd
    rng = np.random.default_rng(p)
    X = rng.standard_normal((400, 60)) @ rng.standard_normal((60, 3000)) \
        + 0.01 * rng.standard_normal((400, 3000))
    r = p + (p if k is None else k)
    om = rng.standard_normal((3000, r)).astype(np.float32)
    U, S, Vh = randomized_svd(X, p, k=k, q=1, omega=om, device=dev)
    assert U.shape == (400, p) and S.shape == (p,) and Vh.shape == (p, 3000)
    _, So, _ = gp_ref.randomized_svd(X, p, k=k, q=1, omega=om)
    tol = 1e-9 * So + 1e-12 * So[0] ** 2 / So
    assert np.all(np.abs(S - So) <= tol)
    np.testing.assert_allclose(U.T @ U, np.eye(p), atol=1e-10)


def test_init_model_caches_reference_dtype(dev, tmp_path):
    """float32 ensembles (fit_models / load_model's default dtype) cache float32
    pca_*_{U,S,Vh}.npy like the reference (src/svd.py:51, model.py:87-89); float64 stays
    float64."""
    from gladsgp_amd import model as gm
    rng = np.random.default_rng(3)
    t = rng.random((40, 8))
    y = 1.0 + np.sin(2 * np.pi * t @ rng.uniform(0, 1, 8))[:, None] * rng.standard_normal(
        (1, 500)) + 0.05 * rng.standard_normal((40, 500))
    for dt in (np.float32, np.float64):
        d = tmp_path / np.dtype(dt).name
        gm.init_model(t.astype(dt), y.astype(dt), "dt", 4, data_dir=str(d), device=dev,
                      verbose=False)
        for a in ("U", "S", "Vh"):
            assert np.load(d / f"pca_dt_{a}.npy").dtype == dt


@pytest.mark.parametrize("n", [16, 20])
def test_init_model_matches_reference_pmax25_call(dev, golden_dir, tmp_path, n):
    """The build's init_model (n < 25 runs: Omega's first n columns, gladsgp_amd/model.py)
    against the reference's randomized_svd called as src/model.py:81-84 calls it
    (tests/golden/svd_ref_pmax25.npz: pmax = 25, Omega (ny, 25)): cached S to rtol on the n - 1
    nonzero values, U / Vh up to sign on the leading well-separated vectors, the same cached
    shapes and dtypes, and the same advance of numpy's global RNG."""
    from gladsgp_amd import model as gm
    g = np.load(os.path.join(golden_dir, "svd_ref_pmax25.npz"))
    t, y = g[f"n{n}_t"], g[f"n{n}_y"]
    ny = y.shape[1]
    np.random.seed(int(g[f"n{n}_seed"]))
    gm.init_model(t, y, "pm", 5, data_dir=str(tmp_path), device=dev, verbose=False)
    assert np.random.random() == float(g[f"n{n}_next_random"])
    U = np.load(tmp_path / "pca_pm_U.npy")
    S = np.load(tmp_path / "pca_pm_S.npy")
    Vh = np.load(tmp_path / "pca_pm_Vh.npy")
    S_ref, U_ref, Vh_ref = g[f"n{n}_S"], g[f"n{n}_U"], g[f"n{n}_Vh"]
    assert U.shape == U_ref.shape == (n, n) and S.shape == S_ref.shape == (n,)
    assert Vh.shape == Vh_ref.shape == (n, ny)
    assert U.dtype == S.dtype == Vh.dtype == np.float32
    np.testing.assert_allclose(S[: n - 1], S_ref[: n - 1], rtol=2e-4, atol=1e-4 * S_ref[0])
    assert S[-1] <= 1e-4 * S[0]
    checked = 0
    for i in range(4):
        if S_ref[i] - S_ref[i + 1] > 1e-2 * S_ref[0]:
            sg = np.sign(U[:, i] @ U_ref[:, i])
            np.testing.assert_allclose(sg * U[:, i], U_ref[:, i], atol=1e-3)
            np.testing.assert_allclose(sg * Vh[i], Vh_ref[i], atol=1e-3)
            checked += 1
    assert checked >= 2
