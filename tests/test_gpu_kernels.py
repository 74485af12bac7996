"""GPU parity: libgpfit kernels vs the numpy fp64 oracle (called through the C ABI).

Tolerances (fp64, stated per SURVEY §8c and measured):
  Gram          max|dG| <= 8 eps * s          (exp differs by a few ulp between libm and ocml)
  Cholesky      ||L L^T - G||_F / ||G||_F <= 1e-13 ; ||L^-1 L - I||_max <= 1e-9 (kappa-limited)
  logdet        |d| <= 1e-9 * n
  predict (C2)  max|dmean| <= 1e-8 max|mean| , max|dvar| <= 1e-9 s   (kappa(G) ~ 1e8 at 1e-6 jitter)
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import gp_ref

pytestmark = pytest.mark.gpu

EPS = np.finfo(np.float64).eps


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    from gladsgp_amd import kernels  # noqa: F401 (loads libgpfit.so)
    return torch.device("cuda:0")


def _t(x, dev):
    return torch.as_tensor(np.asarray(x, dtype=np.float64), device=dev)


def _c2(golden_dir):
    return np.load(os.path.join(golden_dir, "c2_golden.npz"))


def test_library_is_native(dev):
    from gladsgp_amd import _capi
    lib = _capi.lib()
    assert lib.gp_version() >= 100
    with open("/proc/self/maps") as f:
        assert "libgpfit.so" in f.read()


@pytest.mark.parametrize("n,d", [(1, 1), (7, 3), (64, 8), (129, 8), (512, 8), (300, 17)])
def test_gram_matches_oracle(dev, n, d):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(n + d)
    X = rng.random((n, d))
    beta = rng.uniform(0.5, 5.0, d)
    s, delta = 1.3, 1e-6
    G = kernels.gram(_t(X, dev), _t(beta, dev), s, delta)[0].cpu().numpy()
    ref = gp_ref.gram_ardse(X, beta, s, delta)
    assert np.max(np.abs(G - ref)) <= 8 * EPS * s
    np.testing.assert_array_equal(G, G.T)


def test_gram_batched_and_c2_golden(dev, golden_dir):
    from gladsgp_amd import kernels
    g = _c2(golden_dir)
    rng = np.random.default_rng(3)
    betas = np.stack([g["beta"], rng.uniform(0.5, 5, 8), rng.uniform(0.1, 2, 8)])
    s = np.array([1.0, 0.7, 2.0])
    delta = np.array([1e-6, 1e-4, 1e-2])
    G = kernels.gram(_t(g["X"], dev), _t(betas, dev), _t(s, dev), _t(delta, dev)).cpu().numpy()
    idx = g["gram_idx"]
    np.testing.assert_allclose(G[0][idx[:, 0], idx[:, 1]], g["gram_vals"], rtol=0, atol=8 * EPS)
    for b in range(3):
        ref = gp_ref.gram_ardse(g["X"], betas[b], s[b], delta[b])
        assert np.max(np.abs(G[b] - ref)) <= 8 * EPS * s[b]


def test_cross_matches_oracle(dev):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(11)
    X, Xs = rng.random((200, 8)), rng.random((333, 8))
    beta = rng.uniform(0.5, 5, 8)
    Kt = kernels.cross(_t(X, dev), _t(Xs, dev), _t(beta, dev), 0.9)[0].cpu().numpy()
    ref = gp_ref.cross_ardse(Xs, X, beta, 0.9)
    assert np.max(np.abs(Kt - ref)) <= 8 * EPS


@pytest.mark.parametrize("n", [1, 5, 63, 64, 65, 127, 128, 129, 200, 512, 1000, 2100])
def test_cholesky_inverse(dev, n):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(n)
    X = rng.random((n, 8))
    beta = rng.uniform(0.5, 5, 8)
    G = gp_ref.gram_ardse(X, beta, 1.0, 1e-4)
    Gt = _t(G, dev).unsqueeze(0).contiguous()
    ch = kernels.cholesky_inverse(Gt)
    assert int(ch.info[0]) == 0
    L = ch.L[0].cpu().numpy()
    Linv = ch.Linv[0].cpu().numpy()
    Lref = np.linalg.cholesky(G)
    assert np.linalg.norm(L @ L.T - G) / np.linalg.norm(G) <= 1e-13
    assert np.max(np.abs(L - Lref)) <= 1e-10 * np.max(np.abs(Lref))
    assert np.max(np.abs(Linv @ L - np.eye(n))) <= 1e-9
    np.testing.assert_allclose(float(ch.logdet[0]), 2 * np.sum(np.log(np.diag(Lref))),
                               rtol=0, atol=1e-9 * n)
    # padding of the L^-1 buffer and its upper triangle are zero
    full = ch.linv_buf[0].transpose(0, 1).cpu().numpy()
    assert np.all(np.triu(full, 1) == 0)
    assert np.all(full[n:, :] == 0) and np.all(full[:, n:] == 0)


@pytest.mark.parametrize("n,B", [(5, 1), (65, 2), (129, 1), (700, 2), (1000, 1)])
def test_cholesky_inverse_poisoned_buffer(dev, n, B):
    """The factorisation writes every entry of the padded L^-1 buffer itself -- the persistent
    kernel's zero tasks (upper tiles, pure-padding tile row / column) and its zero-padded
    diagonal blocks replace the caller-stream memset (round 4) -- so a buffer pre-filled with
    NaN comes back exactly zero above the diagonal and in the padding, and the same L^-1 as a
    zero-filled one."""
    from gladsgp_amd import _capi, kernels
    rng = np.random.default_rng(100 + n)
    X = rng.random((n, 8))
    G = np.stack([gp_ref.gram_ardse(X, rng.uniform(0.5, 5, 8), 1.0, 1e-4) for _ in range(B)])
    npad = kernels.padded_n(n)
    ws_b = int(_capi.lib().gp_potrf_inv_ws_bytes(n, B))
    ws = torch.empty(max(ws_b, 256), dtype=torch.uint8, device=dev)
    outs = []
    for fill in (float("nan"), 0.0):
        A = _t(G, dev).contiguous()
        Linv = torch.full((B, npad, npad), fill, dtype=torch.float64, device=dev)
        info = torch.empty(B, dtype=torch.int32, device=dev)
        logdet = torch.empty(B, dtype=torch.float64, device=dev)
        _capi.call("gp_potrf_inv_ws", A.data_ptr(), n, n, n * n, Linv.data_ptr(), npad,
                   npad * npad, B, info.data_ptr(), logdet.data_ptr(), ws.data_ptr(),
                   ws.numel(), torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize()
        assert info.cpu().tolist() == [0] * B
        outs.append(Linv.transpose(1, 2).cpu().numpy())          # [b][row][col]
    full = outs[0]
    assert np.all(np.isfinite(full))
    for b in range(B):
        assert np.all(np.triu(full[b], 1) == 0)
        assert np.all(full[b][n:, :] == 0) and np.all(full[b][:, n:] == 0)
        Lref = np.linalg.cholesky(G[b])
        assert np.max(np.abs(full[b][:n, :n] @ Lref - np.eye(n))) <= 1e-9
    assert np.array_equal(full, outs[1])


def test_cholesky_upper_triangle_untouched(dev):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(2)
    n = 150
    X = rng.random((n, 4))
    G = gp_ref.gram_ardse(X, np.ones(4), 1.0, 1e-3)
    A = G.copy()
    A[np.triu_indices(n, 1)] = 123.0   # LAPACK potrf('L') never reads/writes the upper part
    At = _t(A.T.copy(), dev).unsqueeze(0).contiguous()   # column-major buffer
    ch = kernels.cholesky_inverse(At)
    buf = ch.a_buf[0].transpose(0, 1).cpu().numpy()
    assert np.all(buf[np.triu_indices(n, 1)] == 123.0)
    np.testing.assert_allclose(np.tril(buf), np.linalg.cholesky(G), atol=1e-12)


@pytest.mark.parametrize("n,bad", [(10, 3), (100, 1), (100, 64), (100, 65), (300, 200)])
def test_cholesky_info_not_pd(dev, n, bad):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(n)
    A = rng.standard_normal((n, n))
    G = A @ A.T + n * np.eye(n)
    G[bad - 1, bad - 1] = -1.0
    _, info_ref = gp_ref.cholesky(G)
    ch = kernels.cholesky_inverse(_t(G, dev).unsqueeze(0).contiguous())
    assert int(ch.info[0]) == info_ref == bad


def test_cholesky_batch_persistent_update(dev):
    """A batch large enough that the update grid is capped: workers walk several tiles."""
    from gladsgp_amd import kernels
    rng = np.random.default_rng(21)
    n, B = 1100, 6
    Gs = []
    for b in range(B):
        X = rng.random((n, 8))
        Gs.append(gp_ref.gram_ardse(X, rng.uniform(0.5, 5, 8), 1.0, 1e-3))
    ch = kernels.cholesky_inverse(_t(np.stack(Gs), dev).contiguous())
    assert ch.info.cpu().tolist() == [0] * B
    for b in range(B):
        L = ch.L[b].cpu().numpy()
        assert np.linalg.norm(L @ L.T - Gs[b]) / np.linalg.norm(Gs[b]) <= 1e-13
        Linv = ch.Linv[b].cpu().numpy()
        assert np.max(np.abs(Linv @ L - np.eye(n))) <= 1e-9


def test_cholesky_batch_mixed_info(dev):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(9)
    n = 96
    Gs = []
    for b in range(4):
        A = rng.standard_normal((n, n))
        G = A @ A.T + n * np.eye(n)
        if b == 2:
            G[70, 70] = -3.0
        Gs.append(G)
    ch = kernels.cholesky_inverse(_t(np.stack(Gs), dev).contiguous())
    assert ch.info.cpu().tolist() == [0, 0, 71, 0]
    for b in (0, 1, 3):
        L = ch.L[b].cpu().numpy()
        assert np.linalg.norm(L @ L.T - Gs[b]) / np.linalg.norm(Gs[b]) <= 1e-13


def _predict_gpu(dev, X, Xs, w, beta, s, delta, s_pred=None, m_chunk=0):
    from gladsgp_amd import kernels
    s_pred = s if s_pred is None else s_pred
    G = kernels.gram(_t(X, dev), _t(beta, dev), s, delta)
    ch = kernels.cholesky_inverse(G)
    ch.check()
    mean, var = kernels.predict(ch, _t(X, dev), _t(Xs, dev), _t(beta, dev), s, s_pred,
                                _t(w, dev), m_chunk=m_chunk)
    return mean[0].cpu().numpy(), var[0].cpu().numpy()


def test_predict_c2_golden(dev, golden_dir):
    g = _c2(golden_dir)
    mean, var = _predict_gpu(dev, g["X"], g["Xs"], g["y"], g["beta"], float(g["s"]),
                             float(g["delta"]))
    assert np.max(np.abs(mean - g["mean"])) <= 1e-8 * np.max(np.abs(g["mean"]))
    assert np.max(np.abs(var - g["var"])) <= 1e-9 * float(g["s"])


def test_predict_c2_full_m10k(dev, golden_dir):
    """BASELINE config 2: real 512x8 design, m = 10k seeded test points."""
    g = _c2(golden_dir)
    Xs = np.random.default_rng(2).random((10000, 8))
    mean_ref, var_ref = gp_ref.predict(g["X"], Xs, g["y"], g["beta"], 1.0, 1e-6)
    mean, var = _predict_gpu(dev, g["X"], Xs, g["y"], g["beta"], 1.0, 1e-6)
    assert np.max(np.abs(mean - mean_ref)) <= 1e-8 * np.max(np.abs(mean_ref))
    assert np.max(np.abs(var - var_ref)) <= 1e-9


@pytest.mark.parametrize("n,m,d,chunk", [(1, 1, 1, 0), (5, 51, 1, 0), (65, 129, 3, 0),
                                         (130, 300, 8, 128), (256, 1000, 8, 384),
                                         (700, 257, 16, 0),
                                         # z = L^-1 w's two passes at npad = 1152 (an odd
                                         # number of 128-row tiles), default and small chunks
                                         (1100, 2000, 8, 0), (1100, 300, 8, 128)])
def test_predict_edges(dev, n, m, d, chunk):
    rng = np.random.default_rng(n * 7 + m)
    X, Xs = rng.random((n, d)), rng.random((m, d))
    beta = rng.uniform(0.5, 3, d)
    w = rng.standard_normal(n)
    s, delta = 1.5, 1e-3
    mean_ref, var_ref = gp_ref.predict(X, Xs, w, beta, s, delta, s_pred=s + 0.01)
    mean, var = _predict_gpu(dev, X, Xs, w, beta, s, delta, s_pred=s + 0.01, m_chunk=chunk)
    np.testing.assert_allclose(mean, mean_ref, rtol=0, atol=1e-9 * max(1, np.abs(mean_ref).max()))
    np.testing.assert_allclose(var, var_ref, rtol=0, atol=1e-10 * s)


def test_predict_batched_per_problem_params(dev):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(4)
    n, m, d, B = 300, 500, 8, 5
    X, Xs = rng.random((n, d)), rng.random((m, d))
    betas = rng.uniform(0.5, 4, (B, d))
    s = rng.uniform(0.5, 2, B)
    delta = rng.uniform(1e-5, 1e-2, B)
    sp = s + rng.uniform(0, 0.1, B)
    W = rng.standard_normal((B, n))
    G = kernels.gram(_t(X, dev), _t(betas, dev), _t(s, dev), _t(delta, dev))
    ch = kernels.cholesky_inverse(G)
    mean, var = kernels.predict(ch, _t(X, dev), _t(Xs, dev), _t(betas, dev), _t(s, dev),
                                _t(sp, dev), _t(W, dev), m_chunk=256)
    mean, var = mean.cpu().numpy(), var.cpu().numpy()
    for b in range(B):
        mr, vr = gp_ref.predict(X, Xs, W[b], betas[b], s[b], delta[b], s_pred=sp[b])
        np.testing.assert_allclose(mean[b], mr, atol=1e-9 * np.abs(mr).max())
        np.testing.assert_allclose(var[b], vr, atol=1e-10)


def test_nll_known_answer(dev, golden_dir):
    """GPmodule objective at the notebook-02 optimum (fun = -3.989954265337257)."""
    from gladsgp_amd import kernels
    ka = json.load(open(os.path.join(golden_dir, "nb02_known_answer.json")))
    x = np.asarray(ka["x_train"]).reshape(-1, 1)
    y = np.asarray(ka["y_train"])
    s, beta, delta = gp_ref.gpmodule_theta_to_kernel(ka["oracle_theta"], ka["nugget"])
    ch = kernels.cholesky_inverse(kernels.gram(_t(x, dev), _t(beta, dev), s, delta))
    v = float(kernels.nll(ch, _t(y, dev))[0])
    assert abs(v - ka["oracle_fun"]) < 1e-12
    assert abs(v - ka["printed_fun"]) < 1e-7


def test_nll_c2(dev, golden_dir):
    from gladsgp_amd import kernels
    g = _c2(golden_dir)
    ch = kernels.cholesky_inverse(kernels.gram(_t(g["X"], dev), _t(g["beta"], dev), 1.0, 1e-6))
    assert abs(float(ch.logdet[0]) - float(g["logdet"])) <= 1e-8 * abs(float(g["logdet"]))
    v = float(kernels.nll(ch, _t(g["y"], dev))[0])
    assert abs(v - float(g["nll"])) <= 1e-8 * abs(float(g["nll"]))


def test_cpu_tensor_rejected(dev):
    from gladsgp_amd import kernels
    with pytest.raises(ValueError):
        kernels.gram(torch.zeros(4, 2, dtype=torch.float64), [1.0, 1.0], 1.0, 0.0)


def test_two_phase_predict_and_overlap_match_single(dev):
    """gp_predict_cross + gp_predict_solve and gp_fit_predict (serial and with a context)
    == gp_predict, bit for bit."""
    from gladsgp_amd import kernels
    rng = np.random.default_rng(21)
    n, m, d, B = 333, 5000, 8, 3
    X, Xs = rng.random((n, d)), rng.random((m, d))
    betas = rng.uniform(0.5, 4, (B, d))
    s = rng.uniform(0.5, 2, B)
    delta = rng.uniform(1e-5, 1e-3, B)
    W = rng.standard_normal((B, n))
    Xd, Xsd = _t(X, dev), _t(Xs, dev)
    ch = kernels.cholesky_inverse(kernels.gram(Xd, _t(betas, dev), _t(s, dev), _t(delta, dev)))
    m1, v1 = kernels.predict(ch, Xd, Xsd, _t(betas, dev), _t(s, dev), _t(s, dev), _t(W, dev),
                             m_chunk=1024)
    prep = kernels.predict_prepare(Xd, Xsd, _t(betas, dev), _t(s, dev), batch=B, m_chunk=1024)
    m2, v2 = kernels.predict_solve(ch, prep, _t(s, dev), _t(W, dev))
    assert torch.equal(m1, m2) and torch.equal(v1, v2)
    # gp_fit_predict with a context: cross-covariance on the masked stream under the
    # factorisation; and without one: every step in order on the caller's stream
    with kernels.FitPredictContext(dev) as fctx:
        m3, v3, ch3 = kernels.fit_predict(Xd, Xsd, _t(betas, dev), _t(s, dev), _t(delta, dev),
                                          _t(s, dev), _t(W, dev), m_chunk=1024, ctx=fctx)
        # the same context again with more chunks (its per-chunk events grow on demand; each
        # chunk's TRMM waits for its own chunk's cross-covariance only)
        m5, v5, _ = kernels.fit_predict(Xd, Xsd, _t(betas, dev), _t(s, dev), _t(delta, dev),
                                        _t(s, dev), _t(W, dev), m_chunk=384, ctx=fctx)
        # gp_ctx_set_aux_chunks: none / one / two of the chunks' cross-covariance on the aux
        # stream, the rest on the prediction stream before their TRMM; then all again
        late = []
        for k in (0, 1, 2, -1):
            fctx.set_aux_chunks(k)
            late.append(kernels.fit_predict(Xd, Xsd, _t(betas, dev), _t(s, dev),
                                            _t(delta, dev), _t(s, dev), _t(W, dev), m_chunk=384,
                                            ctx=fctx)[:2])
        torch.cuda.synchronize()
    assert torch.equal(m1, m3) and torch.equal(v1, v3)
    assert torch.equal(m1, m5) and torch.equal(v1, v5)
    for mk, vk in late:
        assert torch.equal(m1, mk) and torch.equal(v1, vk)
    assert torch.equal(ch3.L, ch.L) and torch.equal(ch3.Linv, ch.Linv)
    assert torch.equal(ch3.logdet, ch.logdet) and int(ch3.info.abs().sum()) == 0
    m4, v4, _ = kernels.fit_predict(Xd, Xsd, _t(betas, dev), _t(s, dev), _t(delta, dev),
                                    _t(s, dev), _t(W, dev), m_chunk=1024)
    torch.cuda.synchronize()
    assert torch.equal(m1, m4) and torch.equal(v1, v4)


@pytest.mark.parametrize("n,m,B", [(64, 700, 1), (129, 300, 2), (513, 5000, 3)])
def test_fit_predict_edge_shapes(dev, n, m, B):
    """gp_fit_predict == gram -> cholesky_inverse -> predict at odd sizes: one 64-block (the
    cross-covariance starts at once), partial tiles, fewer test points than one chunk."""
    from gladsgp_amd import kernels
    rng = np.random.default_rng(n + m)
    d = 5
    X, Xs = rng.random((n, d)), rng.random((m, d))
    betas = rng.uniform(0.5, 4, (B, d))
    s = rng.uniform(0.5, 2, B)
    delta = rng.uniform(1e-5, 1e-3, B)
    W = rng.standard_normal((B, n))
    Xd, Xsd = _t(X, dev), _t(Xs, dev)
    ch = kernels.cholesky_inverse(kernels.gram(Xd, _t(betas, dev), _t(s, dev), _t(delta, dev)))
    m1, v1 = kernels.predict(ch, Xd, Xsd, _t(betas, dev), _t(s, dev), _t(s, dev), _t(W, dev))
    with kernels.FitPredictContext(dev) as fctx:
        m2, v2, ch2 = kernels.fit_predict(Xd, Xsd, _t(betas, dev), _t(s, dev), _t(delta, dev),
                                          _t(s, dev), _t(W, dev), ctx=fctx)
        torch.cuda.synchronize()
    assert torch.equal(m1, m2) and torch.equal(v1, v2)
    assert torch.equal(ch.logdet, ch2.logdet)
    for b in range(B):
        ref_m, ref_v = gp_ref.predict(X, Xs, W[b], betas[b], s[b], delta[b])
        np.testing.assert_allclose(m2[b].cpu().numpy(), ref_m, rtol=0,
                                   atol=1e-8 * max(1.0, np.abs(ref_m).max()))
        np.testing.assert_allclose(v2[b].cpu().numpy(), ref_v, rtol=0, atol=1e-9 * s[b])


def test_fit_predict_reports_non_pd(dev):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(3)
    n, m, d = 200, 1000, 3
    X, Xs = rng.random((n, d)), rng.random((m, d))
    betas = np.full((2, d), 1.0)
    s = np.array([1.0, 1.0])
    delta = np.array([1e-4, -3.0])          # problem 1 is indefinite
    W = rng.standard_normal((2, n))
    with pytest.raises(ValueError, match="not positive definite"):   # check=True (default)
        kernels.fit_predict(_t(X, dev), _t(Xs, dev), _t(betas, dev), _t(s, dev),
                            _t(delta, dev), _t(s, dev), _t(W, dev))
    mean, var, ch = kernels.fit_predict(_t(X, dev), _t(Xs, dev), _t(betas, dev), _t(s, dev),
                                        _t(delta, dev), _t(s, dev), _t(W, dev), check=False)
    torch.cuda.synchronize()
    info = ch.info.cpu().numpy()
    assert info[0] == 0 and info[1] > 0
    with pytest.raises(ValueError):
        ch.check()
    ref_m, _ = gp_ref.predict(X, Xs, W[0], betas[0], s[0], delta[0])
    np.testing.assert_allclose(mean[0].cpu().numpy(), ref_m, rtol=0,
                               atol=1e-8 * max(1.0, np.abs(ref_m).max()))


def test_native_comm_world1(dev):
    """gp_comm_* (RCCL C-ABI) at world size 1: broadcast leaves the buffer, gather stacks it."""
    from gladsgp_amd import _capi
    from gladsgp_amd import dist as gd
    assert _capi.lib().gp_comm_available() == 1
    ctx = gd.Context(0, 1, 0, dev, None)
    comm = gd.NativeComm(ctx)
    x = torch.arange(1000, dtype=torch.float64, device=dev)
    comm.bcast_(x)
    g = comm.gather(x)
    torch.cuda.synchronize()
    assert torch.equal(x, torch.arange(1000, dtype=torch.float64, device=dev))
    assert g.shape == (1, 1000) and torch.equal(g[0], x)
    comm.close()


@pytest.mark.parametrize("n,B", [(1, 1), (63, 2), (64, 1), (200, 3), (777, 2), (1500, 1)])
def test_potrf_plain_matches_potrf_inv(dev, n, B):
    """gp_potrf (L only, LAPACK dpotrf('L')) == gp_potrf_inv's L bit for bit, with the same
    logdet; the strict upper triangle is left untouched."""
    from gladsgp_amd import kernels
    rng = np.random.default_rng(n)
    X = rng.random((n, 6))
    betas = rng.uniform(0.5, 4, (B, 6))
    s = rng.uniform(0.5, 2, B)
    delta = rng.uniform(1e-6, 1e-3, B)
    G = kernels.gram(_t(X, dev), _t(betas, dev), _t(s, dev), _t(delta, dev))
    G2 = G.clone()
    ch = kernels.cholesky_inverse(G)
    sentinel = torch.triu(torch.full_like(G2, 7.0), diagonal=1).transpose(-1, -2)
    G2 = torch.where(sentinel == 7.0, sentinel, G2).contiguous()   # buffer's strict upper = 7
    L, info, logdet = kernels.cholesky(G2)
    torch.cuda.synchronize()
    assert int(info.abs().sum()) == 0
    assert torch.equal(L, ch.L)
    assert torch.equal(logdet, ch.logdet)
    assert bool((torch.triu(G2.transpose(-1, -2), diagonal=1)[
        torch.triu(torch.ones(n, n, device=dev, dtype=torch.bool), diagonal=1).expand(B, n, n)]
        == 7.0).all())
    for b in range(B):
        ref = np.linalg.cholesky(gp_ref.gram_ardse(X, betas[b], s[b], delta[b]))
        np.testing.assert_allclose(L[b].cpu().numpy(), ref, rtol=0, atol=1e-12)


def test_potrf_plain_reports_non_pd(dev):
    from gladsgp_amd import kernels
    rng = np.random.default_rng(5)
    X = rng.random((300, 3))
    G = kernels.gram(_t(X, dev), _t(np.ones((2, 3)), dev), _t([1.0, 1.0], dev),
                     _t([1e-4, -3.0], dev))
    ref_info = gp_ref.cholesky(gp_ref.gram_ardse(X, np.ones(3), 1.0, -3.0))[1]
    _, info, _ = kernels.cholesky(G)
    info = info.cpu().numpy()
    assert info[0] == 0 and info[1] == ref_info


@pytest.mark.parametrize("n,B", [(1, 1), (64, 1), (65, 2), (300, 3), (1100, 1)])
def test_trtri_matches_inverse(dev, n, B):
    """gp_trtri(L) vs numpy's inverse of the same L, and vs gp_potrf_inv's L^-1."""
    from gladsgp_amd import kernels
    rng = np.random.default_rng(n + 1)
    X = rng.random((n, 5))
    betas = rng.uniform(0.5, 3, (B, 5))
    G = kernels.gram(_t(X, dev), _t(betas, dev), _t(np.ones(B), dev), _t(np.full(B, 1e-3), dev))
    ch = kernels.cholesky_inverse(G)
    tr = kernels.trtri(ch.L)
    torch.cuda.synchronize()
    assert int(tr.info.abs().sum()) == 0
    npad = kernels.padded_n(n)
    Li = tr.linv_buf.transpose(-1, -2).cpu().numpy()
    assert np.all(Li[:, :n, n:] == 0) and np.all(Li[:, n:, :] == 0)
    for b in range(B):
        L = ch.L[b].cpu().numpy()
        inv = np.linalg.inv(L)
        X_ = Li[b, :n, :n]
        assert np.all(np.triu(X_, 1) == 0)
        scale = np.abs(inv).max()
        assert np.max(np.abs(X_ - inv)) <= 1e-10 * scale
        assert np.max(np.abs(X_ @ L - np.eye(n))) <= 1e-10
        assert np.max(np.abs(X_ - ch.Linv[b].cpu().numpy())) <= 1e-10 * scale
    assert npad == Li.shape[-1]
    # log|A| from the factor agrees with the factorisation's
    np.testing.assert_allclose(tr.logdet.cpu().numpy(), ch.logdet.cpu().numpy(), rtol=1e-12)


def test_trtri_reports_zero_diagonal(dev):
    from gladsgp_amd import kernels
    L = torch.eye(130, dtype=torch.float64, device=dev).repeat(2, 1, 1)
    L[1, 70, 70] = 0.0
    tr = kernels.trtri(L)
    assert tr.info.cpu().tolist() == [0, 71]
    assert torch.equal(tr.Linv[0], torch.eye(130, dtype=torch.float64, device=dev))


def test_predict_from_cholesky_factor(dev):
    """gp_predict_chol(L) (a caller holding a LAPACK factor) == gp_predict(L^-1) to rounding."""
    from gladsgp_amd import kernels
    rng = np.random.default_rng(9)
    n, m, d, B = 700, 3000, 8, 2
    X, Xs = rng.random((n, d)), rng.random((m, d))
    betas = rng.uniform(0.5, 4, (B, d))
    s = np.array([1.0, 1.7])
    delta = np.array([1e-5, 1e-3])
    W = rng.standard_normal((B, n))
    G = kernels.gram(_t(X, dev), _t(betas, dev), _t(s, dev), _t(delta, dev))
    L, info, _ = kernels.cholesky(G)
    mean, var, info2 = kernels.predict_chol(L, _t(X, dev), _t(Xs, dev), _t(betas, dev),
                                            _t(s, dev), _t(s, dev), _t(W, dev))
    assert int(info.abs().sum()) == 0 and int(info2.abs().sum()) == 0
    for b in range(B):
        mr, vr = gp_ref.predict(X, Xs, W[b], betas[b], s[b], delta[b])
        np.testing.assert_allclose(mean[b].cpu().numpy(), mr, rtol=0,
                                   atol=1e-8 * max(1.0, np.abs(mr).max()))
        np.testing.assert_allclose(var[b].cpu().numpy(), vr, rtol=0, atol=1e-9 * s[b])


@pytest.mark.parametrize("n,ell", [(64, 0.05), (64, 0.2), (300, 0.05), (1000, 0.1)])
def test_cholesky_grid_gram_ill_conditioned(dev, n, ell):
    """Regression: 1-D grid Grams (BASELINE C1's shape, x = linspace(1/8, 7/8, n)) whose
    Schur-complement pivots fall to ~1e-4 |A| within a few columns.  Round 1's diagonal factor
    mixed the two rounding-level copies of the symmetric trailing block and lost L from column
    ~10 (kappa ~1e6); checked here against numpy at kappa up to ~1e8."""
    from gladsgp_amd import kernels
    x = np.linspace(1 / 8, 7 / 8, n).reshape(-1, 1)
    s, beta, delta = gp_ref.gpmodule_theta_to_kernel([0.3, ell], 1e-3)
    G = gp_ref.gram_ardse(x, beta, s, delta)
    L_ref = np.linalg.cholesky(G)
    ch = kernels.cholesky_inverse(kernels.gram(_t(x, dev), _t(beta, dev), s, delta))
    L, info, logdet = kernels.cholesky(kernels.gram(_t(x, dev), _t(beta, dev), s, delta))
    assert int(ch.info[0]) == 0 and int(info[0]) == 0
    for Lg in (ch.L[0].cpu().numpy(), L[0].cpu().numpy()):
        assert np.linalg.norm(Lg @ Lg.T - G) / np.linalg.norm(G) <= 1e-13
        kappa = np.linalg.cond(G)
        assert np.max(np.abs(Lg - L_ref)) <= 1e-16 * kappa * np.abs(L_ref).max() * 10
    np.testing.assert_allclose(float(ch.logdet[0]), 2 * np.sum(np.log(np.diag(L_ref))),
                               rtol=1e-10)
    Li = ch.Linv[0].cpu().numpy()
    assert np.max(np.abs(Li @ L_ref - np.eye(n))) <= 1e-16 * np.linalg.cond(G) * 100


@pytest.mark.parametrize("n,ld", [(1, 1), (7, 9), (128, 128), (1000, 1024)])
def test_pack_unpack_tril_round_trip(dev, n, ld):
    """gp_pack_tril / gp_unpack_tril (the round-4 single-GP broadcast payload, kept as a plain
    lower-triangle utility; the payload is now the tile-packed layout, test_gpu_sched.py):
    column c from row c on, column after column; unpacking writes the lower triangle only."""
    from gladsgp_amd import _capi
    rng = np.random.default_rng(n)
    A = rng.standard_normal((n, ld))                       # [col][row] = column-major, ld rows
    At = torch.as_tensor(A, device=dev).contiguous()
    v = torch.empty(n * (n + 1) // 2, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    _capi.call("gp_pack_tril", At.data_ptr(), n, ld, v.data_ptr(), st)
    ref = np.concatenate([A[c, c:n] for c in range(n)])
    assert np.array_equal(v.cpu().numpy(), ref)
    B = torch.full((n, ld), 7.0, dtype=torch.float64, device=dev)
    _capi.call("gp_unpack_tril", v.data_ptr(), n, B.data_ptr(), ld, st)
    Bh = B.cpu().numpy()
    for c in range(n):
        assert np.array_equal(Bh[c, c:n], A[c, c:n])
        assert np.all(Bh[c, :c] == 7.0) and np.all(Bh[c, n:] == 7.0)
