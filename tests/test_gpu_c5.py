"""GPU parity of BASELINE config 5 and of the fused field reconstruction.

* gp_field (get_y's one-pass kernel: y = (w K + e) sd + mu, narrowed in the epilogue) equals
  the generic path -- gp_dgemm, the per-row error term, gp_standardize(inverse), a float32
  cast -- bit for bit, for 1-64 PCs, ragged row / column counts, a column block of K read
  through its row stride, with and without the error term and the back-transform, float32 and
  float64 outputs; and numpy's fp64 product within rounding;
* the bench's own C5 chain (gladsgp_amd.pipeline.FieldPipeline at full size: 512 x 10k
  float32 field, randomized_svd(Y_std, 64, k=0, q=1), 64 PC GPs at m = 100k, the 100k x 10k
  field on the device) against the oracle: singular values and the basis (up to each PC's
  sign) against gp_ref's own SVD with the same Omega; the PC GPs' mean / var and the field
  rows on the GPU's basis against gp_ref.sepia_predict_w + (w K) sd + mu on ~1,500 test
  points spread over every 8192-point chunk and the tail; two runs bit-identical.
"""
import numpy as np
import pytest
import torch

from oracle import gp_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch.device("cuda:0")


def _generic(w2, K, sd, mu, e, f32):
    """The pre-gp_field get_y arithmetic: gp_dgemm + error + gp_standardize(inverse) + cast."""
    from gladsgp_amd import blas
    from gladsgp_amd.blas import CM, gemm
    rows = w2.shape[0]
    Yc = gemm(False, False, CM.of_rowmajor(K.contiguous()), CM.of_rowmajor(w2))
    y = Yc.t[:rows, :K.shape[1]]
    if e is not None:
        y = y + e.reshape(rows, 1)
    if sd is not None:
        y = blas.standardize(y.contiguous(), mu, sd, inverse=True)
    return y.to(torch.float32) if f32 else y.contiguous()


@pytest.mark.parametrize("P", [1, 7, 25, 33, 64])
@pytest.mark.parametrize("rows,ncols", [(1, 1), (37, 300), (1000, 513), (4099, 1000)])
def test_field_kernel_equals_generic_path(dev, P, rows, ncols):
    from gladsgp_amd import blas
    rng = np.random.default_rng(P * 1000 + rows + ncols)
    w = torch.as_tensor(rng.standard_normal((rows, P)), device=dev)
    Kfull = torch.as_tensor(rng.standard_normal((P, ncols + 40)), device=dev)
    K = Kfull[:, 17:17 + ncols]                     # a column block: row stride ncols + 40
    sd = torch.as_tensor(rng.uniform(0.1, 3.0, ncols), device=dev)
    mu = torch.as_tensor(rng.standard_normal(ncols), device=dev)
    e = torch.as_tensor(rng.standard_normal(rows), device=dev)
    for f32 in (True, False):
        for use_e, use_sd in ((False, True), (True, True), (True, False), (False, False)):
            args = (sd if use_sd else None, mu if use_sd else None, e if use_e else None)
            got = blas.field(w, K, *args, f32=f32)
            ref = _generic(w, K, *args, f32)
            assert got.dtype == (torch.float32 if f32 else torch.float64)
            assert torch.equal(got, ref), (f32, use_e, use_sd)
    wn, Kn = w.cpu().numpy(), K.cpu().numpy()
    yn = (wn @ Kn + e.cpu().numpy()[:, None]) * sd.cpu().numpy() + mu.cpu().numpy()
    got = blas.field(w, K, sd, mu, e).cpu().numpy()
    np.testing.assert_allclose(got, yn, rtol=1e-12, atol=1e-12 * np.abs(yn).max())


@pytest.mark.parametrize("off", [0, 1, 2, 3])
def test_field_f32_output_views_any_alignment(dev, off):
    """float32 output into a column block of a wider buffer: 16-B row pieces where the rows are
    16-B aligned (off = 0), 4-B stores otherwise; the same bits either way, nothing written
    outside the block."""
    from gladsgp_amd import blas
    rng = np.random.default_rng(40 + off)
    rows, P, ncols = 333, 64, 700
    w = torch.as_tensor(rng.standard_normal((rows, P)), device=dev)
    K = torch.as_tensor(rng.standard_normal((P, ncols)), device=dev)
    sd = torch.as_tensor(rng.uniform(0.1, 3.0, ncols), device=dev)
    mu = torch.as_tensor(rng.standard_normal(ncols), device=dev)
    ref = blas.field(w, K, sd, mu, f32=True)
    big = torch.full((rows, ncols + 8), 7.0, dtype=torch.float32, device=dev)
    view = big[:, off:off + ncols]
    blas.field(w, K, sd, mu, f32=True, out=view)
    assert torch.equal(view, ref)
    assert bool((big[:, :off] == 7.0).all()) and bool((big[:, off + ncols:] == 7.0).all())


def test_get_y_beyond_field_pcs_uses_generic_path(dev):
    """P above gp_field_max_pcs() (64) reconstructs through gp_dgemm + gp_standardize: the
    kernel refuses it (-4) and get_y stays correct."""
    from gladsgp_amd import _capi, blas
    assert blas.field_max_pcs() == 64
    w = torch.zeros((4, 65), dtype=torch.float64, device=dev)
    K = torch.zeros((65, 10), dtype=torch.float64, device=dev)
    with pytest.raises(_capi.GPFitError):
        blas.field(w, K)


N, D, NY, M, P = 512, 8, 10_000, 100_000, 64


def _sample_points():
    idx = np.concatenate([np.arange(300), np.arange(300, M - 200, 97), np.arange(M - 200, M)])
    return np.unique(idx)


@pytest.fixture(scope="module")
def c5(dev):
    from gladsgp_amd.pipeline import FieldPipeline, synthetic_c5
    t, Y, omega, smp, t_pred = synthetic_c5(N, D, NY, M, P)
    pipe = FieldPipeline(t, Y, omega, smp, t_pred, P, device=dev)
    res = pipe.run()
    torch.cuda.synchronize()
    yield dict(t=t, Y=Y, omega=omega, smp=smp, t_pred=t_pred, pipe=pipe, res=res)
    pipe.close()


def test_c5_svd_and_basis_vs_oracle(c5):
    res = c5["res"]
    mu, sd, ys = gp_ref.standardize(c5["Y"])
    _, S_o, Vh_o = gp_ref.randomized_svd(ys, P, k=0, q=1, omega=c5["omega"])
    S_g = res["S"].cpu().numpy()
    np.testing.assert_allclose(S_g, S_o, rtol=1e-9)
    K_o = gp_ref.pca_basis(S_o, Vh_o, P, N).astype(np.float32).astype(np.float64)
    K_g = res["K"].cpu().numpy()
    sgn = np.sign(np.sum(K_g * K_o, axis=1))
    # K is stored float32-rounded (create_K_basis(K.astype(float32))): one float32 ulp apart
    np.testing.assert_allclose(K_g * sgn[:, None], K_o, rtol=0, atol=2e-7 * np.abs(K_o).max())
    assert res["y"].shape == (1, M, NY) and res["y"].dtype == torch.float32


def test_c5_predictions_and_field_vs_oracle(c5):
    res = c5["res"]
    idx = _sample_points()
    K_g = res["K"].cpu().numpy()
    mu, sd, ys = gp_ref.standardize(c5["Y"])
    w_hat = gp_ref.pc_weights(ys, K_g)
    np.testing.assert_allclose(res["w_hat"].cpu().numpy(), w_hat, atol=1e-9 * np.abs(w_hat).max())
    lam = np.sum(K_g * K_g, axis=1)
    mean_o, var_o = gp_ref.sepia_predict_w(c5["t"], c5["t_pred"][idx], w_hat, c5["smp"], lam)
    mean_g = res["mean"][:, idx].cpu().numpy()
    var_g = res["var"][:, idx].cpu().numpy()
    s_max = float(np.max(1.0 / c5["smp"]["lamUz"] + 1.0 / c5["smp"]["lamWs"]))
    np.testing.assert_allclose(mean_g, mean_o, rtol=0, atol=1e-8 * np.abs(mean_o).max())
    np.testing.assert_allclose(var_g, var_o, rtol=0, atol=1e-9 * s_max)
    assert np.all(var_g >= 0) and np.all(var_g <= s_max)
    w32 = mean_g.astype(np.float32).astype(np.float64)           # preds.w.astype(float32)
    y_o = np.einsum("smp,py->smy", w32, K_g) * sd + mu
    y_g = res["y"][:, idx].cpu().numpy().astype(np.float64)
    # float32 storage: within 1 float32 ulp of the fp64 oracle value (plus fp64 rounding)
    tol = np.spacing(np.abs(y_o).astype(np.float32)).astype(np.float64) + 1e-12 * np.abs(y_o).max()
    assert np.all(np.abs(y_g - y_o) <= tol)


def test_c5_run_is_deterministic(c5):
    res2 = c5["pipe"].run()
    torch.cuda.synchronize()
    res = c5["res"]
    for k in ("S", "K", "mean", "var"):
        assert torch.equal(res[k], res2[k]), k
    idx = torch.as_tensor(_sample_points(), device=res["y"].device)
    assert torch.equal(res["y"][:, idx], res2["y"][:, idx])
