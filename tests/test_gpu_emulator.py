"""GPU parity of the drop-in surface (gladsgp_amd.model / .emulator) against the oracle's
restatement of src/model.py + the GPMSA predictive equations."""
import os
import types

import numpy as np
import pytest
import torch

from oracle import gp_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def _ensemble(n=96, ny=1500, d=8, seed=0):
    rng = np.random.default_rng(seed)
    t = rng.random((n, d))
    modes = rng.standard_normal((6, ny)) * (0.5 ** np.arange(6))[:, None]
    coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, d) + k) for k in range(6)], 1)
    y = 3.0 + coef @ modes + 1e-2 * rng.standard_normal((n, ny))
    y[:, :3] = 1.0   # constant nodes (sd floored, src/model.py:62-64)
    return t, y


def _samples(S, d, P, seed=1):
    rng = np.random.default_rng(seed)
    return {"betaU": rng.uniform(0.2, 3.0, (S, (d + 1) * P)),
            "lamUz": rng.uniform(0.5, 3.0, (S, P)),
            "lamWs": rng.uniform(200, 3000, (S, P)),
            "lamWOs": rng.uniform(50, 500, (S, 1))}


def _ref_prep(t, y, p, omega):
    mu, sd, ystd = gp_ref.standardize(y, 1e-6)
    U, S, Vh = gp_ref.randomized_svd(ystd, 25, k=0, q=1, omega=omega)
    K = gp_ref.pca_basis(S, Vh, p, y.shape[0]).astype(np.float32).astype(np.float64)
    return mu, sd, ystd, S, K


def test_init_model_matches_restatement(dev, tmp_path):
    from gladsgp_amd import model as gm
    t, y = _ensemble()
    p = 5
    np.random.seed(3)
    omega = np.random.normal(size=(y.shape[1], 25)).astype(np.float32)
    data, model = gm.init_model(t, y, "synth", p, data_dir=str(tmp_path), omega=omega,
                                device=dev, verbose=False)
    mu, sd, ystd, S, K = _ref_prep(t, y, p, omega)
    sdd = data.sim_data
    np.testing.assert_allclose(sdd.y_mean.cpu().numpy(), mu, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(sdd.y_sd.cpu().numpy(), sd, rtol=1e-12)
    np.testing.assert_allclose(sdd.y_std.cpu().numpy(), ystd, atol=1e-10)
    # cached PCA files with the reference's names, re-read on the next call
    for a in ("U", "S", "Vh"):
        assert os.path.exists(tmp_path / f"pca_synth_{a}.npy")
    S_saved = np.load(tmp_path / "pca_synth_S.npy")
    np.testing.assert_allclose(S_saved[:p], S[:p], rtol=1e-9)
    Kd = sdd.K.cpu().numpy()
    sgn = np.sign(np.sum(Kd * K, axis=1))
    np.testing.assert_allclose(Kd * sgn[:, None], K, rtol=1e-6, atol=1e-6 * np.abs(K).max())
    # PC weights and LamSim (SEPIA sim-only w, diag(K K^T)) for the GPU's own basis
    w_ref = gp_ref.pc_weights(ystd, Kd)
    np.testing.assert_allclose(model.w_hat.cpu().numpy(), w_ref, atol=1e-8)
    np.testing.assert_allclose(model.LamSim.cpu().numpy(), np.sum(Kd * Kd, axis=1), rtol=1e-12)
    prec = gm.pc_precision(data)
    np.testing.assert_allclose(prec, gp_ref.pc_precision(ystd, Kd), rtol=1e-9)
    # second call reuses the cache (recompute=False) and gives the same basis
    data2, _ = gm.init_model(t, y, "synth", p, data_dir=str(tmp_path), device=dev,
                             verbose=False)
    np.testing.assert_array_equal(data2.sim_data.K.cpu().numpy(), Kd)


def test_emulator_prediction_matches_restatement(dev, tmp_path):
    from gladsgp_amd import model as gm
    from gladsgp_amd.emulator import EmulatorPrediction, SepiaEmulatorPrediction
    assert SepiaEmulatorPrediction is EmulatorPrediction
    t, y = _ensemble(n=80, ny=900)
    p, S = 4, 3
    data, model = gm.init_model(t, y, "e", p, data_dir=str(tmp_path), device=dev,
                                verbose=False)
    samples = _samples(S, t.shape[1], p)
    t_pred = np.random.default_rng(7).random((37, t.shape[1]))
    pred = EmulatorPrediction(model=model, samples=samples, t_pred=t_pred)
    assert pred.w.shape == (S, 37, p) and pred.var.shape == (S, 37, p)
    w_hat = model.w_hat.cpu().numpy()
    lam = model.LamSim.cpu().numpy()
    mean_r, var_r = gp_ref.sepia_predict_w(t, t_pred, w_hat, samples, lam)
    np.testing.assert_allclose(pred.w, mean_r, atol=1e-9 * max(1, np.abs(mean_r).max()))
    np.testing.assert_allclose(pred.var, var_r, atol=1e-10)
    # field reconstruction y = (w K) sd + mu  (SEPIA get_y)
    Kd = data.sim_data.K.cpu().numpy()
    y_ref = gp_ref.reconstruct_y(pred.w, Kd, data.sim_data.y_mean.cpu().numpy(),
                                 data.sim_data.y_sd.cpu().numpy())
    np.testing.assert_allclose(pred.get_y(), y_ref, rtol=1e-10, atol=1e-10)
    # + the reference's error term: sd_y * N(0, 1/sqrt(lamWOs_s)) per (sample, point)
    # (assess_all_models.py:493-497) or per sample (time_predictions.py:84-87)
    sd_y = data.sim_data.y_sd.cpu().numpy()
    for per_point in (True, False):
        e = pred.error_draws(np.random.default_rng(11), per_point=per_point)
        ye = pred.get_y(add_error=True, rng=np.random.default_rng(11), per_point=per_point)
        e3 = e[:, :, None] if per_point else e[:, None, :]
        np.testing.assert_allclose(ye, y_ref + e3 * sd_y, rtol=1e-10, atol=1e-10)
    z = pred.error_draws(np.random.default_rng(0), per_point=True)
    assert z.shape == (S, 37)
    np.testing.assert_allclose(np.std(z * np.sqrt(pred.lamWOs)[:, None]), 1.0, atol=0.3)
    # predictive nugget flag
    pred0 = EmulatorPrediction(model=model, samples=samples, t_pred=t_pred, pred_nugget=False)
    _, var0 = gp_ref.sepia_predict_w(t, t_pred, w_hat, samples, lam, pred_nugget=False)
    np.testing.assert_allclose(pred0.var, var0, atol=1e-10)
    # small unit budget forces several groups: same answer
    predg = EmulatorPrediction(model=model, samples=samples, t_pred=t_pred,
                               budget_bytes=1 << 17)
    np.testing.assert_allclose(predg.w, pred.w, atol=0, rtol=0)


def test_model_io_and_loglik(dev, tmp_path):
    from gladsgp_amd import model as gm
    t, y = _ensemble(n=64, ny=700, seed=4)
    p = 3
    data, model = gm.init_model(t, y, "io", p, data_dir=str(tmp_path), device=dev,
                                verbose=False)
    samples = _samples(10, t.shape[1], p, seed=5)
    model.set_samples(samples)
    model.save_model_info(str(tmp_path / "io_model"))
    _, model2 = gm.init_model(t, y, "io", p, data_dir=str(tmp_path), device=dev,
                              verbose=False)
    model2.restore_model_info(str(tmp_path / "io_model"))
    got = model2.get_samples(numsamples=4, nburn=2)
    idx = np.arange(2, 10)[np.linspace(0, 7, 4).astype(int)]
    for k in samples:
        np.testing.assert_array_equal(got[k], samples[k][idx])
    # log-likelihood building block: sum over PCs of -NLL_j at the given parameters
    pr = {k: v[0] for k, v in samples.items()}
    ll = model.log_likelihood(pr)
    w_hat = model.w_hat.cpu().numpy()
    lam = model.LamSim.cpu().numpy()
    beta, s, delta, _ = gp_ref.sepia_gp_params({k: v[:1] for k, v in samples.items()}, lam,
                                               t.shape[1], p)
    ref = 0.0
    for j in range(p):
        G = gp_ref.gram_ardse(t, beta[0, j], s[0, j], delta[0, j])
        L = np.linalg.cholesky(G)
        z = np.linalg.solve(L, w_hat[:, j])
        ref -= 0.5 * z @ z + np.sum(np.log(np.diag(L)))
    np.testing.assert_allclose(ll, ref, rtol=1e-10)


def test_load_model_reference_layout(dev, tmp_path):
    """load_model reads X_standard CSV + Y_physical .npy (ny x n, transposed) like model.py."""
    from gladsgp_amd import model as gm
    t, y = _ensemble(n=48, ny=400, seed=9)
    d = t.shape[1]
    csv = tmp_path / "x.csv"
    np.savetxt(csv, t, delimiter=",", header=",".join(f"t{i}" for i in range(d)), fmt="%.6e")
    np.save(tmp_path / "y.npy", y.T)
    cfg = types.SimpleNamespace(X_standard=str(csv), Y_physical=str(tmp_path / "y.npy"),
                                data_dir=str(tmp_path), exp="cfg")
    os.makedirs(tmp_path / "models", exist_ok=True)
    data, model = gm.init_model(np.loadtxt(csv, delimiter=",", skiprows=1).astype(np.float32)[:40],
                                y.astype(np.float32)[:40], "cfg_n040", 2,
                                data_dir=str(tmp_path / "models"), device=dev, verbose=False)
    model.set_samples(_samples(4, d, 2))
    model.save_model_info(str(tmp_path / "models" / "cfg_n040_p02"))
    data2, model2 = gm.load_model(cfg, 40, 2, device=dev)
    assert model2.samples is not None and model2.P == 2 and model2.n == 40
    np.testing.assert_array_equal(data2.sim_data.K.cpu().numpy(), data.sim_data.K.cpu().numpy())


def test_c5_field_emulator(dev):
    """n = 512 runs of a 10k-node field (smooth seeded function of the design
    times fixed modes, + 1e-3 noise), a 64-PC basis from the GPU randomized_svd(Y_std, 64, k=0,
    q=1) (plot_PC_RMSE.py:91's call), 64 PC GPs predicted for two posterior samples through
    EmulatorPrediction; mean / variance checked against the oracle on the GPU's own basis."""
    from gladsgp_amd.emulator import EmulatorData, EmulatorModel, EmulatorPrediction
    from gladsgp_amd.svd import randomized_svd
    rng = np.random.default_rng(55)
    n, d, ny, P = 512, 8, 10000, 64
    t = rng.random((n, d))
    modes = rng.standard_normal((16, ny)) * (0.7 ** np.arange(16))[:, None]
    coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, d) + k) for k in range(16)], 1)
    y = coef @ modes + 1e-3 * rng.standard_normal((n, ny))
    data = EmulatorData(t, y, device=dev)
    data.standardize_y()
    np.random.seed(64)
    U, S, Vh = randomized_svd(data.sim_data.y_std, P, k=0, q=1)
    K = (S[:, None] * Vh / np.sqrt(n)).contiguous()
    data.create_K_basis(K)
    model = EmulatorModel(data)
    assert model.P == P and model.w_hat.shape == (n, P)
    samples = _samples(2, d, P, seed=56)
    t_pred = rng.random((300, d))
    pred = EmulatorPrediction(model=model, samples=samples, t_pred=t_pred)
    assert pred.w.shape == (2, 300, P)
    w_hat = model.w_hat.cpu().numpy()
    lam = model.LamSim.cpu().numpy()
    mean_r, var_r = gp_ref.sepia_predict_w(t, t_pred, w_hat, samples, lam)
    np.testing.assert_allclose(pred.w, mean_r, atol=1e-9 * max(1, np.abs(mean_r).max()))
    np.testing.assert_allclose(pred.var, var_r, atol=1e-10 * max(1, np.abs(var_r).max()))
    # the oracle's PC weights for this basis agree with the GPU's (pinv(K), model.py:219)
    ystd = data.sim_data.y_std.cpu().numpy()
    np.testing.assert_allclose(w_hat, gp_ref.pc_weights(ystd, K.cpu().numpy()), atol=1e-7)
