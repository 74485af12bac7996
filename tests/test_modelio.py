"""CPU: the pickle-free model-state files (gladsgp_amd.modelio) that replace SEPIA's
save_model_info / restore_model_info pickle (src/model.py:149, 238)."""
import numpy as np
import pytest

from gladsgp_amd import modelio


def _sepia_like_samples(S=6, d=8, P=5, seed=0):
    rng = np.random.default_rng(seed)
    return {"betaU": rng.uniform(0.1, 3, (S, d + 1, P)),      # SEPIA's (S,) + val_shape
            "lamUz": rng.uniform(0.5, 3, (S, 1, P)),
            "lamWs": rng.uniform(100, 3000, (S, 1, P)),
            "lamWOs": rng.uniform(50, 500, (S, 1, 1)),
            "logPost": rng.standard_normal((S, 1))}


def test_round_trip_flattens_parameter_samples(tmp_path):
    smp = _sepia_like_samples()
    params = {"lamWOs": np.array([[123.0]])}
    steps = {"lamWOs": np.array([[10.0]])}
    f = modelio.save_model_npz(str(tmp_path / "synth_n016_p05"), smp, params, steps)
    assert f.endswith("synth_n016_p05.npz")
    got, gp, gs = modelio.load_model_npz(str(tmp_path / "synth_n016_p05"))
    assert got["betaU"].shape == (6, 9 * 5)
    # C order: betaU[s].reshape(d+1, P) is the SEPIA layout again (mcmc_diagnostics_advanced:57)
    np.testing.assert_array_equal(got["betaU"].reshape(6, 9, 5), smp["betaU"])
    assert got["lamUz"].shape == (6, 5) and got["lamWOs"].shape == (6, 1)
    np.testing.assert_array_equal(got["logPost"], smp["logPost"])
    assert float(gp["lamWOs"][0, 0]) == 123.0 and float(gs["lamWOs"][0, 0]) == 10.0


def test_missing_npz_next_to_sepia_pickle_names_the_export(tmp_path):
    (tmp_path / "m_n016_p05.pkl").write_bytes(b"not read")
    with pytest.raises(FileNotFoundError, match="export_sepia_samples"):
        modelio.load_model_npz(str(tmp_path / "m_n016_p05"))
    with pytest.raises(FileNotFoundError):
        modelio.load_model_npz(str(tmp_path / "absent"))


def test_export_tool_writes_the_layout(tmp_path):
    """tools/export_sepia_samples.export on a SEPIA-shaped model object (duck-typed)."""
    import importlib.util
    import os
    import types
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location(
        "export_tool", os.path.join(root, "tools", "export_sepia_samples.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    smp = _sepia_like_samples(S=3)
    par = {k: types.SimpleNamespace(val=smp[k][0], mcmcStepParam=np.ones_like(smp[k][0]))
           for k in ("betaU", "lamUz", "lamWs", "lamWOs")}
    model = types.SimpleNamespace(get_samples=lambda: smp, params=types.SimpleNamespace(**par))
    f = mod.export(model, str(tmp_path / "x"))
    got, gp, gs = modelio.load_model_npz(f)
    np.testing.assert_array_equal(got["lamWs"].reshape(3, 1, 5), smp["lamWs"])
    np.testing.assert_array_equal(gp["betaU"], smp["betaU"][0])
    np.testing.assert_array_equal(gs["lamUz"], np.ones((1, 5)))
