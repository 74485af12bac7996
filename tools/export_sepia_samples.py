#!/usr/bin/env python
"""Export a fitted SEPIA model's state to the pickle-free .npz gladsgp_amd reads.

Run ONCE in the environment that has SEPIA (and the reference's src/ on the path), on the
model files the reference's fit_models wrote (src/model.py:238):

    python tools/export_sepia_samples.py <train_config.py> <m> <p> [out_path]

It rebuilds the SEPIA model exactly as the reference's ``load_model`` does
(src/model.py:109-150, which restores the pickle with SEPIA's own restore_model_info), then
writes ``model.get_samples()`` plus the current values / step sizes to ``out_path + '.npz'``
(default: the model path) with gladsgp_amd.modelio.save_model_npz.  gladsgp_amd's
``load_model`` / ``restore_model_info`` then read that file; nothing is ever unpickled there.
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gladsgp_amd.modelio import save_model_npz  # noqa: E402


def export(model, out_path):
    samples = model.get_samples()
    params = {k: getattr(model.params, k).val for k in ("betaU", "lamUz", "lamWs", "lamWOs")}
    steps = {k: getattr(model.params, k).mcmcStepParam
             for k in ("betaU", "lamUz", "lamWs", "lamWOs")}
    return save_model_npz(out_path, samples, params, steps)


def main(argv):
    cfg_file, m, p = argv[1], int(argv[2]), int(argv[3])
    spec = importlib.util.spec_from_file_location("train_config", cfg_file)
    cfg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cfg)
    from src import model as ref_model        # the reference's src/model.py (needs SEPIA)
    _, model = ref_model.load_model(cfg, m, p)
    name = "{}_n{:03d}_p{:02d}".format(cfg.exp, m, p)
    out = argv[4] if len(argv) > 4 else os.path.join(cfg.data_dir, "models", name)
    print("wrote", export(model, out))


if __name__ == "__main__":
    main(sys.argv)
