"""Pickle-free model-state files (model I/O compatibility).

The reference saves fitted SEPIA models with ``model.save_model_info(path)`` and reloads them
with ``model.restore_model_info(path)`` (``src/model.py:149, 238``): a pickle.  This build never
unpickles, so model state travels as ``path + '.npz'`` holding plain arrays:
  * ``samples_<name>``: the MCMC samples dict as ``model.get_samples()`` returns it —
    ``betaU`` ``(S, (d+1) P)`` (or SEPIA's ``(S,) + val_shape``), ``lamUz`` / ``lamWs``
    ``(S, P)``, ``lamWOs`` ``(S, 1)`` (``mcmc_diagnostics_simple.py:31-37``), ``logPost``;
  * ``param_<name>`` / ``step_<name>``: current values and Metropolis step sizes.
A SEPIA fit is migrated once, in the SEPIA environment, by ``tools/export_sepia_samples.py``
(which calls :func:`save_model_npz` on ``model.get_samples()``).  Pure numpy: no device needed.
"""
from __future__ import annotations

import os

import numpy as np

PARAM_NAMES = ("betaU", "lamUz", "lamWs", "lamWOs")


def npz_path(path: str) -> str:
    return path if path.endswith(".npz") else path + ".npz"


def save_model_npz(path: str, samples: dict | None, params: dict | None = None,
                   steps: dict | None = None) -> str:
    """Write samples / values / step sizes as plain arrays to ``path + '.npz'``."""
    arrs = {f"samples_{k}": np.asarray(v) for k, v in (samples or {}).items()}
    arrs.update({f"param_{k}": np.asarray(v) for k, v in (params or {}).items()})
    arrs.update({f"step_{k}": np.asarray(v) for k, v in (steps or {}).items()})
    f = npz_path(path)
    np.savez(f, **arrs)
    return f


def load_model_npz(path: str):
    """(samples, params, steps) from ``path + '.npz'`` (allow_pickle=False).  Samples of the
    four parameters come back as (S, prod(val_shape)) float64 in C order; a missing .npz next
    to a SEPIA pickle raises an error that names the export step."""
    f = npz_path(path)
    base = path[:-4] if path.endswith(".npz") else path
    if not os.path.exists(f) and any(os.path.exists(base + ext) for ext in (".pkl", "")):
        raise FileNotFoundError(
            f"{f} not found, but a SEPIA model file exists at {base}[.pkl]: SEPIA's pickled "
            "model info is deliberately not read (no unpickling).  Export its samples once in "
            "the SEPIA environment with tools/export_sepia_samples.py (writes samples_<name> "
            "arrays to <path>.npz), then restore from that.")
    samples, params, steps = {}, {}, {}
    with np.load(f, allow_pickle=False) as z:
        for k in z.files:
            if k.startswith("samples_"):
                v = np.asarray(z[k], dtype=np.float64)
                name = k[8:]
                if name in PARAM_NAMES and v.ndim >= 1:
                    v = v.reshape(v.shape[0], -1)
                samples[name] = v
            elif k.startswith("param_"):
                params[k[6:]] = np.asarray(z[k])
            elif k.startswith("step_"):
                steps[k[5:]] = np.asarray(z[k])
    return samples, params, steps
