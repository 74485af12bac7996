"""ctypes binding of libgpfit.so (the C ABI declared in include/gpfit.h).

This is the whole host/device boundary: every product computation goes through one of these
symbols.  There is no CPU fallback — if the library is missing or cannot be loaded, every
entry point raises :class:`GPFitUnavailable`.

``torch`` is imported before the library is loaded on purpose: torch's bundled HIP runtime
(soname ``libamdhip64.so.7``) is then the one libgpfit binds to, so torch tensors, streams and
our kernels share one runtime and one device context.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

from ._build import LIB_PATH

c_int, c_ll, c_void_p, c_double_p = ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p, ctypes.c_void_p

GPFIT_ERR_HIP = -1000
GPFIT_ERR_INTERNAL = -2000
GPFIT_ERR_RCCL = -3000

# name -> (restype, argtypes); pointers are passed as integers (tensor.data_ptr()).
SIGNATURES = {
    "gp_version": (c_int, []),
    "gp_padded_n": (c_int, [c_int]),
    "gp_gram_ardse": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p,
                              c_void_p, c_void_p, c_int, c_ll, c_int, c_void_p]),
    "gp_cross_ardse": (c_int, [c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int,
                               c_void_p, c_int, c_void_p, c_void_p, c_int, c_ll, c_int,
                               c_void_p]),
    "gp_potrf_inv": (c_int, [c_void_p, c_int, c_int, c_ll, c_void_p, c_int, c_ll, c_int,
                             c_void_p, c_void_p, c_void_p]),
    "gp_potrf": (c_int, [c_void_p, c_int, c_int, c_ll, c_int, c_void_p, c_void_p, c_void_p]),
    "gp_potrf_inv_ws_bytes": (c_ll, [c_int, c_int]),
    "gp_potrf_inv_ws": (c_int, [c_void_p, c_int, c_int, c_ll, c_void_p, c_int, c_ll, c_int,
                                c_void_p, c_void_p, c_void_p, c_ll, c_void_p]),
    "gp_potrf_ws_bytes": (c_ll, [c_int, c_int]),
    "gp_potrf_ws": (c_int, [c_void_p, c_int, c_int, c_ll, c_int, c_void_p, c_void_p, c_void_p,
                            c_ll, c_void_p]),
    "gp_trtri": (c_int, [c_void_p, c_int, c_int, c_ll, c_void_p, c_int, c_ll, c_int, c_void_p,
                         c_void_p]),
    "gp_predict_ws_bytes": (c_ll, [c_int, c_int, c_int, c_int]),
    "gp_predict_chol_ws_bytes": (c_ll, [c_int, c_int, c_int, c_int]),
    "gp_predict_chol": (c_int, [c_void_p, c_int, c_ll, c_void_p, c_int, c_void_p, c_int, c_int,
                                c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                c_int, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                c_ll, c_int, c_void_p]),
    "gp_predict": (c_int, [c_void_p, c_int, c_ll, c_void_p, c_int, c_void_p, c_int, c_int,
                           c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                           c_void_p, c_void_p, c_int, c_int, c_void_p, c_ll, c_int, c_void_p]),
    "gp_predict_ex": (c_int, [c_void_p, c_int, c_ll, c_void_p, c_int, c_void_p, c_int, c_int,
                              c_int, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                              c_void_p, c_void_p, c_int, c_int, c_void_p, c_ll, c_int, c_int,
                              c_void_p, c_ll, c_void_p]),
    "gp_predict_z_ws_bytes": (c_ll, [c_int, c_int]),
    "gp_predict_z": (c_int, [c_void_p, c_int, c_ll, c_int, c_int, c_void_p, c_int, c_void_p, c_ll,
                             c_int, c_void_p, c_ll, c_void_p]),
    "gp_linv_packed_elems": (c_ll, [c_int]),
    "gp_pack_linv": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "gp_unpack_linv": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "gp_predict_prepared_ws_bytes": (c_ll, [c_int, c_int, c_int, c_int]),
    "gp_predict_cross": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                 c_int, c_void_p, c_int, c_void_p, c_ll, c_int, c_void_p]),
    "gp_predict_solve": (c_int, [c_void_p, c_int, c_ll, c_int, c_int, c_void_p, c_void_p, c_int,
                                 c_void_p, c_void_p, c_int, c_int, c_void_p, c_ll, c_int,
                                 c_void_p]),
    "gp_trmv": (c_int, [c_void_p, c_int, c_ll, c_int, c_void_p, c_int, c_void_p, c_int, c_int,
                        c_void_p]),
    "gp_nll": (c_int, [c_void_p, c_int, c_ll, c_int, c_void_p, c_int, c_void_p, c_void_p,
                       c_void_p, c_int, c_void_p]),
    "gp_fit_predict_ws_bytes": (c_ll, [c_int, c_int, c_int, c_int]),
    "gp_fit_predict": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                               c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                               c_int, c_ll, c_void_p, c_int, c_ll, c_void_p, c_void_p,
                               c_void_p, c_void_p, c_int, c_int, c_void_p, c_ll, c_int,
                               c_void_p, c_void_p]),
    "gp_ctx_create": (c_int, [ctypes.c_double, c_int, c_void_p]),
    "gp_ctx_destroy": (c_int, [c_void_p]),
    "gp_ctx_set_aux_chunks": (c_int, [c_void_p, c_int]),
    "gp_host_legacy_normal_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_ll,
                                          c_void_p, c_int]),
    "gp_loglik_ws_bytes": (c_ll, [c_int, c_int]),
    "gp_loglik": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_void_p,
                          c_void_p, c_int, c_int, c_void_p, c_ll, c_void_p, c_void_p,
                          c_void_p]),
    "gp_loglik_status": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "gp_mcmc_group_prep": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                   c_void_p, c_void_p]),
    "gp_mcmc_group_decide": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "gp_mcmc_group_step": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p,
                                   c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                   c_void_p]),
    "gp_realize": (c_int, [c_void_p, c_void_p, c_ll, ctypes.c_ulonglong, ctypes.c_ulonglong,
                           c_void_p, c_void_p]),
    "gp_dgemm_ws_bytes": (c_ll, [c_int, c_int, c_int]),
    "gp_dgemm": (c_int, [c_int, c_int, c_int, c_int, c_int, ctypes.c_double, c_void_p, c_int,
                         c_void_p, c_int, ctypes.c_double, c_void_p, c_int, c_void_p, c_ll,
                         c_void_p]),
    "gp_gemm_ex": (c_int, [c_int, c_int, c_int, c_int, c_int, ctypes.c_double, c_void_p, c_int,
                           c_int, c_void_p, c_int, c_int, ctypes.c_double, c_void_p, c_int,
                           c_void_p, c_ll, c_void_p]),
    "gp_sim_stats": (c_int, [c_void_p, c_int, c_int, c_ll, ctypes.c_double, c_void_p, c_void_p,
                             c_void_p]),
    "gp_standardize": (c_int, [c_void_p, c_int, c_int, c_ll, c_void_p, c_void_p, c_void_p, c_ll,
                               c_int, c_void_p]),
    "gp_mean_var": (c_int, [c_void_p, c_ll, c_int, c_void_p, c_void_p, c_void_p]),
    "gp_field_max_pcs": (c_int, []),
    "gp_field": (c_int, [c_void_p, c_ll, c_int, c_int, c_void_p, c_ll, c_int, c_void_p,
                         c_void_p, c_void_p, c_void_p, c_ll, c_int, c_void_p]),
    "gp_shift_diag": (c_int, [c_void_p, c_int, c_int, ctypes.c_double, c_void_p]),
    "gp_rowscale": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "gp_syevj": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int,
                         ctypes.c_double, c_void_p, c_int, c_void_p]),
    "gp_comm_available": (c_int, []),
    "gp_comm_unique_id": (c_int, [c_void_p]),
    "gp_comm_init": (c_int, [c_int, c_int, c_void_p, c_void_p]),
    "gp_comm_destroy": (c_int, [c_void_p]),
    "gp_bcast": (c_int, [c_void_p, c_void_p, c_ll, c_int, c_void_p]),
    "gp_pack_tril": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "gp_unpack_tril": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p]),
    "gp_gather": (c_int, [c_void_p, c_void_p, c_ll, c_void_p, c_int, c_void_p]),
    "gp_profile_enable": (c_int, [c_int]),
    "gp_profile_select": (ctypes.c_uint, [ctypes.c_uint]),
    "gp_profile_reset": (c_int, []),
    "gp_profile_read": (c_int, [c_int, c_void_p, c_void_p, c_void_p]),
    "gp_set_poll_budget": (c_ll, [c_ll]),
    "gp_set_potrf_path": (c_int, [c_int]),
    "gp_set_predict_path": (c_int, [c_int]),
}

PROF_GRAM, PROF_POTRF, PROF_TRMM, PROF_CROSS = 0, 1, 2, 3
LINV_PADDED, LINV_PACKED = 0, 1        # GPFIT_LINV_PADDED / GPFIT_LINV_PACKED


class GPFitUnavailable(RuntimeError):
    """libgpfit.so is not built or cannot be loaded (no fallback path exists)."""


class GPFitError(RuntimeError):
    """A libgpfit entry point returned a non-zero status."""

    def __init__(self, func: str, rc: int):
        if rc <= GPFIT_ERR_RCCL:
            msg = f"{func}: RCCL error {GPFIT_ERR_RCCL - rc} (or librccl not loadable)"
        elif rc == GPFIT_ERR_INTERNAL:
            msg = (f"{func}: internal error: a factorisation gave up (info = -1, a bounded wait "
                   "of the persistent kernel ran out) -- results since the last check are invalid")
        elif rc <= GPFIT_ERR_HIP:
            msg = f"{func}: HIP error {GPFIT_ERR_HIP - rc}"
        else:
            msg = f"{func}: invalid argument #{-rc}"
        super().__init__(msg)
        self.func = func
        self.rc = rc


_LIB = None


def lib() -> ctypes.CDLL:
    """Load (once) and return the configured library handle."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise GPFitUnavailable(
            f"{LIB_PATH} is missing: build it with `python -m gladsgp_amd._build` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    try:
        handle = ctypes.CDLL(LIB_PATH)
    except OSError as exc:  # pragma: no cover - environment specific
        raise GPFitUnavailable(f"cannot load {LIB_PATH}: {exc}") from exc
    for name, (res, args) in SIGNATURES.items():
        # a symbol an older build lacks (same-box A/B of library builds, tools/ab_*.sh) stays
        # unbound and fails where it is called; tests/test_capi.py checks the shipped build
        # exports every one
        fn = getattr(handle, name, None)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    # GPFIT_TRMM_RES (A/B runs, bench.py / tools/ab_res*.sh): 0 = cross-covariance chunks + the
    # pair TRMM everywhere, 2 = the column-resident kernel from materialised chunks
    mode = os.environ.get("GPFIT_TRMM_RES", "1")
    if mode in ("0", "2") and getattr(handle, "gp_set_predict_path", None) is not None:
        handle.gp_set_predict_path(1 if mode == "0" else 2)
    _LIB = handle
    return handle


def call(name: str, *args) -> int:
    """Invoke entry point ``name``; raise :class:`GPFitError` on a non-zero return."""
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise GPFitError(name, rc)
    return rc


def exported_symbols() -> list[str]:
    return list(SIGNATURES)


MCMC_MAX_GROUP = 4            # GPFIT_MCMC_MAX_GROUP
MCMC_DIST = {"Gamma": 0, "Beta": 1, "Normal": 2, "Uniform": 3}
MCMC_STEP = {"Uniform": 0, "BetaRho": 1}


class McmcState(ctypes.Structure):
    """gp_mcmc_state (include/gpfit.h): the sampler's device buffers and priors."""
    _fields_ = [(nm, c_void_p) for nm in (
        "betaU", "lamUz", "lamWs", "lamWOs", "ll", "lam", "u", "step_betaU", "step_lamUz",
        "step_lamWs", "step_lamWOs", "acc", "lp", "scratch")] + [
        ("P", c_int), ("d", c_int), ("dist", c_int * 4), ("steptype", c_int * 4),
        ("pa", ctypes.c_double * 4), ("pb", ctypes.c_double * 4), ("lo", ctypes.c_double * 4),
        ("hi", ctypes.c_double * 4)]
