"""Column-major fp64 dense helpers over libgpfit (GEMM, statistics, eigensolver).

A column-major (rows x cols) matrix is a torch tensor ``t`` of shape (cols, ld) with element
(i, j) at ``t[j, i]`` — i.e. the row-major view of its transpose.  :class:`CM` carries the
logical shape and leading dimension so the GEMM call reads like BLAS.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _capi
from .kernels import F64, _stream


@dataclass
class CM:
    """Column-major view: logical ``rows x cols`` with leading dimension ``ld``."""

    t: torch.Tensor
    rows: int
    cols: int
    ld: int

    @property
    def f32(self) -> bool:
        """Stored as float32 (read by gp_gemm_ex and widened to fp64 on load)."""
        return self.t.dtype == torch.float32

    @staticmethod
    def empty(rows: int, cols: int, device) -> "CM":
        t = torch.empty((max(cols, 1), max(rows, 1)), dtype=F64, device=device)
        return CM(t, rows, cols, max(rows, 1))

    @staticmethod
    def of_rowmajor(a: torch.Tensor) -> "CM":
        """A C-order (r x c) tensor seen column-major is its transpose: (c x r), ld = c -- or,
        for a row-strided view (unit column stride, row stride >= c: the ensemble's padded
        y_std), ld = its row stride, without a copy."""
        if a.dim() == 2 and a.shape[0] > 1 and a.shape[1] > 0 and a.stride(1) == 1 and \
                a.stride(0) >= a.shape[1]:
            return CM(a, a.shape[1], a.shape[0], a.stride(0))
        a = a.contiguous()
        r, c = a.shape
        return CM(a, c, r, c)

    def rowmajor_T(self) -> torch.Tensor:
        """The logical matrix transposed, as a C-order torch tensor (cols x rows) view."""
        return self.t[: self.cols, : self.rows]

    def logical(self) -> torch.Tensor:
        return self.rowmajor_T().transpose(0, 1)

    def ptr(self) -> int:
        return self.t.data_ptr()


_WS: dict = {}


def _ws(nbytes: int, device) -> torch.Tensor | None:
    if nbytes <= 0:
        return None
    key = str(device)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _WS[key] = buf
    return buf


def gemm(transa: bool, transb: bool, A: CM, B: CM, alpha: float = 1.0, beta: float = 0.0,
         C: CM | None = None) -> CM:
    """C = alpha op(A) op(B) + beta C on MFMA (split-K for long inner dimensions).  A or B may
    be float32 (gp_gemm_ex widens them on load: the same fp64 result as on an fp64 copy); C is
    fp64."""
    m = A.cols if transa else A.rows
    k = A.rows if transa else A.cols
    kb = B.cols if transb else B.rows
    n = B.rows if transb else B.cols
    if k != kb:
        raise ValueError(f"gemm: inner dimensions differ ({k} vs {kb})")
    dev = A.t.device
    if C is None:
        C = CM.empty(m, n, dev)
        beta = 0.0
    lib = _capi.lib()
    nbytes = lib.gp_dgemm_ws_bytes(m, n, k)
    ws = _ws(nbytes, dev)
    for nm, M in (("A", A), ("B", B)):
        if M.t.dtype not in (torch.float32, F64):
            raise TypeError(f"gemm: {nm} must be float32 or float64, got {M.t.dtype}")
    if C.t.dtype != F64:
        raise TypeError("gemm: C must be float64")
    _capi.call("gp_gemm_ex", int(transa), int(transb), m, n, k, float(alpha), A.ptr(),
               int(A.f32), A.ld, B.ptr(), int(B.f32), B.ld, float(beta), C.ptr(), C.ld,
               ws.data_ptr() if ws is not None else None, nbytes if ws is not None else 0,
               _stream(dev))
    return C


def sim_stats(Y: torch.Tensor, sd_floor: float = 1e-6):
    """mu, sd(ddof=1, floored) over rows of a C-order (n x ny) ensemble (src/model.py:60-64)."""
    Y = Y.contiguous()
    n, ny = Y.shape
    mu = torch.empty(ny, dtype=F64, device=Y.device)
    sd = torch.empty(ny, dtype=F64, device=Y.device)
    _capi.call("gp_sim_stats", Y.data_ptr(), n, ny, ny, float(sd_floor), mu.data_ptr(),
               sd.data_ptr(), _stream(Y.device))
    return mu, sd


def standardize(Y: torch.Tensor, mu: torch.Tensor, sd: torch.Tensor, inverse: bool = False,
                out: torch.Tensor | None = None) -> torch.Tensor:
    """(Y - mu)/sd, or Y sd + mu when ``inverse`` (C-order rows x ny)."""
    Y = Y.contiguous()
    n, ny = Y.shape
    out = torch.empty_like(Y) if out is None else out
    _capi.call("gp_standardize", Y.data_ptr(), n, ny, ny, mu.data_ptr(), sd.data_ptr(),
               out.data_ptr(), out.stride(0), int(inverse), _stream(Y.device))
    return out


def field_max_pcs() -> int:
    return int(_capi.lib().gp_field_max_pcs())


def field(W: torch.Tensor, K: torch.Tensor, sd: torch.Tensor | None = None,
          mu: torch.Tensor | None = None, err: torch.Tensor | None = None, f32: bool = False,
          out: torch.Tensor | None = None) -> torch.Tensor:
    """Y = (W K + err) sd + mu in one pass (gp_field; SepiaEmulatorPrediction.get_y):
    W (rows x P) and K (P x ncols, row stride free) row-major fp64 on the device, sd / mu
    (ncols) or both None (standardised field), err (rows) or None; Y (rows x ncols) float32 when
    ``f32`` else float64."""
    rows, P = W.shape
    if K.shape[0] != P or K.stride(1) != 1 or W.stride(1) != 1:
        raise ValueError("field: W (rows x P) and K (P x ncols) must be row-major, K.shape[0] = P")
    ncols = K.shape[1]
    if out is None:
        out = torch.empty((rows, ncols), dtype=torch.float32 if f32 else F64, device=W.device)
    if (sd is None) != (mu is None):
        raise ValueError("field: sd and mu go together")
    for t in (sd, mu, err):
        if t is not None and (t.dtype != F64 or not t.is_contiguous()):
            raise ValueError("field: sd / mu / err must be contiguous float64")
    if err is not None and err.numel() != rows:
        raise ValueError(f"field: err has {err.numel()} values for {rows} rows")
    _capi.call("gp_field", W.data_ptr(), W.stride(0), rows, P, K.data_ptr(), K.stride(0), ncols,
               sd.data_ptr() if sd is not None else None,
               mu.data_ptr() if mu is not None else None,
               err.data_ptr() if err is not None else None, out.data_ptr(), out.stride(0),
               int(f32), _stream(W.device))
    return out


def mean_var(x: torch.Tensor, ddof: int = 0):
    """(mean, var) of all elements of ``x`` (device scalars tensor of 2)."""
    x = x.contiguous()
    out = torch.empty(2, dtype=F64, device=x.device)
    work = torch.empty(1024, dtype=F64, device=x.device)
    _capi.call("gp_mean_var", x.data_ptr(), x.numel(), int(ddof), out.data_ptr(),
               work.data_ptr(), _stream(x.device))
    return out


def shift_diag(G: CM, factor: float) -> None:
    _capi.call("gp_shift_diag", G.ptr(), G.rows, G.ld, float(factor), _stream(G.t.device))


def rowscale(M: CM, f: torch.Tensor, inverse: bool = False) -> None:
    _capi.call("gp_rowscale", M.ptr(), M.rows, M.cols, M.ld, f.data_ptr(), int(inverse),
               _stream(M.t.device))


def syevj(A: CM, max_sweeps: int = 30, tol: float = 1e-15, want_sqrt: bool = False):
    """Eigen-decomposition of a symmetric r x r matrix (destroyed): (W desc, V, sweeps)."""
    r = A.rows
    dev = A.t.device
    W = torch.empty(r, dtype=F64, device=dev)
    V = CM.empty(r, r, dev)
    sweeps = torch.zeros(1, dtype=torch.int32, device=dev)
    _capi.call("gp_syevj", A.ptr(), r, A.ld, W.data_ptr(), V.ptr(), V.ld, int(max_sweeps),
               float(tol), sweeps.data_ptr(), int(want_sqrt), _stream(dev))
    return W, V, sweeps
