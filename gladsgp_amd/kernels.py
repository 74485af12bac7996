"""Tensor-level entry points over libgpfit (device memory and streams from PyTorch-ROCm).

PyTorch is plumbing here: it owns the device buffers and the current HIP stream; every
arithmetic step runs in the HIP kernels behind :mod:`gladsgp_amd._capi`.

Layout convention: libgpfit is column-major (LAPACK).  A column-major n x n matrix M is held in
a torch tensor ``buf`` of shape (batch, n_cols, ld) with ``buf[b, j, i] = M[i, j]``; the
logical matrix is ``buf.transpose(-1, -2)``.  Symmetric matrices (the Gram) look the same
either way.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _capi

F64 = torch.float64


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _check_device(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a HIP device tensor (got {t.device}); "
                         "libgpfit has no CPU path")


def _as_f64(x, device, name) -> torch.Tensor:
    t = torch.as_tensor(x, dtype=F64, device=device)
    _check_device(t, name)
    return t.contiguous()


def _per_batch(x, batch: int, device, name) -> torch.Tensor:
    t = _as_f64(x, device, name).reshape(-1)
    if t.numel() == 1 and batch > 1:
        t = t.expand(batch).contiguous()
    if t.numel() != batch:
        raise ValueError(f"{name}: expected {batch} values, got {t.numel()}")
    return t


def _beta(beta, batch: int, d: int, device) -> torch.Tensor:
    t = _as_f64(beta, device, "beta")
    if t.dim() == 1:
        t = t.reshape(1, -1)
    if t.shape[0] == 1 and batch > 1:
        t = t.expand(batch, t.shape[1]).contiguous()
    if tuple(t.shape) != (batch, d):
        raise ValueError(f"beta: expected shape ({batch}, {d}), got {tuple(t.shape)}")
    return t


def padded_n(n: int) -> int:
    return _capi.lib().gp_padded_n(int(n))


def gram(X: torch.Tensor, beta, s, delta, batch: int | None = None) -> torch.Tensor:
    """G[b] = s[b] exp(-sum_k beta[b,k] (x_i - x_j)_k^2) + delta[b] I   -> (batch, n, n)."""
    X = _as_f64(X, None if not torch.is_tensor(X) else X.device, "X")
    n, d = X.shape
    bt = torch.as_tensor(beta)
    batch = batch or (bt.shape[0] if bt.dim() == 2 else 1)
    dev = X.device
    beta_t = _beta(beta, batch, d, dev)
    s_t = _per_batch(s, batch, dev, "s")
    d_t = _per_batch(delta, batch, dev, "delta")
    G = torch.empty((batch, n, n), dtype=F64, device=dev)
    _capi.call("gp_gram_ardse", X.data_ptr(), n, d, d, beta_t.data_ptr(), d, s_t.data_ptr(),
               d_t.data_ptr(), G.data_ptr(), n, n * n, batch, _stream(dev))
    return G


def cross(X: torch.Tensor, Xs: torch.Tensor, beta, s, batch: int | None = None) -> torch.Tensor:
    """K*^T[b] (n x m) held column-major: returns tensor (batch, m, n), [b, j, i] = K*[j, i]."""
    X = _as_f64(X, X.device, "X")
    Xs = _as_f64(Xs, X.device, "Xs")
    n, d = X.shape
    m = Xs.shape[0]
    bt = torch.as_tensor(beta)
    batch = batch or (bt.shape[0] if bt.dim() == 2 else 1)
    beta_t = _beta(beta, batch, d, X.device)
    s_t = _per_batch(s, batch, X.device, "s")
    Kt = torch.empty((batch, m, n), dtype=F64, device=X.device)
    _capi.call("gp_cross_ardse", X.data_ptr(), n, d, Xs.data_ptr(), m, d, d, beta_t.data_ptr(),
               d, s_t.data_ptr(), Kt.data_ptr(), n, m * n, batch, _stream(X.device))
    return Kt


@dataclass
class Cholesky:
    """Result of :func:`cholesky_inverse` (buffers are column-major, see module doc)."""

    n: int
    a_buf: torch.Tensor      # (batch, n, n): lower triangle holds L (col-major)
    linv_buf: torch.Tensor   # (batch, npad, npad): L^-1 (col-major, zero-padded)
    info: torch.Tensor       # (batch,) int32, LAPACK potrf info
    logdet: torch.Tensor     # (batch,) float64, log|A|

    @property
    def L(self) -> torch.Tensor:
        return torch.tril(self.a_buf.transpose(-1, -2))

    @property
    def Linv(self) -> torch.Tensor:
        return self.linv_buf.transpose(-1, -2)[:, : self.n, : self.n]

    def check(self) -> None:
        check_info(self.info)


class FactorizationInternalError(RuntimeError):
    """info = -1: the persistent factorisation gave up on a bounded wait (an internal error of
    the library, never a property of the matrix)."""


def check_info(info: torch.Tensor) -> None:
    """Raise for any problem whose factorisation did not succeed: info = -1 is an internal
    error (:class:`FactorizationInternalError`), info = j > 0 the LAPACK non-positive-definite
    pivot (ValueError).  Synchronises with the device."""
    vals = info.cpu()
    bad = torch.nonzero(vals).flatten().tolist()
    if not bad:
        return
    internal = [b for b in bad if int(vals[b]) < 0]
    if internal:
        raise FactorizationInternalError(
            f"internal factorisation error (info = -1: a bounded wait of the persistent kernel "
            f"gave up) for problems {internal}; results are invalid")
    raise ValueError(f"matrix not positive definite (info={vals[bad].tolist()} for "
                     f"problems {bad})")


class Workspace:
    """Reusable device scratch (grown on demand, never shrunk; 256-B aligned torch storage)."""

    def __init__(self):
        self.buf = None

    def get(self, nbytes: int, device) -> torch.Tensor:
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != device:
            self.buf = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
        return self.buf


_POTRF_WS = {}


def _potrf_ws(device, nbytes: int) -> torch.Tensor:
    w = _POTRF_WS.setdefault(str(device), Workspace())
    return w.get(nbytes, device)


def cholesky_inverse(G: torch.Tensor, overwrite: bool = True,
                     workspace: Workspace | None = None) -> Cholesky:
    """Blocked MFMA Cholesky A = L L^T with L^-1, logdet and LAPACK info per problem
    (gp_potrf_inv_ws: the factorisation's scratch comes from ``workspace``, by default a
    per-device one reused across calls on the current stream)."""
    _check_device(G, "G")
    if G.dtype != F64:
        raise TypeError("G must be float64")
    if G.dim() == 2:
        G = G.unsqueeze(0)
    batch, n, n2 = G.shape
    if n != n2:
        raise ValueError("G must be square")
    A = G if (overwrite and G.is_contiguous()) else G.contiguous().clone()
    npad = padded_n(n)
    Linv = torch.empty((batch, npad, npad), dtype=F64, device=G.device)
    info = torch.empty(batch, dtype=torch.int32, device=G.device)
    logdet = torch.empty(batch, dtype=F64, device=G.device)
    nbytes = int(_capi.lib().gp_potrf_inv_ws_bytes(n, batch))
    ws = (workspace.get(nbytes, G.device) if workspace is not None
          else _potrf_ws(G.device, nbytes))
    _capi.call("gp_potrf_inv_ws", A.data_ptr(), n, n, n * n, Linv.data_ptr(), npad, npad * npad,
               batch, info.data_ptr(), logdet.data_ptr(), ws.data_ptr(), ws.numel(),
               _stream(G.device))
    return Cholesky(n, A, Linv, info, logdet)


PredictWorkspace = Workspace   # scratch of predict / fit_predict / predict_prepare


_DEFAULT_WS = PredictWorkspace()


@dataclass
class PackedLinv:
    """L^-1 in the tile-packed layout (gp_pack_linv: column c of the padded buffer from row
    16 floor(c/16) on, about half the padded square) -- the single-GP broadcast's payload, which
    :func:`predict` reads in place -- with, optionally, z = L^-1 w (gp_predict_z)."""

    n: int
    buf: torch.Tensor                 # (batch, gp_linv_packed_elems(n)) float64
    info: torch.Tensor                # (batch,) int32
    z: torch.Tensor | None = None     # (batch, padded_n(n)) float64

    def check(self) -> None:
        check_info(self.info)


def linv_packed_elems(n: int) -> int:
    return int(_capi.lib().gp_linv_packed_elems(int(n)))


def pack_linv(chol: Cholesky, out: torch.Tensor | None = None) -> torch.Tensor:
    """The tile-packed L^-1 of every problem: (batch, gp_linv_packed_elems(n)) (gp_pack_linv)."""
    batch, npad = chol.linv_buf.shape[0], chol.linv_buf.shape[1]
    E = linv_packed_elems(chol.n)
    if out is None:
        out = torch.empty((batch, E), dtype=F64, device=chol.linv_buf.device)
    for b in range(batch):
        _capi.call("gp_pack_linv", chol.linv_buf[b].data_ptr(), chol.n, npad,
                   out[b].data_ptr(), _stream(out.device))
    return out


_Z_WS = {}


def predict_z(chol, w, out: torch.Tensor | None = None) -> torch.Tensor:
    """z = L^-1 w per problem, (batch, padded_n(n)), zero past n, with exactly the arithmetic
    :func:`predict` applies internally (gp_predict_z); ``chol`` a Cholesky or a PackedLinv."""
    packed = isinstance(chol, PackedLinv)
    L = chol.buf if packed else chol.linv_buf
    dev, batch, n = L.device, L.shape[0], chol.n
    npad = padded_n(n)
    w_t = _as_f64(w, dev, "w").reshape(batch, n)
    if out is None:
        out = torch.empty((batch, npad), dtype=F64, device=dev)
    nbytes = int(_capi.lib().gp_predict_z_ws_bytes(n, batch))
    ws = _Z_WS.setdefault(str(dev), Workspace()).get(nbytes, dev)
    _capi.call("gp_predict_z", L.data_ptr(), npad, L.stride(0),
               _capi.LINV_PACKED if packed else _capi.LINV_PADDED, n, w_t.data_ptr(), n,
               out.data_ptr(), out.stride(0) if batch > 1 else npad, batch, ws.data_ptr(),
               ws.numel(), _stream(dev))
    return out


def predict(chol, X: torch.Tensor, Xs: torch.Tensor, beta, s, s_pred, w,
            m_chunk: int = 0, workspace: PredictWorkspace | None = None,
            out: tuple[torch.Tensor, torch.Tensor] | None = None,
            z: torch.Tensor | None = None):
    """Posterior mean / marginal variance at Xs for every problem: returns (batch, m) x 2.

    ``chol`` is a :class:`Cholesky` (padded L^-1) or a :class:`PackedLinv` (read in place);
    ``z`` (or the PackedLinv's own) is L^-1 w from :func:`predict_z`, which then skips the
    library's own (``w`` is not read).  Every form gives bit-identical results (gp_predict_ex).
    """
    packed = isinstance(chol, PackedLinv)
    L = chol.buf if packed else chol.linv_buf
    if z is None and packed:
        z = chol.z
    dev = L.device
    X = _as_f64(X, dev, "X")
    Xs = _as_f64(Xs, dev, "Xs")
    n, d = X.shape
    if n != chol.n:
        raise ValueError("X rows do not match the factorisation")
    m = Xs.shape[0]
    batch = L.shape[0]
    npad = padded_n(n)
    beta_t = _beta(beta, batch, d, dev)
    s_t = _per_batch(s, batch, dev, "s")
    sp_t = _per_batch(s_pred, batch, dev, "s_pred")
    w_t = None
    if z is None:
        w_t = _as_f64(w, dev, "w")
        if w_t.dim() == 1:
            w_t = w_t.reshape(1, -1)
        if tuple(w_t.shape) != (batch, n):
            raise ValueError(f"w: expected shape ({batch}, {n}), got {tuple(w_t.shape)}")
    else:
        z = z.reshape(batch, -1)
        if z.dtype != F64 or z.device != dev or z.shape[1] < npad or z.stride(1) != 1:
            raise ValueError(f"z: expected float64 ({batch}, {npad}) rows on {dev}")
    if out is None:
        mean = torch.empty((batch, m), dtype=F64, device=dev)
        var = torch.empty((batch, m), dtype=F64, device=dev)
    else:
        mean, var = out
    nbytes = _capi.lib().gp_predict_ws_bytes(n, m, batch, int(m_chunk))
    ws = (workspace or _DEFAULT_WS).get(nbytes, dev)
    _capi.call("gp_predict_ex", L.data_ptr(), npad, L.stride(0) if packed else npad * npad,
               X.data_ptr(), d, Xs.data_ptr(), d, n, m, d, beta_t.data_ptr(), d,
               s_t.data_ptr(), sp_t.data_ptr(), w_t.data_ptr() if w_t is not None else None, n,
               mean.data_ptr(), var.data_ptr(), mean.stride(0) if batch > 1 else m, batch,
               ws.data_ptr(), ws.numel(), int(m_chunk),
               _capi.LINV_PACKED if packed else _capi.LINV_PADDED,
               z.data_ptr() if z is not None else None,
               z.stride(0) if z is not None else 0, _stream(dev))
    return mean, var


def nll(chol: Cholesky, w) -> torch.Tensor:
    """1/2 ||L^-1 w||^2 + 1/2 log|A| per problem (GPmodule objective, no 2pi)."""
    dev = chol.linv_buf.device
    batch = chol.linv_buf.shape[0]
    npad = chol.linv_buf.shape[1]
    n = chol.n
    w_t = _as_f64(w, dev, "w").reshape(batch, n)
    out = torch.empty(batch, dtype=F64, device=dev)
    work = torch.empty((batch, n), dtype=F64, device=dev)
    _capi.call("gp_nll", chol.linv_buf.data_ptr(), npad, npad * npad, n, w_t.data_ptr(), n,
               chol.logdet.data_ptr(), out.data_ptr(), work.data_ptr(), batch, _stream(dev))
    return out


class LoglikWorkspace:
    """Device scratch of :func:`loglik` for fixed (n, batch): allocated once, so a Metropolis
    sweep calls gp_loglik with no allocation and no host synchronisation."""

    def __init__(self, n: int, batch: int, device):
        self.n, self.batch = n, batch
        nbytes = int(_capi.lib().gp_loglik_ws_bytes(n, batch))
        # zero-filled: the library's sticky internal-error word starts clear
        self.buf = torch.zeros(max(nbytes, 256), dtype=torch.uint8, device=device)
        self.info = torch.zeros(batch, dtype=torch.int32, device=device)

    def check_status(self, reset: bool = True) -> None:
        """Raise :class:`FactorizationInternalError` if any :func:`loglik` on this workspace
        since the last check had an internal factorisation error (gp_loglik_status; syncs the
        current stream).  A non-positive-definite proposal is not an error (ll = -inf)."""
        rc = _capi.lib().gp_loglik_status(self.buf.data_ptr(), self.n, self.batch,
                                          1 if reset else 0, _stream(self.buf.device))
        if rc == _capi.GPFIT_ERR_INTERNAL:
            raise FactorizationInternalError(
                "gp_loglik: a factorisation gave up (info = -1) since the last check; the "
                "chain's likelihood values are invalid")
        if rc != 0:
            raise _capi.GPFitError("gp_loglik_status", rc)


def loglik(X: torch.Tensor, beta: torch.Tensor, s: torch.Tensor, delta: torch.Tensor,
           w: torch.Tensor, ws: LoglikWorkspace, out: torch.Tensor | None = None) -> torch.Tensor:
    """ll[b] = -(1/2 w_b^T G_b^-1 w_b + 1/2 log|G_b|), G_b = s_b exp(-sum beta_b (dx)^2) + delta_b I;
    -inf where G_b is not positive definite (gp_loglik: Gram -> Cholesky -> quadratic form).

    X (n, d); beta (batch, d); s, delta (batch,); w (batch, n) -- all float64 on the device.
    """
    n, d = X.shape
    batch = ws.batch
    if n != ws.n or beta.shape != (batch, d) or w.shape != (batch, n):
        raise ValueError("loglik: shapes do not match the workspace")
    for t, nm in ((X, "X"), (beta, "beta"), (s, "s"), (delta, "delta"), (w, "w")):
        if t.dtype != F64 or not t.is_contiguous():
            raise TypeError(f"{nm} must be contiguous float64")
    out = torch.empty(batch, dtype=F64, device=X.device) if out is None else out
    _capi.call("gp_loglik", X.data_ptr(), n, d, d, beta.data_ptr(), d, s.data_ptr(),
               delta.data_ptr(), w.data_ptr(), n, batch, ws.buf.data_ptr(), ws.buf.numel(),
               out.data_ptr(), ws.info.data_ptr(), _stream(X.device))
    return out


def trmv(chol: Cholesky, w) -> torch.Tensor:
    """z = L^-1 w per problem -> (batch, n)."""
    dev = chol.linv_buf.device
    batch = chol.linv_buf.shape[0]
    npad = chol.linv_buf.shape[1]
    n = chol.n
    w_t = _as_f64(w, dev, "w").reshape(batch, n)
    z = torch.empty((batch, n), dtype=F64, device=dev)
    _capi.call("gp_trmv", chol.linv_buf.data_ptr(), npad, npad * npad, n, w_t.data_ptr(), n,
               z.data_ptr(), n, batch, _stream(dev))
    return z


@dataclass
class Prepared:
    """Cross-covariance of every test-point chunk, built by :func:`predict_prepare`."""

    n: int
    m: int
    batch: int
    m_chunk: int
    ws: torch.Tensor


def predict_prepare(X: torch.Tensor, Xs: torch.Tensor, beta, s, batch: int = 1,
                    m_chunk: int = 0, workspace: PredictWorkspace | None = None) -> Prepared:
    """Phase 1 of predict (gp_predict_cross): independent of the factorisation, so it can run
    on a side stream while :func:`cholesky_inverse` runs."""
    dev = X.device
    X = _as_f64(X, dev, "X")
    Xs = _as_f64(Xs, dev, "Xs")
    n, d = X.shape
    m = Xs.shape[0]
    beta_t = _beta(beta, batch, d, dev)
    s_t = _per_batch(s, batch, dev, "s")
    nbytes = _capi.lib().gp_predict_prepared_ws_bytes(n, m, batch, int(m_chunk))
    ws = (workspace or PredictWorkspace()).get(nbytes, dev)
    _capi.call("gp_predict_cross", X.data_ptr(), d, Xs.data_ptr(), d, n, m, d, beta_t.data_ptr(),
               d, s_t.data_ptr(), batch, ws.data_ptr(), ws.numel(), int(m_chunk), _stream(dev))
    return Prepared(n, m, batch, int(m_chunk), ws)


def predict_solve(chol: Cholesky, prep: Prepared, s_pred, w,
                  out: tuple[torch.Tensor, torch.Tensor] | None = None):
    """Phase 2 of predict (gp_predict_solve): mean / variance from a prepared cross-cov."""
    dev = chol.linv_buf.device
    batch, npad = chol.linv_buf.shape[0], chol.linv_buf.shape[1]
    n, m = chol.n, prep.m
    if prep.n != n or prep.batch != batch:
        raise ValueError("prepared cross-covariance does not match the factorisation")
    sp_t = _per_batch(s_pred, batch, dev, "s_pred")
    w_t = _as_f64(w, dev, "w").reshape(batch, n)
    if out is None:
        mean = torch.empty((batch, m), dtype=F64, device=dev)
        var = torch.empty((batch, m), dtype=F64, device=dev)
    else:
        mean, var = out
    _capi.call("gp_predict_solve", chol.linv_buf.data_ptr(), npad, npad * npad, n, m,
               sp_t.data_ptr(), w_t.data_ptr(), n, mean.data_ptr(), var.data_ptr(),
               mean.stride(0) if batch > 1 else m, batch, prep.ws.data_ptr(), prep.ws.numel(),
               prep.m_chunk, _stream(dev))
    return mean, var


class FitPredictContext:
    """Caller-owned execution context of :func:`fit_predict` (``gp_ctx_create``): the three
    library streams (factorisation | cross-covariance | prediction) on ``device``.

    Destroy it with :meth:`close` (or use it as a context manager) while the HIP runtime is up:
    the owner decides the teardown order, the library keeps no global state.
    """

    def __init__(self, device=None, cross_start: float = -1.0, aux_free_cus: int = -1,
                 aux_chunks: int = -1):
        import ctypes
        self.device = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        self._h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _capi.call("gp_ctx_create", float(cross_start), int(aux_free_cus),
                       ctypes.addressof(self._h))
            if aux_chunks != -1:
                self.set_aux_chunks(aux_chunks)

    def set_aux_chunks(self, nchunks: int) -> None:
        """Chunks whose cross-covariance runs beside the factorisation / earlier TRMMs
        (``gp_ctx_set_aux_chunks``; -1 = all, the default)."""
        _capi.call("gp_ctx_set_aux_chunks", self._h.value, int(nchunks))

    @property
    def handle(self) -> int | None:
        return self._h.value

    def close(self) -> None:
        if self._h.value:
            with torch.cuda.device(self.device):
                _capi.call("gp_ctx_destroy", self._h.value)
            self._h.value = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def fit_predict(X, Xs, beta, s, delta, s_pred, w, m_chunk: int = 0,
                workspace: PredictWorkspace | None = None, out=None,
                ctx: FitPredictContext | None = None, check: bool = True):
    """Gram -> Cholesky/L^-1 -> predict for ``batch`` GPs in one gp_fit_predict call.

    With ``ctx`` the cross-covariance runs on the context's own stream under the
    factorisation's latency-bound tail, then the per-chunk TRMM + mean/var; without it every
    step runs in order on the current stream.  ``check`` synchronises and raises if a Gram was
    not positive definite or its factorisation had an internal error (info = -1): the mean /
    var would be unspecified.  Returns (mean, var, chol).
    """
    dev = X.device
    X = _as_f64(X, dev, "X")
    Xs = _as_f64(Xs, dev, "Xs")
    n, d = X.shape
    m = Xs.shape[0]
    bt = torch.as_tensor(beta)
    batch = bt.shape[0] if bt.dim() == 2 else 1
    beta_t = _beta(beta, batch, d, dev)
    s_t = _per_batch(s, batch, dev, "s")
    d_t = _per_batch(delta, batch, dev, "delta")
    sp_t = _per_batch(s_pred, batch, dev, "s_pred")
    w_t = _as_f64(w, dev, "w").reshape(batch, n)
    npad = padded_n(n)
    G = torch.empty((batch, n, n), dtype=F64, device=dev)
    Linv = torch.empty((batch, npad, npad), dtype=F64, device=dev)
    info = torch.empty(batch, dtype=torch.int32, device=dev)
    logdet = torch.empty(batch, dtype=F64, device=dev)
    if out is None:
        mean = torch.empty((batch, m), dtype=F64, device=dev)
        var = torch.empty((batch, m), dtype=F64, device=dev)
    else:
        mean, var = out
    nbytes = _capi.lib().gp_fit_predict_ws_bytes(n, m, batch, int(m_chunk))
    ws = (workspace or PredictWorkspace()).get(nbytes, dev)
    if ctx is not None and ctx.device != dev:
        raise ValueError(f"context is on {ctx.device}, inputs on {dev}")
    _capi.call("gp_fit_predict", X.data_ptr(), d, Xs.data_ptr(), d, n, m, d, beta_t.data_ptr(),
               d, s_t.data_ptr(), d_t.data_ptr(), sp_t.data_ptr(), w_t.data_ptr(), n,
               G.data_ptr(), n, n * n, Linv.data_ptr(), npad, npad * npad, info.data_ptr(),
               logdet.data_ptr(), mean.data_ptr(), var.data_ptr(),
               mean.stride(0) if batch > 1 else m, batch, ws.data_ptr(), ws.numel(),
               int(m_chunk), ctx.handle if ctx is not None else None, _stream(dev))
    ch = Cholesky(n, G, Linv, info, logdet)
    if check:
        ch.check()
    return mean, var, ch


def cholesky(G: torch.Tensor, overwrite: bool = True):
    """Plain blocked Cholesky (gp_potrf, LAPACK dpotrf('L')): returns (L, info, logdet) with L
    the lower factor as a (batch, n, n) logical tensor."""
    _check_device(G, "G")
    if G.dtype != F64:
        raise TypeError("G must be float64")
    if G.dim() == 2:
        G = G.unsqueeze(0)
    batch, n, n2 = G.shape
    if n != n2:
        raise ValueError("G must be square")
    A = G if (overwrite and G.is_contiguous()) else G.contiguous().clone()
    info = torch.empty(batch, dtype=torch.int32, device=G.device)
    logdet = torch.empty(batch, dtype=F64, device=G.device)
    nbytes = int(_capi.lib().gp_potrf_ws_bytes(n, batch))
    ws = _potrf_ws(G.device, nbytes)
    _capi.call("gp_potrf_ws", A.data_ptr(), n, n, n * n, batch, info.data_ptr(),
               logdet.data_ptr(), ws.data_ptr(), ws.numel(), _stream(G.device))
    return torch.tril(A.transpose(-1, -2)), info, logdet


def _lapack_buf(L: torch.Tensor) -> torch.Tensor:
    """(batch, n, n) logical lower factor -> contiguous column-major buffer [b, j, i] = L[i, j]."""
    _check_device(L, "L")
    if L.dim() == 2:
        L = L.unsqueeze(0)
    return L.to(F64).transpose(-1, -2).contiguous()


def trtri(L: torch.Tensor) -> Cholesky:
    """L^-1 of a lower factor (gp_trtri, LAPACK dtrtri('L','N')); returns a :class:`Cholesky`
    whose ``info`` flags a zero diagonal, usable with :func:`predict` / :func:`nll`."""
    Lb = _lapack_buf(L)
    batch, n, _ = Lb.shape
    npad = padded_n(n)
    Linv = torch.empty((batch, npad, npad), dtype=F64, device=Lb.device)
    info = torch.empty(batch, dtype=torch.int32, device=Lb.device)
    _capi.call("gp_trtri", Lb.data_ptr(), n, n, n * n, Linv.data_ptr(), npad, npad * npad, batch,
               info.data_ptr(), _stream(Lb.device))
    logdet = 2.0 * torch.log(torch.diagonal(Lb, dim1=-2, dim2=-1)).sum(-1)
    return Cholesky(n, Lb, Linv, info, logdet)


def predict_chol(L: torch.Tensor, X, Xs, beta, s, s_pred, w, m_chunk: int = 0,
                 workspace: PredictWorkspace | None = None):
    """Posterior mean / variance from a Cholesky factor L (gp_predict_chol: gp_trtri into the
    workspace, then gp_predict).  Returns (mean, var, info)."""
    Lb = _lapack_buf(L)
    dev = Lb.device
    batch, n, _ = Lb.shape
    X = _as_f64(X, dev, "X")
    Xs = _as_f64(Xs, dev, "Xs")
    d = X.shape[1]
    m = Xs.shape[0]
    beta_t = _beta(beta, batch, d, dev)
    s_t = _per_batch(s, batch, dev, "s")
    sp_t = _per_batch(s_pred, batch, dev, "s_pred")
    w_t = _as_f64(w, dev, "w").reshape(batch, n)
    mean = torch.empty((batch, m), dtype=F64, device=dev)
    var = torch.empty((batch, m), dtype=F64, device=dev)
    info = torch.empty(batch, dtype=torch.int32, device=dev)
    nbytes = _capi.lib().gp_predict_chol_ws_bytes(n, m, batch, int(m_chunk))
    ws = (workspace or PredictWorkspace()).get(nbytes, dev)
    _capi.call("gp_predict_chol", Lb.data_ptr(), n, n * n, X.data_ptr(), d, Xs.data_ptr(), d, n,
               m, d, beta_t.data_ptr(), d, s_t.data_ptr(), sp_t.data_ptr(), w_t.data_ptr(), n,
               mean.data_ptr(), var.data_ptr(), m, batch, info.data_ptr(), ws.data_ptr(),
               ws.numel(), int(m_chunk), _stream(dev))
    return mean, var, info


def realize(mean: torch.Tensor, var: torch.Tensor, seed: int, offset: int = 0,
            out: torch.Tensor | None = None) -> torch.Tensor:
    """One marginal draw per entry, mean + sqrt(max(var, 0)) z with z from Philox4x32-10 keyed
    by ``seed`` at counter offset ``offset`` (gp_realize); deterministic per (seed, offset)."""
    _check_device(mean, "mean")
    if mean.dtype != F64 or var.dtype != F64 or mean.shape != var.shape:
        raise TypeError("mean / var must be float64 tensors of one shape")
    mean_c, var_c = mean.contiguous(), var.contiguous()
    out = torch.empty_like(mean_c) if out is None else out
    _capi.call("gp_realize", mean_c.data_ptr(), var_c.data_ptr(), mean_c.numel(),
               int(seed) & (2 ** 64 - 1), int(offset) & (2 ** 64 - 1), out.data_ptr(),
               _stream(mean.device))
    return out
