"""Randomized fixed-rank SVD on the GPU — drop-in for ``src/svd.py`` (``randomized_svd``).

Reference: ``src/svd.py:12-82`` (Halko et al. 2011): Gaussian test matrix Omega (ny x (p+k),
float32, drawn from ``np.random``), ``Y = X Omega``, ``q`` power iterations ``Y = X X^T Y``,
``Q = qr(Y)``, ``B = Q^T X``, ``U_B, S, V = svd(B)``, ``U = Q U_B``, truncation to ``p``.

Build (all arithmetic in libgpfit, fp64):
  * every product is an MFMA GEMM (``gp_gemm_ex``; the ny-long inner products use split-K;
    a float32 X -- the reference's own fit / load dtype -- is read as stored and widened on
    load, never copied to fp64);
    the power iteration is evaluated as ``X (X^T Y)`` — the same matrix as the reference's
    left-associated ``(X X^T) Y`` without forming the n x n Gram;
  * ``qr(Y)`` is shifted CholeskyQR3 (Fukaya et al. 2020): ``Y`` after a power step is very
    ill-conditioned, so the first pass factors ``Y^T Y + s I`` (s = 11 (n r + r(r+1)) u ||Y||^2,
    a trace bound), two plain CholeskyQR passes then restore orthogonality to ~u.  The
    Cholesky + inverse is ``gp_potrf_inv``;
  * a rank-deficient ``Y`` (e.g. ``init_model``'s ``r = min(25, n, ny)`` on a column-centred
    ensemble of n <= 25 runs, rank <= n - 1) makes a CholeskyQR pass fail; numpy's Householder
    QR still returns an orthonormal Q there.  The fallback: eigen-basis of ``Y^T Y``
    (gp_syevj) for the numerically nonzero directions, CholeskyQR2 to restore orthogonality,
    and a seeded orthonormal completion of the null directions (B = Q^T X sees only range(X)
    there, so any completion gives the reference's U, S, Vh up to the zero singular values);
  * ``svd(B)`` comes from the Jacobi eigendecomposition of ``B B^T`` (``gp_syevj``, r <= 1024):
    ``S = sqrt(eig)``, ``V^T = S^-1 U_B^T B``.
Singular vectors are unique up to sign (and rotation inside clusters); tests compare signed.
The reference's ``return_error`` bound is always 0 because ``S`` is truncated before ``S[p]``
is read (src/svd.py:66-76): mirrored.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _capi, kernels
from .blas import CM, gemm, rowscale, shift_diag, syevj

_U = 2.0 ** -53


def _device(dev) -> torch.device:
    if dev is not None:
        return torch.device(dev)
    if not torch.cuda.is_available():
        raise RuntimeError("randomized_svd runs on the GPU (libgpfit); no HIP device found")
    return torch.device("cuda", torch.cuda.current_device())


def _to_device(a, dev) -> torch.Tensor:
    """Device copy in the array's own dtype when float32 or float64 (anything else: float64);
    host arrays cross PCIe as stored."""
    if torch.is_tensor(a):
        return a.to(device=dev) if a.dtype in (torch.float32, torch.float64) else \
            a.to(device=dev, dtype=torch.float64)
    a = np.ascontiguousarray(np.asarray(a))
    if a.dtype not in (np.float32, np.float64):
        a = a.astype(np.float64)
    return torch.from_numpy(a).to(dev)


def _chol_qr(Y: CM, shift: bool) -> CM:
    G = gemm(True, False, Y, Y)                              # r x r  = Y^T Y
    r = G.rows
    if shift:
        shift_diag(G, 11.0 * (Y.rows * r + r * (r + 1)) * _U)
    ch = kernels.cholesky_inverse(G.t[:r, :r].reshape(1, r, r).contiguous())
    ch.check()
    Linv = CM(ch.linv_buf[0], r, r, ch.linv_buf.shape[1])
    return gemm(False, True, Y, Linv)                        # Y L^-T


def orthonormalize(Y: CM) -> CM:
    """Orthonormal n x r basis containing range(Y) (r <= n): shifted CholeskyQR3, or the
    rank-revealing fallback when Y is (numerically) rank deficient."""
    try:
        Q = _chol_qr(Y, shift=True)
        Q = _chol_qr(Q, shift=False)
        return _chol_qr(Q, shift=False)
    except ValueError:       # a pass hit a non-positive pivot: rank(Y) < r
        return _orthonormalize_deficient(Y)


def _orthonormalize_deficient(Y: CM, rel_tol: float = 1e-10, seed: int = 0x5EED) -> CM:
    n, r = Y.rows, Y.cols
    dev = Y.t.device
    G = gemm(True, False, Y, Y)                              # r x r = Y^T Y
    lam, V, _ = syevj(G, want_sqrt=False)                    # descending
    lam_h = lam.cpu().numpy()
    k = int(np.sum(lam_h > rel_tol * max(lam_h[0], 0.0))) if r else 0
    parts = []
    if k:
        Vk = CM(V.t[:k], r, k, V.ld)                         # first k eigenvectors
        Q1 = gemm(False, False, Y, Vk)                       # n x k, cond <= rel_tol^-1/2
        Q1 = _chol_qr(_chol_qr(_chol_qr(Q1, shift=True), shift=False), shift=False)
        parts.append(Q1)
    if k < r:
        # seeded Gaussian columns, projected off range(Q1) twice, then CholeskyQR2
        z = np.random.default_rng(seed).standard_normal((r - k, n))
        Z = CM.of_rowmajor(torch.as_tensor(z, dtype=torch.float64, device=dev))  # n x (r-k)
        if k:
            for _ in range(2):
                P = gemm(True, False, parts[0], Z)           # k x (r-k)
                gemm(False, False, parts[0], P, alpha=-1.0, beta=1.0, C=Z)
        parts.append(_chol_qr(_chol_qr(Z, shift=False), shift=False))
    Q = CM.empty(n, r, dev)
    c = 0
    for part in parts:
        Q.t[c:c + part.cols, :n] = part.t[: part.cols, :n]
        c += part.cols
    return Q


def legacy_normal_f32(shape, threads: int | None = None) -> np.ndarray:
    """``np.random.normal(size=shape).astype(np.float32)`` on numpy's global legacy generator,
    bit for bit (``src/svd.py:51``), drawn by libgpfit's host generator
    (``gp_host_legacy_normal_f32``: vectorised MT19937, the polar method's log / sqrt on
    ``threads`` host threads); numpy's global state is advanced exactly as that call would."""
    out, state = _legacy_normal_from(np.random.get_state(), shape, threads)
    np.random.set_state(state)
    return out


def _legacy_normal_from(state, shape, threads: int | None = None):
    """The draw of :func:`legacy_normal_f32` from an explicit numpy state tuple, touching no
    global state: returns (deviates, the state numpy's own call would leave)."""
    import os
    name, key, pos, has_gauss, cached = state[:5]
    if name != "MT19937":
        raise ValueError(f"legacy_normal_f32: global generator is {name}, not MT19937")
    if threads is None:
        env = os.environ.get("OMP_NUM_THREADS")
        threads = int(env) if env and env.isdigit() and int(env) > 0 else \
            len(os.sched_getaffinity(0))
        threads = min(threads, 16)
    out = np.empty(shape, dtype=np.float32)
    key = np.array(key, dtype=np.uint32, copy=True)
    pos_c, hg_c, g_c = ctypes.c_int(int(pos)), ctypes.c_int(int(has_gauss)), \
        ctypes.c_double(float(cached))
    _capi.call("gp_host_legacy_normal_f32", key.ctypes.data, ctypes.addressof(pos_c),
               ctypes.addressof(hg_c), ctypes.addressof(g_c), int(out.size), out.ctypes.data,
               int(threads))
    return out, ("MT19937", key, pos_c.value, hg_c.value, g_c.value)


class LegacyNormalDraw:
    """:func:`legacy_normal_f32` on a host worker thread.  numpy's global state is read here, on
    the calling thread, and set to the advanced state by :meth:`result`, on the calling thread
    again: the worker runs only the C generator on its own copy of the state, so it never reads
    or writes numpy's global generator (a main-thread draw in between would see the state before
    this draw, as if it had come first, and :meth:`result` then overwrites its advance)."""

    def __init__(self, shape, threads: int | None = None):
        from concurrent.futures import ThreadPoolExecutor
        st = np.random.get_state()
        if st[0] != "MT19937":
            raise ValueError(f"legacy_normal_f32: global generator is {st[0]}, not MT19937")
        pool = ThreadPoolExecutor(max_workers=1)
        self._fut = pool.submit(_legacy_normal_from, st, shape, threads)
        pool.shutdown(wait=False)
        self._out = None

    def result(self) -> np.ndarray:
        if self._out is None:
            self._out, state = self._fut.result()
            np.random.set_state(state)
        return self._out


def randomized_svd(X, p, k=None, q=1, return_error=False, omega=None, device=None):
    """Same signature and return shapes as ``src/svd.py:randomized_svd``.

    ``X`` is (m, n) (numpy or torch); returns ``(U (m, p), S (p,), Vh (p, n))`` as numpy arrays
    when ``X`` is numpy, torch device tensors otherwise.  ``omega`` overrides the test matrix;
    by default it is drawn exactly as the reference does (``np.random.normal(size=(n, p+k))``
    cast to float32), so a seeded ``np.random`` reproduces the reference's Omega.
    Output dtype follows the reference's numpy promotion (src/svd.py:51-68: a float32 X times
    the float32 Omega stays float32, float64 X gives float64); the arithmetic is fp64 either way.
    """
    as_numpy = not torch.is_tensor(X)
    f32_out = (np.asarray(X).dtype == np.float32) if as_numpy else (X.dtype == torch.float32)
    dev = _device(device if as_numpy else (device or X.device))
    # a float32 X stays float32 on the device: the GEMMs that stream it (gp_gemm_ex) widen it
    # exactly as they load it, so there is no fp64 copy of the ensemble (5.5 GB at the fit's
    # 512 x 1,347,945) and the products are bit-identical to those of an fp64 copy
    Xt = _to_device(X, dev)
    if not (Xt.dim() == 2 and Xt.stride(1) == 1 and Xt.stride(0) >= Xt.shape[1]):
        Xt = Xt.contiguous()        # (a row-strided view -- the padded y_std -- is read in place)
    m_rows, n_cols = Xt.shape
    if k is None:
        k = p
    r = p + k
    if r > 1024:
        raise ValueError("randomized_svd: p + k must be <= 1024 (Jacobi core)")
    if omega is None:
        omega = legacy_normal_f32((n_cols, r))
    Om = _to_device(omega, dev).contiguous()      # float32 (as drawn) or float64
    Xc = CM.of_rowmajor(Xt)          # (n_cols x m_rows), ld = n_cols
    # Omega as drawn (float32, row-major n_cols x r = column-major r x n_cols, ld = r), read
    # in place and widened exactly on load: with the tall-skinny kernels' unmasked fast path
    # X Omega runs 1.13 ms against 1.23 for an fp64 column-major copy of Omega (which the
    # masked kernel needed: 2.1 vs 1.3-1.5 ms, profiles/r05/r05k_ts_probe.log), and the copy
    # itself is gone (profiles/r05/r05_tsfast_ab.log).  Same sums, same bits.
    Oc = CM.of_rowmajor(Om)          # (r x n_cols)
    Y = gemm(True, True, Xc, Oc)     # (m_rows x r) = X Omega
    for _ in range(q):
        # Z = X^T Y made as Z^T = Y^T X (r x n_cols: the same products in the same order, laid
        # out row-major), so X Z reads Z's r values of each k contiguously, as X Omega reads
        # Omega (profiles/r05/r05_tsfast2_pca.log: X Z with a column-major Z was the slowest
        # of the four ensemble-streaming products)
        Zt = gemm(True, True, Y, Xc)     # (r x n_cols) = Y^T X = (X^T Y)^T
        Y = gemm(True, True, Xc, Zt)     # (m_rows x r) = X X^T Y
    if r > m_rows:
        # more test vectors than rows: range(Y) is all of R^m_rows (numpy's reduced QR gives
        # an m_rows x m_rows Q), so keep m_rows of them
        Y = CM(Y.t[:m_rows], m_rows, m_rows, Y.ld)
    Q = orthonormalize(Y)
    B = gemm(True, True, Q, Xc)      # (r x n_cols) = Q^T X
    G = gemm(False, True, B, B)      # (r x r) = B B^T
    S, UB, _ = syevj(G, want_sqrt=True)      # singular values of B, descending
    Vh = gemm(True, False, UB, B)    # U_B^T B
    rowscale(Vh, S, inverse=True)    # S^-1 U_B^T B
    U = gemm(False, False, Q, UB)    # (m_rows x r)
    U_t = U.logical()[:, :p].contiguous()
    S_t = S[:p].contiguous()
    Vh_t = Vh.logical()[:p, :].contiguous()
    out = (U_t, S_t, Vh_t)
    if f32_out:
        out = tuple(t.to(torch.float32) for t in out)
    if as_numpy:
        out = tuple(t.cpu().numpy() for t in out)
    if return_error:
        return out, 0.0
    return out
