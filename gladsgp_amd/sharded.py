"""Test-point sharding of single-output GPs across ranks ("single-output GP").

The reference's scalar consumers predict one GP (P = 1) per model at many test points:
``fit_scalar_models.py:477-481`` (64 posterior samples), ``mean_response.py:114-126``
(16 samples), and the BASELINE C2/C3 configurations (one GP, m = 10k / 100k).  Their units
(sample, PC) are too few to deal across 8 GPUs, so here the m test points are split instead:
rank r predicts the contiguous block ``shard_range`` of the points and one gather brings the
(mean, var) blocks to rank 0.

Two ways to get every rank the factor it needs:

* ``mode="redundant"``: every rank builds the Gram and factorises it itself (gp_fit_predict
  on its block; the Amdahl term is the factorisation, ~2 ms of a 27 ms C3 step);
* ``mode="broadcast"``: rank 0 alone factorises and broadcasts L^-1 (tile-packed, half the
  bytes of the padded square, read by the other ranks' prediction in place) with z = L^-1 w,
  while its own block is shortened by the factorisation's time in test-point equivalents
  (``balanced_split``), so all ranks finish together.

:class:`PipelinedPredictor` runs a *stream* of GPs as a two-stage pipeline: in step k rank 0
factorises GP k+1 and broadcasts its L^-1 (asynchronously over RCCL, double-buffered) while
every rank predicts GP k on its block; each step ends with one gather to rank 0.  A GP's
latency is two steps; the throughput is what the 1->8 GPU scaling bench reports.

SPMD convention: every rank passes the same hyperparameters and design (as torch DDP code
does); only rank 0's factorisation is used in the broadcast modes.  All arithmetic is in
libgpfit (gp_gram_ardse, gp_potrf_inv_ws, gp_predict, gp_fit_predict); collectives are
torch.distributed (RCCL over xGMI on GPUs, gloo on the CPU tests).
"""
from __future__ import annotations

import time

import numpy as np
import torch
import torch.distributed as tdist

from . import _capi, kernels
from . import dist as gdist

F64 = torch.float64


def split_counts(m: int, world: int, rank0_extra_points: float = 0.0) -> list[int]:
    """Test points per rank: rank 0 takes ``rank0_extra_points`` fewer than an even share (the
    factorisation it runs in addition, in test-point equivalents), the others split the rest
    evenly (balanced to within one point)."""
    if world <= 1:
        return [m]
    m1 = int(np.ceil((m + rank0_extra_points) / world))
    m0 = max(0, m - (world - 1) * m1)
    rest = [b - a for a, b in (gdist.shard_range(m - m0, r, world - 1) for r in range(world - 1))]
    return [m0] + rest


def _offsets(counts: list[int]) -> list[int]:
    return [int(x) for x in np.concatenate([[0], np.cumsum(counts)[:-1]])]


class LinvPacker:
    """The single-GP broadcast's payload, one flat float64 vector:
    ``[L^-1 tile-packed (elems) | z = L^-1 w (npad) | info (1)]``.

    L^-1 travels in the tile-packed layout (gp_pack_linv: column c of the padded buffer from row
    16 floor(c/16) on, about half the padded square, 67 MB at n = 4096) that the prediction
    reads in place (gp_predict_ex), so the receiving ranks run no unpack; z is computed once on
    rank 0 with the prediction's own arithmetic (gp_predict_z), so they run no trmv either
    (round 4 had every rank >= 1 unpack 134 MB and redo the 71 MB trmv each step).  The info
    slot carries rank 0's factorisation status, so every receiver learns from the same
    collective whether the factor it got is valid (a rank-0-only raise before the broadcast
    would leave the other ranks waiting in it)."""

    def __init__(self, npad: int, device=None, n: int | None = None):
        self.npad = npad
        self.n = npad if n is None else n
        q = npad // 16
        self.elems = npad * npad - 128 * q * (q - 1)      # gp_linv_packed_elems
        self.numel = self.elems                           # the L^-1 part (round-4 name)
        self.z_off = self.elems
        self.info_off = self.elems + npad

    def buffer(self, device) -> torch.Tensor:
        return torch.zeros(self.info_off + 1, dtype=F64, device=device)

    @staticmethod
    def order(npad: int) -> torch.Tensor:
        """The tile-packed layout as flat indices into the column-major (npad x npad) buffer
        (host tensor; documents gp_pack_linv's order for host-side tests)."""
        idx = [c * npad + torch.arange((c // 16) * 16, npad) for c in range(npad)]
        return torch.cat(idx)

    def pack(self, linv_buf: torch.Tensor, info: torch.Tensor, out: torch.Tensor,
             w: torch.Tensor | None = None) -> torch.Tensor:
        """Rank 0: L^-1 (padded, (1, npad, npad)) tile-packed, z = L^-1 w (when ``w`` is
        given) and the info word into ``out``."""
        _capi.call("gp_pack_linv", linv_buf.data_ptr(), self.n, self.npad, out.data_ptr(),
                   kernels._stream(out.device))
        if w is not None:
            ch = kernels.Cholesky(self.n, None, linv_buf, info, None)
            kernels.predict_z(ch, w, out=self.z(out).reshape(1, self.npad))
        out[self.info_off:].copy_(info.reshape(1).to(F64))
        return out

    def unpack(self, packed: torch.Tensor, linv_buf: torch.Tensor) -> torch.Tensor:
        """Into a padded buffer whose upper triangle and padding are already zero (not needed
        by the prediction, which reads the packed form in place)."""
        _capi.call("gp_unpack_linv", packed.data_ptr(), self.n, linv_buf.data_ptr(),
                   self.npad, kernels._stream(packed.device))
        return linv_buf

    def z(self, packed: torch.Tensor) -> torch.Tensor:
        return packed[self.z_off:self.info_off]

    def info(self, packed: torch.Tensor) -> torch.Tensor:
        """The sender's info (device, int32, shape (1,))."""
        return packed[self.info_off:].to(torch.int32)

    def view(self, packed: torch.Tensor, info: torch.Tensor | None = None) -> kernels.PackedLinv:
        """The payload as the prediction reads it: tile-packed L^-1 and z, in place."""
        return kernels.PackedLinv(self.n, packed[: self.elems].view(1, self.elems),
                                  self.info(packed) if info is None else info,
                                  self.z(packed).view(1, self.npad))


def _wire_bcast(ctx: gdist.Context, t: torch.Tensor, async_op: bool):
    """Broadcast from rank 0: RCCL moves device tensors in place (optionally async); gloo (CPU
    tests, several ranks on one GPU) stages through the host, synchronously."""
    if ctx.backend == "nccl":
        return tdist.broadcast(t, src=0, async_op=async_op)
    gdist.broadcast_(ctx, t)
    return None


def predict_sharded(ctx: gdist.Context, X: torch.Tensor, Xs: torch.Tensor, beta, s, delta,
                    s_pred, w, *, mode: str = "redundant", counts: list[int] | None = None,
                    m_chunk: int = 0, fctx: kernels.FitPredictContext | None = None,
                    workspace: kernels.Workspace | None = None, gather: bool = True,
                    check: bool = True):
    """Posterior mean / variance of one GP at ``Xs`` (m x d, the whole set on every rank),
    the test points split over ranks.

    Returns ``(mean, var)`` of shape (m,) on rank 0 and ``None`` on the others with
    ``gather``; else this rank's block ``(mean_r, var_r, (lo, hi))``.  ``counts`` overrides the
    per-rank split (default: even for "redundant", rank 0 shortened by a measured
    factorisation and prediction times for "broadcast" (:func:`calibrate_split`) -- pass
    :func:`split_counts` / :func:`balanced_split` of your own calibration to avoid the
    measurement).  ``check`` synchronises once and raises if the factorisation
    failed (info != 0); without it the caller owns that check.  Single process: the whole m on
    this device.
    """
    if mode not in ("redundant", "broadcast"):
        raise ValueError(f"mode must be 'redundant' or 'broadcast', got {mode!r}")
    dev = X.device
    # collectives run whenever there is a process group, also at world size 1 (an RCCL
    # communicator of one rank exercises the same code path as the N-GPU runs)
    dist_on = ctx is not None and ctx.distributed
    world = ctx.world if dist_on else 1
    rank = ctx.rank if dist_on else 0
    m = Xs.shape[0]
    n = X.shape[0]
    if counts is None:
        if mode == "broadcast" and dist_on:
            counts, _, _ = calibrate_split(ctx, X, Xs, beta, s, delta, s_pred, w,
                                           m_chunk=m_chunk)
        else:
            counts = [b - a for a, b in (gdist.shard_range(m, r, world) for r in range(world))]
    if len(counts) != world or sum(counts) != m:
        raise ValueError(f"counts {counts} do not split m = {m} over {world} ranks")
    lo = _offsets(counts)[rank]
    hi = lo + counts[rank]
    Xl = Xs[lo:hi].contiguous()
    buf = torch.empty((2, max(hi - lo, 1)), dtype=F64, device=dev)
    if mode == "redundant" or not dist_on:
        if hi > lo:
            kernels.fit_predict(X, Xl, beta, s, delta, s_pred, w, m_chunk=m_chunk,
                                workspace=workspace, out=(buf[0:1, : hi - lo],
                                                          buf[1:2, : hi - lo]),
                                ctx=fctx, check=check)
    else:
        npad = kernels.padded_n(n)
        packer = LinvPacker(npad, dev, n=n)
        packed = packer.buffer(dev)
        if rank == 0:
            G = kernels.gram(X, beta, s, delta)
            ch = kernels.cholesky_inverse(G)
            packer.pack(ch.linv_buf, ch.info, packed, w=w)
        _wire_bcast(ctx, packed, async_op=False)
        if check:                                  # every rank raises alike (rank 0's info)
            kernels.check_info(packer.info(packed))
        # rank 0 from its padded L^-1, the others from the payload in place; z from the payload
        src = ch if rank == 0 else packer.view(packed)
        if hi > lo:
            kernels.predict(src, X, Xl, beta, s, s_pred, w, m_chunk=m_chunk, workspace=workspace,
                            out=(buf[0:1, : hi - lo], buf[1:2, : hi - lo]),
                            z=packer.z(packed).view(1, npad))
    mine = buf[:, : hi - lo]
    if not gather:
        return mine[0], mine[1], (lo, hi)
    if not dist_on:
        return mine[0], mine[1]
    res = gdist.gather_cols(ctx, mine.contiguous(), counts)
    if res is None:
        return None
    return res[0], res[1]


def calibrate(ctx: gdist.Context, X, Xs, beta, s, delta, s_pred, w, points: int = 16384,
              reps: int = 3) -> tuple[float, float]:
    """Rank 0 measures one factorisation (Gram + gp_potrf_inv) and the prediction time per test
    point (median of ``reps``); the pair is broadcast so every rank computes the same split."""
    dev = X.device
    calib = torch.zeros(2, dtype=F64, device=dev)
    if ctx is None or not ctx.distributed or ctx.rank == 0:
        mc = min(Xs.shape[0], points)
        Xc = Xs[:mc].contiguous()
        tf, tp = [], []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            ch = kernels.cholesky_inverse(kernels.gram(X, beta, s, delta))
            torch.cuda.synchronize(dev)
            t1 = time.perf_counter()
            kernels.predict(ch, X, Xc, beta, s, s_pred, w)
            torch.cuda.synchronize(dev)
            tf.append(t1 - t0)
            tp.append((time.perf_counter() - t1) / mc)
        calib[0], calib[1] = sorted(tf)[reps // 2], sorted(tp)[reps // 2]
    if ctx is not None and ctx.distributed:
        gdist.broadcast_(ctx, calib)
    return float(calib[0]), float(calib[1])


def balanced_split(m: int, world: int, t_fact: float, T, granule: int = 128) -> list[int]:
    """Test points per rank for the pipelined schedule, from measured times: rank 0 runs the
    factorisation (``t_fact``) and predicts m0 points, ranks 1.. predict the rest split evenly;
    m0 minimises max(t_fact + T(m0), T(m1)), m1 = ceil((m - m0) / (world - 1)).  ``T(points)``
    is the prediction time of that many points (non-decreasing; on the GPU a staircase in the
    TRMM's residency rounds of 32 column panels: 4096 points at n = 4096, so a point-linear
    model misplaces the split by up to a round, ~0.9 ms of a ~3.4 ms step at 8 ranks).  m0 is
    a multiple of ``granule`` (the TRMM's 128-point panel) or all of m."""
    if world <= 1:
        return [m]
    cache = {}

    def t(points):
        if points <= 0:
            return 0.0
        if points not in cache:
            cache[points] = float(T(points))
        return cache[points]

    def m1_of(m0):
        return -(-(m - m0) // (world - 1))

    # f(m0) = t_fact + T(m0) - T(m1(m0)) is non-decreasing in m0: find its sign change
    lo, hi = 0, -(-m // world) // granule + 1          # in granules
    if t_fact >= t(m1_of(0)):
        best = 0
    else:
        while hi - lo > 1:
            mid = (lo + hi) // 2
            if t_fact + t(min(m, mid * granule)) - t(m1_of(min(m, mid * granule))) < 0:
                lo = mid
            else:
                hi = mid
        cands = {min(m, lo * granule), min(m, hi * granule)}
        best = min(cands, key=lambda m0: (max(t_fact + t(m0), t(m1_of(m0))), -m0))
    m0 = best
    rest = [b - a for a, b in (gdist.shard_range(m - m0, r, world - 1) for r in range(world - 1))]
    return [m0] + rest


def calibrate_split(ctx: gdist.Context, X, Xs, beta, s, delta, s_pred, w, m_chunk: int = 0,
                    reps: int = 3):
    """Rank 0 measures the factorisation (Gram + gp_potrf_inv + the broadcast payload's pack and
    z) and the prediction time of candidate point counts (kernels.predict from that payload on
    the first points of ``Xs``, median of ``reps``)
    and picks the split with :func:`balanced_split`; the counts are broadcast so every rank
    uses the same.  Returns (counts, t_fact, t_point) -- t_point at a full 16384-point chunk,
    for reporting.  One rank: ([m], nan, nan) with nothing measured.  The result is memoised
    per (device, n, m, world, m_chunk), so one-shot :func:`predict_sharded` callers pay the
    measurement once per shape (pass ``counts`` to skip it entirely)."""
    dev = X.device
    world = ctx.world if ctx is not None and ctx.distributed else 1
    m = Xs.shape[0]
    key = (str(dev), X.shape[0], m, world, int(m_chunk))
    if world == 1:
        # one rank: the split is [m] whatever the times (a one-rank communicator rehearsal
        # included); nothing to measure
        return [m], float("nan"), float("nan")
    if key in _SPLIT_CACHE:
        # the split depends on the shapes, not on the GP's values: measured once per shape
        # (every rank holds the same cache entry, so no collective is needed)
        return _SPLIT_CACHE[key]
    buf = torch.zeros(world + 2, dtype=F64, device=dev)
    if ctx is None or not ctx.distributed or ctx.rank == 0:
        # rank 0's extra work per GP: Gram + factorisation + the payload (tile-packed L^-1 and
        # z = L^-1 w); every rank's prediction: from the payload with z given (no trmv), as
        # PipelinedPredictor and predict_sharded(mode="broadcast") run it
        npad = kernels.padded_n(X.shape[0])
        packer = LinvPacker(npad, dev, n=X.shape[0])
        payload = packer.buffer(dev)
        tf = []
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            ch = kernels.cholesky_inverse(kernels.gram(X, beta, s, delta))
            packer.pack(ch.linv_buf, ch.info, payload, w=w)
            torch.cuda.synchronize(dev)
            tf.append(time.perf_counter() - t0)
        t_fact = sorted(tf)[reps // 2]
        ws = kernels.PredictWorkspace()
        view = packer.view(payload)

        def T(points):
            Xc = Xs[:points].contiguous()
            kernels.predict(view, X, Xc, beta, s, s_pred, None, m_chunk=m_chunk, workspace=ws)
            ts = []
            for _ in range(reps):
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                kernels.predict(view, X, Xc, beta, s, s_pred, None, m_chunk=m_chunk,
                                workspace=ws)
                torch.cuda.synchronize(dev)
                ts.append(time.perf_counter() - t0)
            return sorted(ts)[reps // 2]

        counts = balanced_split(m, world, t_fact, T)
        mp = min(m, 16384)
        buf[0], buf[1] = t_fact, T(mp) / mp
        buf[2:] = torch.as_tensor(counts, dtype=F64)
    if ctx is not None and ctx.distributed:
        gdist.broadcast_(ctx, buf)
    vals = buf.cpu().tolist()
    res = ([int(round(v)) for v in vals[2:]], vals[0], vals[1])
    _SPLIT_CACHE[key] = res
    return res


# calibrate_split's results per (device, n, m, world, m_chunk): one-shot predict_sharded callers
# pay the measurement once per shape, not on every call
_SPLIT_CACHE: dict = {}


class PipelinedPredictor:
    """A stream of single-output GPs over shared (X, Xs), test points split over ranks, as a
    two-stage pipeline: ``step(params_next)`` has rank 0 factorise the next GP and broadcast its
    L^-1 (async over RCCL, into the other buffer of a double-buffered pair) while every rank
    predicts the current GP on its block; the (mean, var) blocks are gathered to rank 0.

    Usage::

        pp = PipelinedPredictor(ctx, X, Xs, w, counts=None)     # calibrates the split
        pp.start(gp0)                 # gp = (beta, s, delta, s_pred): factorise + broadcast GP 0
        for k in range(K):
            res_k = pp.step(gp_{k+1})  # predicts GP k; GP k+1 factorised meanwhile
        res_last = pp.step(None)      # drains the pipeline

    ``step`` returns GP k's (2, m) (mean, var) on rank 0 and None elsewhere.  ``w`` (n,) is the
    training output shared by the GPs (a different w per GP: pass it in the gp tuple as a fifth
    element).
    """

    def __init__(self, ctx: gdist.Context, X: torch.Tensor, Xs: torch.Tensor, w: torch.Tensor,
                 counts: list[int] | None = None, calib_gp=None, m_chunk: int = 0,
                 receiver_path: bool = False):
        self.ctx = ctx
        self.dev = X.device
        self.X = X.contiguous()
        self.n = X.shape[0]
        self.m = Xs.shape[0]
        self.w = w.reshape(1, self.n).contiguous()
        self.m_chunk = m_chunk
        # test hook: rank 0 also predicts from the broadcast payload (tile-packed L^-1 + z in
        # place), the path every other rank takes -- so a one-rank run exercises it
        self.receiver_path = receiver_path
        self.dist = ctx is not None and ctx.distributed   # collectives (also at world 1)
        world = ctx.world if self.dist else 1
        self.world, self.rank = world, (ctx.rank if self.dist else 0)
        self.t_fact = self.t_point = None
        if counts is None:
            if self.dist and (world > 1 or calib_gp is not None):
                if calib_gp is None:
                    raise ValueError("PipelinedPredictor: give counts or a calib_gp")
                b, s_, d_, sp = calib_gp[:4]
                counts, self.t_fact, self.t_point = calibrate_split(
                    ctx, self.X, Xs, b, s_, d_, sp, self.w, m_chunk=m_chunk)
            else:
                counts = [self.m]
        self.counts = counts
        lo = _offsets(counts)[self.rank]
        self.ml = counts[self.rank]
        self.Xl = Xs[lo:lo + self.ml].contiguous()
        npad = kernels.padded_n(self.n)
        self.npad = npad
        # rank 0 factorises into padded buffers; the other ranks predict from the payload
        self.linv = [torch.zeros((1, npad, npad), dtype=F64, device=self.dev)
                     for _ in range(2 if self.rank == 0 else 0)]
        self.info = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.logdet = torch.zeros(1, dtype=F64, device=self.dev)
        self.packer = LinvPacker(npad, self.dev, n=self.n)
        self.packed = [self.packer.buffer(self.dev) for _ in range(2)]
        # the first nonzero info among the GPs predicted so far (device; read by check())
        self.status = torch.zeros(1, dtype=torch.int32, device=self.dev)
        # (mean, var) of this rank's block, padded to the widest block so RCCL gathers it in
        # place into rank 0's preallocated (world, 2, mx) buffer (no per-step pad / alloc)
        self.mx = max(max(counts), 1)
        self.out = torch.zeros((2, self.mx), dtype=F64, device=self.dev)
        self.gbuf = self.glist = None
        if self.dist and ctx.backend == "nccl" and self.rank == 0:
            self.gbuf = torch.empty((world, 2, self.mx), dtype=F64, device=self.dev)
            self.glist = list(self.gbuf)
        self.ws = kernels.Workspace()
        self.pws = kernels.Workspace()
        self.k = 0
        self.gps = [None, None]
        self.pending = None
        self.stream = torch.cuda.current_stream(self.dev).cuda_stream

    def _gp(self, gp):
        b, s, d, sp = gp[:4]
        t = lambda a: torch.as_tensor(a, dtype=F64, device=self.dev)  # noqa: E731
        w = self.w if len(gp) < 5 else t(gp[4]).reshape(1, self.n).contiguous()
        return (t(b).reshape(1, -1).contiguous(), t(s).reshape(1), t(d).reshape(1),
                t(sp).reshape(1), w)

    def _factor(self, slot: int) -> None:
        """Rank 0: GP's Gram -> L, L^-1 into linv[slot] (gp_gram_ardse, gp_potrf_inv_ws)."""
        b, s, d, _, _ = self.gps[slot]
        G = kernels.gram(self.X, b, s, d)
        nbytes = int(_capi.lib().gp_potrf_inv_ws_bytes(self.n, 1))
        ws = self.pws.get(nbytes, self.dev)
        npad = self.linv[slot].shape[1]
        _capi.call("gp_potrf_inv_ws", G.data_ptr(), self.n, self.n, self.n * self.n,
                   self.linv[slot].data_ptr(), npad, npad * npad, 1, self.info.data_ptr(),
                   self.logdet.data_ptr(), ws.data_ptr(), ws.numel(), self.stream)

    def _bcast(self, slot: int):
        if self.rank == 0:
            # L^-1 tile-packed + z = L^-1 w of this GP's w + info
            self.packer.pack(self.linv[slot], self.info, self.packed[slot],
                             w=self.gps[slot][4])
        if not self.dist:
            return None
        return _wire_bcast(self.ctx, self.packed[slot], async_op=True)

    def start(self, gp) -> None:
        """Factorise and broadcast the first GP (the pipeline's prologue)."""
        self.k = 0
        self.gps[0] = self._gp(gp)
        if self.rank == 0:
            self._factor(0)
        self.pending = self._bcast(0)

    def step(self, gp_next):
        """Predict GP k (broadcast earlier) on this rank's block while rank 0 factorises and
        broadcasts ``gp_next`` (None: nothing more to factorise); gather GP k's blocks."""
        k = self.k
        cur, nxt = k % 2, (k + 1) % 2
        nxt_req = None
        if gp_next is not None:
            self.gps[nxt] = self._gp(gp_next)
            if self.rank == 0:
                self._factor(nxt)
            nxt_req = self._bcast(nxt)
        if self.pending is not None:
            self.pending.wait()
        got = self.packer.info(self.packed[cur])
        self.status.copy_(torch.where(self.status != 0, self.status, got))
        b, s, _, sp, w = self.gps[cur]
        # rank 0 predicts from its padded L^-1, every other rank from the payload in place (no
        # unpack); all of them with the shipped z (no trmv)
        ch = (kernels.Cholesky(self.n, None, self.linv[cur], self.info, self.logdet)
              if self.rank == 0 and not self.receiver_path
              else self.packer.view(self.packed[cur], self.info))
        if self.ml:
            kernels.predict(ch, self.X, self.Xl, b, s, sp, w, m_chunk=self.m_chunk,
                            workspace=self.ws, out=(self.out[0:1, : self.ml],
                                                    self.out[1:2, : self.ml]),
                            z=self.packer.z(self.packed[cur]).view(1, self.npad))
        if not self.dist:
            res = self.out[:, : self.ml]
        elif self.ctx.backend == "nccl":
            tdist.gather(self.out, gather_list=self.glist, dst=0)
            res = torch.cat([self.gbuf[r, :, :c] for r, c in enumerate(self.counts)], dim=1) \
                if self.rank == 0 else None
        else:
            res = gdist.gather_cols(self.ctx, self.out[:, : self.ml], self.counts)
        self.pending = nxt_req
        self.k = k + 1
        return res

    def finish(self, check: bool = True) -> None:
        """Wait for an outstanding broadcast (after the last ``step``); with ``check``, raise
        (on every rank alike) if any GP predicted so far had a failed factorisation: the steps
        themselves never synchronise with the host."""
        if self.pending is not None:
            self.pending.wait()
            self.pending = None
        if check:
            self.check()

    def check(self) -> None:
        """Raise for the first failed factorisation among the GPs predicted so far
        (:func:`kernels.check_info`; synchronises)."""
        kernels.check_info(self.status)
