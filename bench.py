#!/usr/bin/env python
"""bench.py — GP posterior predictions/sec, fp64, C3 (n=4096 train, m=100k test, d=8).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step is one full pass of the hot path for one GP, from hyperparameters to answers on rank 0:
ARD-SE Gram (n x n) -> blocked MFMA Cholesky + L^-1 -> cross-covariance / TRMM / mean+variance
over the test points.  Inside a step the cross-covariance (independent of the factorisation)
runs on the caller-owned context's own stream beside the latency-bound factorisation
(``--serial``: no context, every kernel in order on one stream).  Inputs are HBM-resident
before the timed region.

Multi-GPU (single-output GP): *strong scaling* of the fixed m = 100k test points
over a stream of GPs.  The headline at N > 1 is a two-stage pipeline (``c3_pipelined``): in step k
rank 0 builds GP k+1's Gram and L, L^-1 and broadcasts L^-1 (RCCL, async, tile-packed, with
z = L^-1 w, double-buffered; the other ranks predict from it in place) while every rank
predicts GP k on its block of the test points, and each step ends with one
gather of the (mean, var) blocks to rank 0 (inside the timed region).  Rank 0's block is
shortened by the factorisation's measured time, consecutive GPs have different
hyperparameters, and the last step is checked against a direct computation.  Beside it
(``unpipelined``): every rank factorises the same Gram redundantly (the Amdahl term) and
predicts ``shard_range(100000, r, N)``; and ``weak``: every rank its own 100k points.
value = 100k * K / max-over-ranks(time).

``--workload c4`` runs BASELINE config 4 instead (multivariate emulator: 32 independent PC
GPs, n = 1024, m = 100k shared test points): rank 0 broadcasts the inputs over RCCL at
setup, the PCs are dealt round-robin to ranks, each step ends with one gather of every
rank's (mean, var) rows to rank 0 (strong scaling: total work fixed).

rank 0 prints ONE JSON line with the metric, a roofline object for the dominant kernel
(trmm_pair_kernel, timed live with HIP events on its own stream via gp_profile_*), auxiliary
rooflines, and a CPU baseline (the numpy fp64 oracle on the host cores, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def _cpu_threads() -> int:
    """Host threads for the CPU baseline: the pool's CPU share when it sets OMP_NUM_THREADS
    (16 per GPU on the MI355X boxes, whose os.cpu_count() shows the whole machine), else every
    CPU this process may run on."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return len(os.sched_getaffinity(0))


_CPU_THREADS = _cpu_threads()
for _v in ("OPENBLAS_NUM_THREADS", "OMP_NUM_THREADS", "MKL_NUM_THREADS"):
    os.environ.setdefault(_v, str(_CPU_THREADS))

import numpy as np  # noqa: E402
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from gladsgp_amd import _capi, dist as gdist, kernels  # noqa: E402

METRIC = "GP posterior predictions/sec fp64, n=4096 m=100k d=8; 1→8 GPU scaling"
FP64_MFMA_PEAK_TFLOPS = 78.6    # MI355X dense FP64 matrix (spec); 70.1 measured (tools/probe_f64)
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E (spec); ~6300 achievable


def c3_inputs(n: int, m: int, d: int):
    """SURVEY §8d C3 recipe (seeded): X = rng(0), a = rng(1), beta = rng(3), X* = rng(2)."""
    X = np.random.default_rng(0).random((n, d))
    a = np.random.default_rng(1).uniform(0, 1, d)
    y = np.sin(2 * np.pi * X @ a) + 0.1 * np.sum(X * X, axis=1)
    beta = np.random.default_rng(3).uniform(0.5, 5.0, d)
    Xs = np.random.default_rng(2).random((m, d))
    return X, y, beta, Xs, 1.0, 1e-6


def c4_inputs(n: int, m: int, d: int, P: int):
    """SURVEY §8d C4 recipe: X = rng(0), beta_j = rng(10+j), w_j = rng(100+j), X* = rng(2)."""
    X = np.random.default_rng(0).random((n, d))
    beta = np.stack([np.random.default_rng(10 + j).uniform(0.5, 5.0, d) for j in range(P)])
    W = np.stack([np.random.default_rng(100 + j).standard_normal(n) for j in range(P)])
    Xs = np.random.default_rng(2).random((m, d))
    return X, W, beta, Xs, np.ones(P), np.full(P, 1e-6)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def _cpu_c3_run(X, y, beta, Xs, s, delta, sample):
    """One oracle C3 run on the host: full Gram + Cholesky + alpha, then the first ``sample``
    test points in 2000-point chunks (cross-covariance, mean, solve_triangular, variance)."""
    from oracle import gp_ref
    import scipy.linalg as sla
    t0 = time.perf_counter()
    G = gp_ref.gram_ardse(X, beta, s, delta)
    L = np.linalg.cholesky(G)
    alpha = sla.cho_solve((L, True), y)
    t_fact = time.perf_counter() - t0
    t1 = time.perf_counter()
    means, vars_ = [], []
    for a in range(0, sample, 2000):
        Ks = gp_ref.cross_ardse(Xs[a:min(sample, a + 2000)], X, beta, s)
        means.append(Ks @ alpha)
        V = sla.solve_triangular(L, Ks.T, lower=True, check_finite=False)
        vars_.append(s - np.einsum("ij,ij->j", V, V))
    return t_fact, time.perf_counter() - t1, means, vars_


def cpu_baseline(X, y, beta, Xs, s, delta, sample: int = 20000, reps: int = 3,
                 faithful_batches: int = 10):
    """numpy fp64 oracle (Gram -> cholesky -> chunked cross-cov + solve_triangular) on the
    host: full n = 4096 factorisation + prediction of the first ``sample`` test points, timed
    ``reps`` times (median), extrapolated linearly in the test points to m -- with OpenBLAS on
    the pool's CPU share (``_CPU_THREADS``) and, beside it, on one thread.  Plus the
    reference-faithful rate: ``faithful_batches`` batches of 4 test points, each re-building
    and re-factorising the Gram as assess_all_models.py:481-489 does per call."""
    from oracle import gp_ref
    import scipy.linalg as sla
    from threadpoolctl import threadpool_limits
    m = Xs.shape[0]
    sample = min(sample, m)
    runs = []
    for _ in range(reps):
        t_fact, t_pred, means, vars_ = _cpu_c3_run(X, y, beta, Xs, s, delta, sample)
        runs.append((t_fact + t_pred / sample * m, t_fact, t_pred))
    runs.sort()
    t_full, t_fact, t_pred = runs[len(runs) // 2]
    s1 = min(2000, m)
    with threadpool_limits(limits=1):
        f1, p1, _, _ = _cpu_c3_run(X, y, beta, Xs, s, delta, s1)
    t_one = f1 + p1 / s1 * m
    # "reference-faithful": re-factorise per batch of 4 points (assess_all_models.py:481-489)
    nb = max(1, min(faithful_batches, m // 4))
    tb = []
    for k in range(nb):
        t2 = time.perf_counter()
        xb = Xs[4 * k:4 * k + 4]
        G4 = gp_ref.gram_ardse(X, beta, s, delta)
        L4 = np.linalg.cholesky(G4)
        a4 = sla.cho_solve((L4, True), y)
        K4 = gp_ref.cross_ardse(xb, X, beta, s)
        _ = K4 @ a4, sla.solve_triangular(L4, K4.T, lower=True)
        tb.append(time.perf_counter() - t2)
    t4 = float(np.sum(tb))
    aff = len(os.sched_getaffinity(0))
    return {
        "value": m / t_full, "unit": "predictions/s", "cores": _CPU_THREADS, "kind": "port",
        "sample": (f"oracle/gp_ref numpy fp64, OpenBLAS {_CPU_THREADS} threads on "
                   f"{cpu_model()} (os.cpu_count()={os.cpu_count()}, affinity={aff}; the "
                   f"pool's CPU share per GPU is OMP_NUM_THREADS={_CPU_THREADS}): full "
                   f"n={X.shape[0]} Gram+Cholesky + predict of the first {sample} of {m} test "
                   f"points, median of {reps} runs (fact {t_fact:.2f} s + predict "
                   f"{t_pred:.2f} s), extrapolated linearly to m={m}"),
        "single_thread_value": m / t_one,
        "single_thread_sample": (f"the same on 1 OpenBLAS thread (threadpoolctl): fact "
                                 f"{f1:.2f} s + predict {p1:.2f} s for {s1} points, "
                                 f"extrapolated to m={m}"),
        "reference_faithful_value": 4.0 * nb / t4,
        "reference_faithful_batch_s": {"min": float(np.min(tb)), "median": float(np.median(tb)),
                                       "max": float(np.max(tb)), "batches": nb},
        "reference_faithful_sample": (f"re-factorise per batch of 4 test points as "
                                      f"assess_all_models.py:481-489 does: {nb} batches "
                                      f"({4 * nb} test points) timed, {t4:.2f} s in all, per "
                                      f"batch min {np.min(tb):.3f} / median "
                                      f"{np.median(tb):.3f} / max {np.max(tb):.3f} s, "
                                      f"{_CPU_THREADS} threads; the rate is per batch (every "
                                      "batch does one full n x n Gram + factorisation, so "
                                      "it extrapolates linearly in the batches: 400 points "
                                      "(the assess_all_models subset) = 100 batches)"),
    }, np.concatenate(means), np.concatenate(vars_)


def read_prof(pid):
    import ctypes
    cnt, tot, mx = ctypes.c_int(0), ctypes.c_double(0), ctypes.c_double(0)
    _capi.call("gp_profile_read", pid, ctypes.addressof(cnt), ctypes.addressof(tot),
               ctypes.addressof(mx))
    return cnt.value, max(tot.value, 1e-9)   # events off (GPFIT_BENCH_NOEVENTS=1): no data


def c3_pipelined(args, ctx, X, y, beta, Xs, s, delta, timed):
    """N > 1 headline: gladsgp_amd.sharded.PipelinedPredictor over a stream of GPs (SURVEY §8e:
    "rank 0 factorises and broadcasts L").  GP k has hyperparameters beta (1 + 1e-3 (k mod 2)),
    so consecutive steps are different GPs.  In step k rank 0 builds GP k+1's Gram and L, L^-1
    (the persistent factorisation) and broadcasts L^-1 over RCCL (async, its lower triangle
    packed, double-buffered), while every rank predicts GP k on its block of the 100k test
    points and the (mean, var) blocks are gathered to rank 0.  Rank 0's block is shortened by
    the factorisation's time in test-point equivalents (measured by the package's calibrate),
    so the ranks finish together.  Every step still does one full Gram + factorisation and one
    full 100k-point prediction; a GP's latency is two steps.
    Returns the timing, the split and a check of the last step against a direct single-rank
    computation of the same GP on rank 0."""
    from gladsgp_amd.sharded import PipelinedPredictor
    dev = ctx.device
    n, d = X.shape
    m = Xs.shape[0]
    Xd = torch.as_tensor(X, device=dev)
    yd = torch.as_tensor(y, device=dev).reshape(1, n)
    sd = torch.tensor([s], dtype=torch.float64, device=dev)
    dd = torch.tensor([delta], dtype=torch.float64, device=dev)
    betas = [torch.as_tensor(beta * (1.0 + 1e-3 * j), device=dev).reshape(1, d) for j in (0, 1)]
    gps = [(betas[j], sd, dd, sd) for j in (0, 1)]
    pp = PipelinedPredictor(ctx, Xd, torch.as_tensor(Xs, device=dev), yd, calib_gp=gps[0],
                            m_chunk=args.m_chunk)
    pp.start(gps[0])
    state = {"res": None}

    def pipe_step():
        state["res"] = pp.step(gps[(pp.k + 1) % 2])

    for _ in range(args.warmup):
        pipe_step()
    torch.cuda.synchronize()
    elapsed = timed(pipe_step, args.steps)
    pp.finish()
    torch.cuda.synchronize()
    check = None
    if ctx.rank == 0:
        # the last step predicted GP k_last = pp.k - 1: recompute it directly on a sample
        k_last = pp.k - 1
        ns = min(2000, m)
        G = kernels.gram(Xd, betas[k_last % 2], sd, dd)
        ch = kernels.cholesky_inverse(G)
        ch.check()
        mu, var = kernels.predict(ch, Xd, torch.as_tensor(Xs[:ns], device=dev), betas[k_last % 2],
                                  sd, sd, yd)
        res = state["res"]
        dm = float((res[0, :ns] - mu[0]).abs().max())
        dv = float((res[1, :ns] - var[0]).abs().max())
        check = {"gp": k_last, "points": ns, "max_abs_dmean": dm, "max_abs_dvar": dv}
        if not (dm <= 1e-10 * max(1.0, float(mu.abs().max())) and dv <= 1e-12):
            raise RuntimeError(f"pipelined result differs from the direct computation: {check}")
    def num(v, scale):      # one rank measures nothing (calibrate_split: the split is [m])
        return None if v is None or v != v else v * scale
    return {"elapsed": elapsed, "counts": pp.counts, "t_fact_ms": num(pp.t_fact, 1e3),
            "t_point_us": num(pp.t_point, 1e6), "check": check}


def _free_port() -> int:
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch_ranks(args) -> int | None:
    """``--gpus N`` (N > 1) run without a torch.distributed launcher (no WORLD_SIZE): start the N
    ranks as ``torch.distributed.run`` in a child process of this parent, which has touched no
    GPU (nothing here initialises HIP), and return the child's exit code.  Under a launcher (or
    N = 1) return None and run in-process."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import signal
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC for RCCL on this host
    # every rank's process group gives up on a missing peer well inside the wall limit
    env.setdefault("GPFIT_PG_TIMEOUT_S", str(max(10, min(180, int(args.wall_limit * 0.6)))))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    # a fresh child in its own process group (no exec), so a hung rank can be ended with the
    # whole group: a stalled collective leaves a JSON record and a non-zero code inside the
    # driver's limit instead of running into it
    t0 = time.perf_counter()
    child = subprocess.Popen(cmd, env=env, start_new_session=True)
    try:
        return child.wait(timeout=args.wall_limit)
    except subprocess.TimeoutExpired:
        for sig, grace in ((signal.SIGTERM, 10), (signal.SIGKILL, 10)):
            try:
                os.killpg(child.pid, sig)
            except ProcessLookupError:
                break
            try:
                child.wait(timeout=grace)
                break
            except subprocess.TimeoutExpired:
                continue
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": args.gpus,
                          "steps": args.steps, "warmup": args.warmup,
                          "error": f"ranks did not finish within --wall-limit "
                                   f"{args.wall_limit:g} s; process group killed",
                          "elapsed_s": round(time.perf_counter() - t0, 1)}), flush=True)
        return 124


def main_dry_run(args):
    """``--dry-run``: the launch / rendezvous / max-over-ranks / JSON path with no GPU work (gloo
    on the host) -- what the CPU test of ``--gpus N`` exercises."""
    ctx = gdist.init_from_env("cpu", backend="gloo")
    if ctx.world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but {ctx.world} ranks joined")
    if args.stall_rank == ctx.rank:       # testing only: a rank that never reaches the barrier
        time.sleep(3600)
    gdist.barrier(ctx)
    t0 = time.perf_counter()
    gdist.barrier(ctx)
    elapsed = gdist.max_over_ranks(ctx, time.perf_counter() - t0)
    if ctx.rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "predictions/s",
                          "n_gpus": ctx.world, "steps": 0, "warmup": 0,
                          "ms_per_step": elapsed * 1e3, "higher_is_better": True,
                          "dry_run": True}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--m", type=int, default=100000, help="test points (whole job)")
    ap.add_argument("--d", type=int, default=8)
    ap.add_argument("--m-chunk", type=int, default=0)
    ap.add_argument("--cpu-sample", type=int, default=20000,
                    help="test points the CPU baseline predicts per run (median of 3 runs)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-weak", action="store_true", help="skip the weak-scaling leg (N > 1)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="testing only: every rank on cuda:0 over gloo (host-staged collectives)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="N > 1: headline = the redundant-factorisation strong split only")
    ap.add_argument("--force-nccl", action="store_true",
                    help="join an RCCL process group even at N = 1, so every collective "
                         "branch of the N > 1 path (broadcast, gather, barrier, the pipelined "
                         "schedule) runs through a one-rank RCCL communicator")
    ap.add_argument("--cpu-faithful-batches", type=int, default=10,
                    help="reference-faithful CPU leg: batches of 4 test points timed "
                         "(assess_all_models.py:481-489 re-factorises per batch)")
    ap.add_argument("--workload", choices=("c3", "c4", "c5", "fit", "latency"), default="c3")
    ap.add_argument("--c5-ny", type=int, default=10000, help="c5: field nodes")
    ap.add_argument("--c5-pcs", type=int, default=64, help="c5: principal components")
    ap.add_argument("--c5-cpu-sample", type=int, default=3000,
                    help="c5: test points the CPU oracle predicts (all PCs) and reconstructs")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch / rendezvous / JSON path only, no GPU work (gloo on the host)")
    ap.add_argument("--wall-limit", type=float, default=540.0,
                    help="--gpus N > 1 without a launcher: seconds before the ranks' process "
                         "group is killed and a JSON error line printed (exit 124)")
    ap.add_argument("--stall-rank", type=int, default=-1,
                    help="testing only (--dry-run): this rank sleeps instead of joining the "
                         "barrier")
    ap.add_argument("--latency-points", type=int, default=20,
                    help="latency: test points timed one at a time (time_predictions.py:68)")
    ap.add_argument("--ny", type=int, default=1347945, help="fit: field size per run")
    ap.add_argument("--fit-pcs", type=int, default=8, help="fit: principal components")
    ap.add_argument("--fit-cpu-sweeps", type=int, default=4,
                    help="fit: Metropolis sweeps the CPU oracle runs (extrapolated)")
    ap.add_argument("--fit-cpu-ny-frac", type=float, default=0.1,
                    help="fit: fraction of the field's nodes the CPU oracle's PCA reads")
    ap.add_argument("--serial", action="store_true",
                    help="c3: no context; gram, potrf, cross-covariance, predict in order on "
                         "one stream")
    ap.add_argument("--cross-start", type=float, default=-1.0,
                    help="c3: gp_ctx cross_start (-1: library default)")
    ap.add_argument("--aux-free-cus", type=int, default=-1,
                    help="c3: CUs the cross-covariance stream leaves free (-1: library default)")
    ap.add_argument("--aux-chunks", type=int, default=None,
                    help="gp_ctx_set_aux_chunks: chunks whose cross-covariance runs on the aux "
                         "stream (-1: all; default: all for c3, 1 for c4)")
    ap.add_argument("--pcs", type=int, default=32, help="c4: number of PC GPs")
    ap.add_argument("--c4-path", choices=("fit_predict", "predict"), default="fit_predict",
                    help="c4: one gp_fit_predict per step with the first --aux-chunks chunks' "
                         "cross-covariance beside the batched factorisation (default; 60.08-"
                         "60.55 vs 60.67-61.13 ms/step, profiles/r04/r04d_c4_aux_chunks.log), "
                         "or gram -> potrf -> gp_predict")
    args = ap.parse_args()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    if args.dry_run:
        return main_dry_run(args)
    if args.workload == "c4":
        return main_c4(args)
    if args.workload == "c5":
        return main_c5(args)
    if args.workload == "fit":
        return main_fit(args)
    if args.workload == "latency":
        return main_latency(args)

    ctx = (gdist.init_from_env("cuda", backend="gloo", device_index=0) if args.share_gpu
           else gdist.init_from_env("cuda", force_group=args.force_nccl))
    multi = ctx.world > 1 or args.force_nccl      # the N > 1 schedule (collectives included)
    if ctx.world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but {ctx.world} ranks joined "
                         "(WORLD_SIZE); refusing to report a mislabelled number")
    dev = ctx.device
    n, m, d = args.n, args.m, args.d
    X, y, beta, Xs, s, delta = c3_inputs(n, m, d)
    lo, hi = gdist.shard_range(m, ctx.rank, ctx.world)
    counts = [gdist.shard_range(m, r, ctx.world)[1] - gdist.shard_range(m, r, ctx.world)[0]
              for r in range(ctx.world)]
    ml = hi - lo
    Xd = torch.as_tensor(X, device=dev)
    Xsd = torch.as_tensor(Xs[lo:hi], device=dev).contiguous()
    yd = torch.as_tensor(y, device=dev).reshape(1, n)
    bd = torch.as_tensor(beta, device=dev).reshape(1, d)
    sd = torch.tensor([s], dtype=torch.float64, device=dev)
    dd = torch.tensor([delta], dtype=torch.float64, device=dev)
    fctx = None if args.serial else kernels.FitPredictContext(
        dev, args.cross_start, args.aux_free_cus, -1 if args.aux_chunks is None else args.aux_chunks)
    ws = kernels.PredictWorkspace()
    out = torch.empty((2, ml), dtype=torch.float64, device=dev)   # rows: mean, var

    def step(Xs_t=Xsd, o=out):
        return kernels.fit_predict(Xd, Xs_t, bd, sd, dd, sd, yd, m_chunk=args.m_chunk,
                                   workspace=ws, out=(o[0:1], o[1:2]), ctx=fctx, check=False)[2]

    def timed(fn, steps):
        gdist.barrier(ctx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        gdist.barrier(ctx)
        return gdist.max_over_ranks(ctx, time.perf_counter() - t0)

    from gladsgp_amd import sharded
    Xs_all = torch.as_tensor(Xs, device=dev)
    gathered = [None]

    def strong_step(check=False):
        # package API (SURVEY §8e single-output GP): rank r predicts its block of the m points
        # with gp_fit_predict (redundant factorisation) and the blocks are gathered to rank 0
        gathered[0] = sharded.predict_sharded(ctx, Xd, Xs_all, bd, sd, dd, sd, yd,
                                              mode="redundant", counts=counts,
                                              m_chunk=args.m_chunk, fctx=fctx, workspace=ws,
                                              check=check)

    for i in range(args.warmup):
        strong_step(check=(i == 0))      # the first warmup step checks info (syncs)
    torch.cuda.synchronize()
    events = os.environ.get("GPFIT_BENCH_NOEVENTS") != "1"
    if events:
        _capi.call("gp_profile_enable", 64 * (args.steps + 1))
    # the timed region records only the dominant kernel's events (one pair around a step's
    # TRMM launches): the Gram / factorisation / cross-covariance pairs would sit on the
    # critical path of every step; they are read from two untimed steps after it
    select = getattr(_capi.lib(), "gp_profile_select", lambda mask: 0)   # (older builds: A/B)
    select(1 << _capi.PROF_TRMM)
    _capi.call("gp_profile_reset")
    elapsed = timed(strong_step, args.steps)
    prof = {"trmm": read_prof(_capi.PROF_TRMM)}
    select(0xFFFFFFFF)
    aux_steps = 2
    _capi.call("gp_profile_reset")
    for _ in range(aux_steps):
        strong_step()
    torch.cuda.synchronize()
    prof.update({k: read_prof(v) for k, v in (("gram", _capi.PROF_GRAM),
                                              ("potrf", _capi.PROF_POTRF),
                                              ("cross", _capi.PROF_CROSS))})
    _capi.call("gp_profile_enable", 0)

    weak = None
    if ctx.world > 1 and not args.no_weak:
        # weak scaling: rank r predicts its own 100k points (rows [r m, (r+1) m) of rng(2)'s
        # stream), no collective inside a step
        Xw = np.random.default_rng(2).random(((ctx.rank + 1) * m, d))[ctx.rank * m:]
        Xwd = torch.as_tensor(Xw, device=dev).contiguous()
        ow = torch.empty((2, m), dtype=torch.float64, device=dev)
        for _ in range(args.warmup):
            step(Xwd, ow)
        t_w = timed(lambda: step(Xwd, ow), args.steps)
        weak = {"value": ctx.world * m * args.steps / t_w, "unit": "predictions/s",
                "ms_per_step": t_w / args.steps * 1e3, "m_test_per_gpu": m,
                "note": "every rank predicts its own 100k points (redundant factorisation, "
                        "no collective)"}
        del Xwd, ow

    res = None if gathered[0] is None else torch.stack(gathered[0])   # (2, m) on rank 0
    if fctx is not None:
        fctx.close()
    pipe = None
    if multi and not args.no_pipeline:
        pipe = c3_pipelined(args, ctx, X, y, beta, Xs, s, delta, timed)
    if ctx.rank != 0:
        return
    K = args.steps
    value = m * K / elapsed
    # algorithmic work: trmm n^2 + mean/var 4n flop per prediction
    tr_cnt, tr_ms = prof["trmm"]
    tr_flops = float(ml) * K * (n * n + 4 * n)
    tr_tfs = tr_flops / (tr_ms * 1e-3) / 1e12
    traffic, traffic_src = None, None
    chunk = args.m_chunk or 16384   # the library's default test-point chunk for one GP
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        tf = os.path.join(ROOT, "profiles", rnd, "pmc_traffic.json")
        tj = json.load(open(tf)) if os.path.exists(tf) else {}
        if tj and n == 4096 and chunk == tj.get("m_chunk") and ml == tj.get("m", 100000):
            traffic = tj["kernels"]["trmm_pair_kernel"]["bytes_per_launch"]
            traffic_src = (f"profiles/{rnd}/pmc_traffic.json (FETCH_SIZE x2 + WRITE_SIZE, per "
                           "launch)")
            break
    roof = {"kernel": "trmm_pair_kernel", "bound": "mfma", "achieved": round(tr_tfs, 3),
            "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tr_tfs / FP64_MFMA_PEAK_TFLOPS, 4),
            "traffic": traffic, "traffic_source": traffic_src, "launches": tr_cnt,
            "avg_launch_ms": round(tr_ms / max(tr_cnt, 1), 4),
            "flop_per_launch": tr_flops / max(tr_cnt, 1),
            "work_note": "n^2 + 4n flop per prediction (lower-triangular L^-1 K*^T + mean/var), "
                         "rank 0's test points"}
    g_cnt, g_ms = prof["gram"]
    g_bytes = (4.0 * n * (n + 1) + 8.0 * n * d) * g_cnt   # lower triangle written + X read
    p_cnt, p_ms = prof["potrf"]
    p_flops = 2.0 * n ** 3 / 3.0 * p_cnt
    c_cnt, c_ms = prof["cross"]
    npad = kernels.padded_n(n)
    c_bytes = 8.0 * npad * ml * aux_steps
    aux = {
        "gram": {"bound": "hbm", "achieved": round(g_bytes / (g_ms * 1e-3) / 1e9, 1),
                 "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(g_bytes / (g_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                 "avg_launch_ms": round(g_ms / max(g_cnt, 1), 4),
                 "work_note": "4n(n+1) B written (lower triangle) + 8nd B read per launch"},
        "potrf_inv": {"bound": "mfma", "achieved": round(p_flops / (p_ms * 1e-3) / 1e12, 3),
                      "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                      "frac": round(p_flops / (p_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
                      "avg_call_ms": round(p_ms / max(p_cnt, 1), 4),
                      "work_note": "potrf n^3/3 + triangular inverse n^3/3"},
        "cross": {"bound": "hbm", "achieved": round(c_bytes / (c_ms * 1e-3) / 1e9, 1),
                  "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": round(c_bytes / (c_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                  "ms_per_step": round(c_ms / aux_steps, 4),
                  "work_note": "8 B written per (padded train row, test point)"},
        "trmm_ms_per_step": round(tr_ms / K, 4),
        "note": "gram / potrf_inv / cross timed over two untimed steps after the timed region "
                "(their event pairs would sit on every step's critical path); the TRMM's over "
                "the timed region",
    }
    line = {
        "metric": METRIC, "value": value, "unit": "predictions/s", "n_gpus": ctx.world,
        "steps": K, "warmup": args.warmup, "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (SURVEY §8d C3 recipe: seeded uniform design, sin target)",
        "config": {"workload": "C3 single-output ARD-SE GP: Gram + Cholesky/L^-1 + predict",
                   "n_train": n, "m_test": m, "d": d, "m_test_rank0": ml,
                   "parallelism": (f"strong: m/{ctx.world} test-point blocks per rank, "
                                   "redundant factorisation, (mean, var) gathered to rank 0 "
                                   "every step" if multi else "1 GPU"),
                   "pipeline": ("serial (one stream)" if args.serial else
                                "gp_fit_predict on a gp_ctx (cross-covariance on the "
                                "context's aux stream, no CU mask, beside the "
                                "factorisation)"),
                   "collectives": (f"{ctx.backend} process group of {ctx.world}"
                                   + (" (--force-nccl: one-rank RCCL rehearsal of the N > 1 "
                                      "path)" if args.force_nccl and ctx.world == 1 else "")
                                   if ctx.distributed else "none (single process)")},
        "roofline": roof, "roofline_aux": aux, "weak": weak, "cpu_baseline": None,
    }
    if res is None or tuple(res.shape) != (2, m):
        raise RuntimeError(f"gathered result has shape {None if res is None else res.shape}")
    if pipe is not None:
        # the pipelined schedule is the headline at N > 1; the redundant-factorisation strong
        # split stays beside it
        line["unpipelined"] = {"value": value, "unit": "predictions/s",
                               "ms_per_step": elapsed / K * 1e3,
                               "parallelism": line["config"]["parallelism"]}
        line["value"] = m * K / pipe["elapsed"]
        line["ms_per_step"] = pipe["elapsed"] / K * 1e3
        line["config"]["parallelism"] = (
            f"pipelined x{ctx.world}: rank 0 builds GP k+1's Gram + L, L^-1 and broadcasts L^-1 "
            "(RCCL, async, tile-packed with z = L^-1 w, double-buffered) while every rank "
            "predicts GP k on its test-point block (ranks >= 1 straight from the payload) and "
            "the blocks are gathered to rank 0; rank 0's block shortened by the "
            "factorisation's time")
        line["config"]["m_test_per_rank"] = pipe["counts"]
        line["config"]["m_test_rank0"] = pipe["counts"][0]
        line["config"]["pipeline"] = ("per rank: gp_predict_ex (cross-covariance, TRMM, "
                                      "mean/var) from the broadcast tile-packed L^-1 and z; "
                                      "rank 0 also gp_gram_ardse + gp_potrf_inv + gp_pack_linv "
                                      "+ gp_predict_z of the next GP, first")
        line["pipeline"] = {"t_fact_ms": pipe["t_fact_ms"], "t_point_us": pipe["t_point_us"],
                            "check_last_step_vs_direct": pipe["check"]}
    if ctx.world == 1 and not args.no_cpu:
        cb, mu_ref, var_ref = cpu_baseline(X, y, beta, Xs, s, delta, args.cpu_sample,
                                           faithful_batches=args.cpu_faithful_batches)
        k = mu_ref.shape[0]
        mu_g = res[0, :k].cpu().numpy()
        var_g = res[1, :k].cpu().numpy()
        cb["parity_vs_gpu"] = {"points": int(k),
                               "max_abs_dmean": float(np.max(np.abs(mu_g - mu_ref))),
                               "max_abs_dvar": float(np.max(np.abs(var_g - var_ref)))}
        line["cpu_baseline"] = cb
    print(json.dumps(line), flush=True)


C4_DEFAULT_CHUNK = 8192   # the library's default test-point chunk for a batch (predict.hip)


def main_c4(args):
    from gladsgp_amd.emulator import assemble_units
    ctx = gdist.init_from_env("cuda", force_group=args.force_nccl)
    dev = ctx.device
    n = args.n if args.n != 4096 else 1024
    m, d, P = args.m, args.d, args.pcs
    # rank 0 owns the inputs; one RCCL broadcast of each at setup (outside the timed region)
    if ctx.rank == 0:
        X, W, beta, Xs, s, delta = c4_inputs(n, m, d, P)
        host = [X, W, beta, Xs, s, delta]
        bufs = [torch.as_tensor(a, dtype=torch.float64, device=dev).contiguous() for a in host]
    else:
        shapes = [(n, d), (P, n), (P, d), (m, d), (P,), (P,)]
        bufs = [torch.empty(sh, dtype=torch.float64, device=dev) for sh in shapes]
    for b in bufs:
        gdist.broadcast_(ctx, b)
    Xd, Wd, Bd, Xsd, Sd, Dd = bufs
    mine = gdist.shard_units(P, ctx.rank, ctx.world)
    idx = torch.as_tensor(mine, dtype=torch.long, device=dev)
    Wl, Bl, Sl, Dl = (t[idx].contiguous() for t in (Wd, Bd, Sd, Dd))
    bl = len(mine)
    ws = kernels.PredictWorkspace()
    mean = torch.empty((bl, m), dtype=torch.float64, device=dev)
    var = torch.empty((bl, m), dtype=torch.float64, device=dev)
    # 1: 57.85-57.97 ms/step vs 58.03-58.14 for 0, 57.99-58.18 for 2, 58.18-58.32 for 3 and
    # 58.34-58.43 for 4, three interleaved rounds on one box (profiles/r05/r05_c4_aux.log; round
    # 4's library, whose factorisation hopped streams, preferred 4: r04j_c4aux.log)
    aux_chunks = 1 if args.aux_chunks is None else args.aux_chunks
    fctx = kernels.FitPredictContext(dev, args.cross_start, args.aux_free_cus,
                                     aux_chunks) if args.c4_path == "fit_predict" else None

    def step():
        if bl and args.c4_path == "fit_predict":
            # one gp_fit_predict over this rank's PCs: the cross-covariance of every chunk runs
            # on the context's stream under the batched factorisation
            kernels.fit_predict(Xd, Xsd, Bl, Sl, Dl, Sl, Wl, m_chunk=args.m_chunk, workspace=ws,
                                out=(mean, var), ctx=fctx, check=False)
        elif bl:
            G = kernels.gram(Xd, Bl, Sl, Dl, batch=bl)
            ch = kernels.cholesky_inverse(G)
            kernels.predict(ch, Xd, Xsd, Bl, Sl, Sl, Wl, m_chunk=args.m_chunk, workspace=ws,
                            out=(mean, var))
        return assemble_units(ctx, mean, var, P)

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    _capi.call("gp_profile_enable", 64 * (args.steps + 1) * max(1, bl))
    _capi.call("gp_profile_reset")
    gdist.barrier(ctx)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    gdist.barrier(ctx)
    elapsed = gdist.max_over_ranks(ctx, time.perf_counter() - t0)
    tr_cnt, tr_ms = read_prof(_capi.PROF_TRMM)
    p_cnt, p_ms = read_prof(_capi.PROF_POTRF)
    _capi.call("gp_profile_enable", 0)
    if fctx is not None:
        fctx.close()
    if ctx.rank != 0:
        return
    K = args.steps
    value = P * m * K / elapsed
    tr_flops = float(bl) * m * K * (n * n + 4 * n)
    traffic, traffic_src = None, None
    for rnd in ("r06", "r05", "r04", "r03"):
        tf = os.path.join(ROOT, "profiles", rnd, "pmc_traffic_c4.json")
        if not (os.path.exists(tf) and ctx.world == 1):
            continue
        tj = json.load(open(tf))
        if (tj.get("n") == n and tj.get("batch") == P and tj.get("m") == m and
                tj.get("m_chunk") == (args.m_chunk or C4_DEFAULT_CHUNK)):
            traffic = tj["kernels"]["trmm_pair_kernel"]["bytes_per_launch"]
            traffic_src = (f"profiles/{rnd}/pmc_traffic_c4.json (FETCH_SIZE x2 + WRITE_SIZE, "
                           "per launch)")
            break
    tr_tfs = tr_flops / (tr_ms * 1e-3) / 1e12 if tr_ms > 0 else 0.0
    line = {
        "metric": "GP posterior predictions/sec fp64, multivariate emulator (C4: 32 PC GPs, "
                  "n=1024, m=100k, d=8)",
        "value": value, "unit": "predictions/s", "n_gpus": ctx.world, "steps": K,
        "warmup": args.warmup, "ms_per_step": elapsed / K * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (SURVEY §8d C4 recipe, seeded; inputs broadcast from rank 0)",
        "config": {"workload": "C4 multivariate emulator: per-PC Gram + Cholesky/L^-1 + "
                               "predict, gather to rank 0",
                   "pcs": P, "n_train": n, "m_test": m, "d": d,
                   "parallelism": f"PC shards x{ctx.world} (RCCL broadcast + gather)",
                   "collectives": (f"{ctx.backend} process group of {ctx.world}"
                                   if ctx.distributed else "none (single process)"),
                   "path": args.c4_path,
                   "aux_chunks": aux_chunks if args.c4_path == "fit_predict" else None},
        "roofline": {"kernel": "trmm_pair_kernel (rank 0's PCs)", "bound": "mfma",
                     "achieved": round(tr_tfs, 3), "peak": FP64_MFMA_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(tr_tfs / FP64_MFMA_PEAK_TFLOPS, 4),
                     "traffic": traffic, "traffic_source": traffic_src, "launches": tr_cnt,
                     "avg_launch_ms": round(tr_ms / max(tr_cnt, 1), 4),
                     "flop_per_launch": tr_flops / max(tr_cnt, 1)},
        "roofline_aux": {"potrf_inv_ms_per_step": round(p_ms / K, 4)},
        "cpu_baseline": None,
    }
    assert out is not None and out[0].shape == (P, m)
    if ctx.world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_c4(X, W, beta, Xs, s, delta, out)
    print(json.dumps(line), flush=True)


def cpu_baseline_c4(X, W, beta, Xs, s, delta, out, pcs: int = 2, sample: int = 2000):
    """The numpy fp64 oracle on the host for C4: ``pcs`` of the PC GPs, each a full n = 1024
    Gram + Cholesky + alpha and the first ``sample`` test points (gp_ref's chunked
    cross-covariance / solve_triangular), extrapolated linearly in the points to m and in the
    PCs to P (the PCs are independent problems of one shape); the GPU's answers for those
    points are checked against it."""
    P, m = W.shape[0], Xs.shape[0]
    per_pc, dm, dv = [], 0.0, 0.0
    for j in range(pcs):
        t_fact, t_pred, means, vars_ = _cpu_c3_run(X, W[j], beta[j], Xs, float(s[j]),
                                                   float(delta[j]), sample)
        per_pc.append(t_fact + t_pred / sample * m)
        mu_g = out[0][j, :sample].cpu().numpy()
        var_g = out[1][j, :sample].cpu().numpy()
        dm = max(dm, float(np.max(np.abs(mu_g - np.concatenate(means)))))
        dv = max(dv, float(np.max(np.abs(var_g - np.concatenate(vars_)))))
    t_all = float(np.mean(per_pc)) * P
    return {"value": P * m / t_all, "unit": "predictions/s", "cores": _CPU_THREADS,
            "kind": "port",
            "sample": (f"oracle/gp_ref numpy fp64, OpenBLAS {_CPU_THREADS} threads on "
                       f"{cpu_model()}: {pcs} of the {P} PC GPs, each the full n={X.shape[0]} "
                       f"Gram + Cholesky + predict of the first {sample} of {m} test points "
                       f"({', '.join(f'{t:.2f}' for t in per_pc)} s per PC extrapolated to "
                       f"m), extrapolated to {P} PCs"),
            "parity_vs_gpu": {"pcs": pcs, "points": sample, "max_abs_dmean": dm,
                              "max_abs_dvar": dv}}


def synthetic_field(n: int, d: int, ny: int, seed: int = 0):
    """A smooth low-rank float32 ensemble of the reference's shape (n runs x ny nodes; the
    reference stores Y_physical as (ny, n), time_predictions.py:39): 12 space modes with
    decaying weight, seeded, plus 1e-3 noise."""
    rng = np.random.default_rng(seed)
    t = rng.random((n, d))
    nm = 12
    modes = (rng.standard_normal((nm, ny)) * (0.6 ** np.arange(nm))[:, None]).astype(np.float32)
    coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, d) + k) for k in range(nm)], 1)
    Y = coef.astype(np.float32) @ modes
    Y += 1e-3 * rng.standard_normal(Y.shape, dtype=np.float32)
    return t, Y


def synthetic_samples(d: int, P: int, N: int = 512, seed: int = 5) -> dict:
    """A posterior-sample dict in SEPIA's layout (betaU (N, (d+1) P), lamUz/lamWs (N, P), lamWOs
    (N, 1)) drawn around GPMSA-typical values (prediction timing needs samples, not a fit)."""
    rng = np.random.default_rng(seed)
    return {"betaU": rng.uniform(0.2, 3.0, (N, (d + 1) * P)),
            "lamUz": rng.uniform(0.5, 3.0, (N, P)),
            "lamWs": rng.uniform(200, 3000, (N, P)),
            "lamWOs": rng.uniform(50, 500, (N, 1))}


def main_latency(args):
    """The reference's own prediction-timing harness, time_predictions.py:53,68-101, at its
    configuration: m = 256 training runs (train_config.py:9), p = 8 PCs (train_config.py:75),
    32 posterior samples (``get_samples(numsamples=32, nburn=256)``, cast to float32), one test
    point per call, a 1,347,945-node field.  Per test point, timed exactly as the harness does:
        preds = SepiaEmulatorPrediction(samples=, model=, t_pred=xi)   (here EmulatorPrediction)
        preds.w = preds.w.astype(float32); emulator_preds = preds.get_y()      -> emulator
        error_preds[j] = sd_y * N(0, 1/sqrt(lamWOs_j)) (host numpy); y = emulator + error
                                                                                 -> full
    plus the device-side alternative get_y(add_error=True) beside it.  Seconds per prediction
    (lower is better); the CPU baseline runs the oracle's restatement of the same per-point
    work (S x P GP solves at n = 256 + the float32 field reconstruction) on the host."""
    import shutil
    import tempfile
    from gladsgp_amd import model as gmodel
    from gladsgp_amd.emulator import EmulatorPrediction
    dev = torch.device("cuda", 0)
    n, d, P, S, ny = 256, 8, 8, 32, args.ny
    t, Y = synthetic_field(n, d, ny)
    tmp = tempfile.mkdtemp(prefix="gladsgp_lat_")
    try:
        np.random.seed(0)
        data, model = gmodel.init_model(t.astype(np.float32), Y, "lat", P, data_dir=tmp,
                                        device=dev, verbose=False)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    model.set_samples(synthetic_samples(d, P))
    samples = model.get_samples(numsamples=32, nburn=256)           # time_predictions.py:53
    for key in samples.keys():
        samples[key] = samples[key].astype(np.float32)
    sd_y = data.sim_data.y_sd.cpu().numpy().astype(np.float32)   # time_predictions.py:65-66
    t_test = np.random.default_rng(9).random((args.latency_points + args.warmup, d)).astype(
        np.float32)
    dt_em, dt_err, dt_y, dt_dev = [], [], [], []
    for i in range(t_test.shape[0]):
        xi = t_test[i:i + 1]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        preds = EmulatorPrediction(samples=samples, model=model, t_pred=xi)
        preds.w = preds.w.astype(np.float32)
        emulator_preds = preds.get_y()
        t1 = time.perf_counter()
        error_preds = np.zeros(emulator_preds.shape, dtype=np.float32)
        for j in range(error_preds.shape[0]):
            error_preds[j] = sd_y * np.random.normal(
                scale=1 / np.sqrt(samples["lamWOs"][j])).astype(np.float32)
        y_preds = emulator_preds + error_preds
        t2 = time.perf_counter()
        # the device-side error term (one scalar per sample, time_predictions.py:84-87 form)
        t3 = time.perf_counter()
        preds2 = EmulatorPrediction(samples=samples, model=model, t_pred=xi)
        preds2.w = preds2.w.astype(np.float32)
        y_dev = preds2.get_y(add_error=True, per_point=False)
        t4 = time.perf_counter()
        if i >= args.warmup:
            dt_em.append(t1 - t0)
            dt_err.append(t2 - t1)
            dt_y.append(t2 - t0)
            dt_dev.append(t4 - t3)
    assert y_preds.shape == (S, 1, ny) and y_dev.shape == (S, 1, ny)
    assert y_preds.dtype == np.float32 and np.all(np.isfinite(y_preds))
    value = float(np.mean(dt_y))
    out_mb = S * ny * 4 / 1e6
    line = {
        "metric": "GladsGP prediction latency (time_predictions.py harness): seconds per "
                  "prediction, n=256 p=8 S=32 ny=1,347,945, one test point per call",
        "value": value, "unit": "s", "n_gpus": 1, "steps": len(dt_y), "warmup": args.warmup,
        "ms_per_step": value * 1e3, "higher_is_better": False, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64 (GP), f32 (field, as the reference casts)",
        "data": "synthetic low-rank float32 field of the reference's shape, synthetic "
                "posterior samples (GPMSA-typical ranges), seeded",
        "config": {"workload": "time_predictions.py: EmulatorPrediction -> .w float32 cast -> "
                               "get_y() -> host error term", "n_train": n, "pcs": P,
                   "samples": S, "ny": ny, "points": len(dt_y)},
        "breakdown": {"emulator_s": float(np.mean(dt_em)), "error_s": float(np.mean(dt_err)),
                      "full_s": value, "full_device_error_s": float(np.mean(dt_dev)),
                      "field_MB_per_prediction": out_mb,
                      "note": "emulator = SEPIA-equivalent prediction + get_y (incl. the "
                              "device-to-host copy of the float32 field, as the reference "
                              "returns numpy); error = the harness's own host numpy loop"},
        "roofline": None, "cpu_baseline": None,
    }
    if not args.no_cpu:
        line["cpu_baseline"] = cpu_latency_baseline(data, model, samples, t_test[0:1], sd_y)
    print(json.dumps(line), flush=True)


def cpu_latency_baseline(data, model, samples, xi, sd_y, reps: int = 3):
    """The oracle's restatement of one time_predictions.py iteration on the host: the S x P
    GP solves at n = 256 (Gram, Cholesky, mean / variance at one point: gp_ref.sepia_predict_w)
    + the float32 field reconstruction y = (w K) sd + mu and the harness's error term.  Median
    of ``reps``; the reference re-factorises per call exactly like this."""
    from oracle import gp_ref
    t = data.sim_data.t_dev.cpu().numpy()
    w_hat = model.w_hat.cpu().numpy()
    lam = model.LamSim.cpu().numpy()
    K = data.sim_data.K.cpu().numpy().astype(np.float32)
    mu = data.sim_data.y_mean.cpu().numpy().astype(np.float32)
    sd = data.sim_data.y_sd.cpu().numpy().astype(np.float32)
    runs = []
    for _ in range(reps):
        t0 = time.perf_counter()
        w, _ = gp_ref.sepia_predict_w(t, xi.astype(np.float64), w_hat, samples, lam)
        w = w.astype(np.float32)
        y = (np.einsum("smp,py->smy", w, K) * sd + mu).astype(np.float32)
        e = np.zeros(y.shape, dtype=np.float32)
        for j in range(y.shape[0]):
            e[j] = sd_y * np.random.normal(scale=1 / np.sqrt(samples["lamWOs"][j])).astype(
                np.float32)
        _ = y + e
        runs.append(time.perf_counter() - t0)
    runs.sort()
    v = runs[len(runs) // 2]
    return {"value": v, "unit": "s", "cores": _CPU_THREADS, "kind": "port",
            "sample": (f"oracle/gp_ref numpy (fp64 GP solves, float32 field), OpenBLAS "
                       f"{_CPU_THREADS} threads on {cpu_model()}: one time_predictions.py "
                       f"iteration (S x P = {w_hat.shape[1] * len(samples['lamUz'])} GPs at "
                       f"n = {t.shape[0]}, field of {K.shape[1]} nodes), median of {reps}")}


def prediction_kernel(n):
    """The prediction kernel gp_fit_predict runs for an n-point design (predict.hip:
    res_eligible): column-resident with the cross-covariance fused in at npad <= 512."""
    from gladsgp_amd import kernels
    if kernels.padded_n(n) <= 512 and os.environ.get("GPFIT_TRMM_RES", "1") != "0":
        return "trmm_res_kernel (column-resident, cross-covariance fused)"
    return "trmm_pair_kernel (the PC GPs' TRMM)"


def main_c5(args):
    """BASELINE config 5: the synthetic GlaDS ensemble through the whole chained
    surface, one step = gladsgp_amd.pipeline.FieldPipeline.run():
      standardise the 512 x 10k float32 field (src/model.py:60-72) -> randomized_svd(Y_std, 64,
      k=0, q=1) (plot_PC_RMSE.py:90-91) -> K = diag(S) Vh / sqrt(n), w_hat, LamSim
      (src/model.py:101, 219) -> the 64 PC GPs at m = 100k test points, mean + variance
      (SepiaEmulatorPrediction, assess_all_models.py:487-489) -> preds.w float32,
      get_y() = the 100k x 10k field on the device (assess_all_models.py:490-492).
    value = S x P x m posterior predictions per step / step time (every step redoes every
    phase from the raw field).  N > 1: inputs broadcast once at setup, every rank runs the
    cheap SVD / basis redundantly, the PC GPs are dealt round-robin with one gather of (mean,
    var) to rank 0, and the field is reconstructed in ny-column blocks after one broadcast of w
    (each rank keeps its block)."""
    from gladsgp_amd.pipeline import FieldPipeline, synthetic_c5
    ctx = gdist.init_from_env("cuda", force_group=args.force_nccl)
    if ctx.world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but {ctx.world} ranks joined")
    dev = ctx.device
    n, d, ny, m, P = 512, args.d, args.c5_ny, args.m, args.c5_pcs
    if ctx.rank == 0:
        t, Y, omega, smp, t_pred = synthetic_c5(n, d, ny, m, P)
        host = [t, Y, omega, t_pred] + [smp[k] for k in ("betaU", "lamUz", "lamWs", "lamWOs")]
        bufs = [torch.as_tensor(np.ascontiguousarray(a), device=dev) for a in host]
    else:
        shapes = [((n, d), torch.float64), ((n, ny), torch.float32), ((ny, P), torch.float32),
                  ((m, d), torch.float64), ((1, (d + 1) * P), torch.float64),
                  ((1, P), torch.float64), ((1, P), torch.float64), ((1, 1), torch.float64)]
        bufs = [torch.empty(sh, dtype=dt, device=dev) for sh, dt in shapes]
    for b in bufs:                                   # one broadcast per input, at setup
        gdist.broadcast_(ctx, b)
    t_d, Y_d, om_d, tp_d = bufs[:4]
    smp = {k: v.cpu().numpy() for k, v in zip(("betaU", "lamUz", "lamWs", "lamWOs"), bufs[4:])}
    S = smp["lamUz"].shape[0]
    pipe = FieldPipeline(t_d, Y_d, om_d, smp, tp_d, P, device=dev,
                         ctx=ctx if ctx.distributed else None, m_chunk=args.m_chunk,
                         aux_chunks=1 if args.aux_chunks is None else args.aux_chunks)
    res = None
    for _ in range(args.warmup):
        res = pipe.run()
    torch.cuda.synchronize()
    _capi.call("gp_profile_enable", 64 * (args.steps + 1) * P)
    select = getattr(_capi.lib(), "gp_profile_select", lambda mask: 0)
    select(1 << _capi.PROF_TRMM)
    _capi.call("gp_profile_reset")
    gdist.barrier(ctx)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = pipe.run()
    torch.cuda.synchronize()
    gdist.barrier(ctx)
    elapsed = gdist.max_over_ranks(ctx, time.perf_counter() - t0)
    tr_cnt, tr_ms = read_prof(_capi.PROF_TRMM)
    select(0xFFFFFFFF)
    _capi.call("gp_profile_enable", 0)
    # per-phase device times: events on the pipeline's stream over two untimed steps after the
    # timed region (event pairs inside it would add their own waits)
    phase_steps = 2
    ph = {}
    for _ in range(phase_steps):
        pipe.events = []
        res = pipe.run()
        torch.cuda.synchronize()
        evs = pipe.events
        for (a, ea), (b, eb) in zip(evs[:-1], evs[1:]):
            ph[b] = ph.get(b, 0.0) + ea.elapsed_time(eb) / phase_steps
    pipe.events = None
    if ctx.rank != 0:
        pipe.close()
        return
    K = args.steps
    preds = S * P * m
    value = preds * K / elapsed
    bl = len(gdist.shard_units(S * P, 0, ctx.world))
    tr_flops = float(bl) * m * K * (n * n + 4 * n)
    tr_tfs = tr_flops / (tr_ms * 1e-3) / 1e12 if tr_ms > 0 else 0.0
    y = res["y"]
    ny_r = y.shape[-1]
    svd_bytes = 4.0 * n * ny * 8 + ny * P * 4          # y_std read by the 4 ensemble products
    svd_s = ph["svd"] * 1e-3
    fy_s = ph["get_y"] * 1e-3
    fy_flop = 2.0 * S * m * ny_r * P
    fy_bytes = S * m * ny_r * y.element_size() + S * m * P * 8 + P * ny_r * 8
    pr_s = ph["predict"] * 1e-3
    c5_traffic = (None, None)
    tf = os.path.join(ROOT, "profiles", "r06", "pmc_traffic_c5.json")
    tj = json.load(open(tf)) if os.path.exists(tf) else {}
    kt = tj.get("kernels", {}).get(prediction_kernel(n).split("<")[0].split(" ")[0], {})
    if kt and (tj.get("n"), tj.get("batch"), tj.get("m")) == (n, P, m):
        c5_traffic = (kt["bytes_per_launch"],
                      "profiles/r06/pmc_traffic_c5.json (FETCH_SIZE x2 + WRITE_SIZE, per launch; "
                      f"algorithmic {kt['algorithmic_bytes_per_launch']:.4g} B)")
    line = {
        "metric": "GP posterior predictions/sec fp64, C5 synthetic GlaDS ensemble (n=512 d=8, "
                  f"{ny}-node field, {P} PCs via randomized_svd, m={m}, field reconstructed)",
        "value": value, "unit": "predictions/s", "n_gpus": ctx.world, "steps": K,
        "warmup": args.warmup, "ms_per_step": elapsed / K * 1e3, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None,
        "dtype": "f64 (SVD, GP); field stored f32 after the reference's .w.astype(float32)",
        "data": "synthetic (SURVEY §8d C5: the reference's Sobol 512x8 design, seeded smooth "
                "96-mode float32 field + 1e-3 noise, Omega drawn as src/svd.py:51 after "
                "np.random.seed(0), GPMSA-typical hyperparameters, X* = rng(2))",
        "config": {"workload": "C5: standardise -> randomized_svd(Y_std, 64, k=0, q=1) -> K, "
                               "w_hat -> 64 PC GPs at m test points (mean + var) -> preds.w "
                               "float32 -> get_y() field on the device",
                   "n_train": n, "d": d, "ny": ny, "pcs": P, "samples": S, "m_test": m,
                   "field_shape": [S, m, ny],
                   "parallelism": (f"PC shards x{ctx.world} (units round-robin, gather of "
                                   "(mean, var) to rank 0) + ny-column field blocks after a "
                                   "broadcast of w; SVD / basis redundant per rank"
                                   if ctx.distributed else "1 GPU"),
                   "collectives": (f"{ctx.backend} process group of {ctx.world}"
                                   if ctx.distributed else "none (single process)")},
        "phases_ms": {k: round(v, 4) for k, v in ph.items()},
        "roofline": {"kernel": prediction_kernel(n), "bound": "mfma",
                     "achieved": round(tr_tfs, 3), "peak": FP64_MFMA_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(tr_tfs / FP64_MFMA_PEAK_TFLOPS, 4),
                     "traffic": c5_traffic[0], "traffic_source": c5_traffic[1],
                     "launches": tr_cnt,
                     "avg_launch_ms": round(tr_ms / max(tr_cnt, 1), 4),
                     "flop_per_launch": tr_flops / max(tr_cnt, 1),
                     "work_note": "n^2 + 4n flop per prediction (the fused kernel also "
                                  "produces the cross-covariance: its exp work is not counted)"},
        "roofline_phases": {
            "svd": {"bound": "hbm", "achieved": round(svd_bytes / svd_s / 1e9, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(svd_bytes / svd_s / 1e9 / HBM_PEAK_GBS, 4),
                    "ms": round(ph["svd"], 4),
                    "work_note": "4 reads of the fp64 y_std (X Omega, Y^T X, X Z, Q^T X) + "
                                 "Omega; the phase also holds CholeskyQR3, the Jacobi "
                                 "eigensolver and their host checks (latency at this size)"},
            "predict": {"bound": "mfma",
                        "achieved": round(float(bl) * m * (n * n + 4 * n) / pr_s / 1e12, 3),
                        "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": round(float(bl) * m * (n * n + 4 * n) / pr_s / 1e12
                                      / FP64_MFMA_PEAK_TFLOPS, 4),
                        "ms": round(ph["predict"], 4),
                        "work_note": "whole EmulatorPrediction phase (Gram, factorisation, "
                                     "cross-covariance, TRMM, finalize, gather) at the TRMM's "
                                     "n^2 + 4n flop per prediction"},
            "get_y": {"bound": "mfma", "achieved": round(fy_flop / fy_s / 1e12, 3),
                      "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                      "frac": round(fy_flop / fy_s / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
                      "hbm_achieved_gbs": round(fy_bytes / fy_s / 1e9, 1),
                      "hbm_frac": round(fy_bytes / fy_s / 1e9 / HBM_PEAK_GBS, 4),
                      "ms": round(ph["get_y"], 4),
                      "work_note": f"2P = {2 * P} fp64 MFMA flop and {y.element_size()} B "
                                   "written per field element (+ w and K read): the fp64 "
                                   "product bounds it (1.63 ms at peak vs 0.5 ms of writes at "
                                   "C5); gp_field"},
        },
        "cpu_baseline": None,
    }
    if ctx.world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_c5(pipe, res, args.c5_cpu_sample)
    pipe.close()
    print(json.dumps(line), flush=True)


def cpu_baseline_c5(pipe, res, sample: int):
    """The oracle on the host for C5: standardise + randomized_svd (same Omega) + basis + PC
    weights in full, then all P PC GPs (gp_ref.sepia_predict_w) and the field y = (w K) sd + mu
    for the first ``sample`` test points, extrapolated linearly in the points to m.  Parity:
    the oracle's singular values against the GPU's; the GPs and the field on the GPU's own basis
    K (singular vectors are unique up to sign: the GP means follow K's signs) against the GPU's
    mean / var / field rows."""
    from oracle import gp_ref
    t = pipe.t.cpu().numpy()
    Y = pipe.y.cpu().numpy()
    om = pipe.omega.cpu().numpy()
    tp = pipe.t_pred[:sample].cpu().numpy()
    n, P, m = t.shape[0], pipe.p, pipe.t_pred.shape[0]
    K_gpu = res["K"].cpu().numpy()
    t0 = time.perf_counter()
    mu, sd, ys = gp_ref.standardize(Y)
    _, S_o, Vh_o = gp_ref.randomized_svd(ys, P, k=0, q=1, omega=om)
    K_o = (gp_ref.pca_basis(S_o, Vh_o, P, n)).astype(np.float32).astype(np.float64)
    w_o = gp_ref.pc_weights(ys, K_o)
    t_basis = time.perf_counter() - t0
    w_hat = gp_ref.pc_weights(ys, K_gpu)                  # the GP inputs on the GPU's basis
    lam = np.sum(K_gpu * K_gpu, axis=1)
    t1 = time.perf_counter()
    mean, var = gp_ref.sepia_predict_w(t, tp, w_hat, pipe.samples, lam)
    y_o = (np.einsum("smp,py->smy", mean.astype(np.float32).astype(np.float64), K_gpu)
           * sd + mu).astype(np.float32)
    t_pts = time.perf_counter() - t1
    del w_o
    t_full = t_basis + t_pts / sample * m
    S = mean.shape[0]
    g_mean = res["mean"][:, :sample].cpu().numpy()
    g_var = res["var"][:, :sample].cpu().numpy()
    g_y = res["y"][:, :sample].cpu().numpy()
    S_g = res["S"].cpu().numpy()
    sgn = np.sign(np.sum(K_gpu * K_o, axis=1))
    return {"value": S * P * m / t_full, "unit": "predictions/s", "cores": _CPU_THREADS,
            "kind": "port",
            "sample": (f"oracle/gp_ref numpy fp64, OpenBLAS {_CPU_THREADS} threads on "
                       f"{cpu_model()}: standardise + randomized_svd + basis + PC weights in "
                       f"full ({t_basis:.2f} s), then all {P} PC GPs and the field for the first "
                       f"{sample} of {m} test points ({t_pts:.2f} s), extrapolated linearly in "
                       f"the points to m"),
            "parity_vs_gpu": {
                "points": sample,
                "max_rel_dS": float(np.max(np.abs(S_g - S_o) / S_o)),
                "max_abs_dK_signed": float(np.max(np.abs(K_gpu * sgn[:, None] - K_o))),
                "max_abs_dmean": float(np.max(np.abs(g_mean - mean))),
                "max_abs_dvar": float(np.max(np.abs(g_var - var))),
                "max_abs_dfield": float(np.max(np.abs(g_y.astype(np.float64) - y_o))),
                "max_abs_field": float(np.max(np.abs(y_o))),
                "note": "mean / var / field on the GPU's basis K; S and K against the oracle's "
                        "own SVD (K up to each PC's sign)"}}


# reference fit timings (timing.csv:9, n=512 P=8: PCA incl. load/standardise,
# tune_step_sizes(100, 5) + do_mcmc(512))
REF_FIT_PCA_S = 31.673
REF_FIT_MCMC_S = 1405.595


def fit_roofline(model, mcmc_s: float, sweeps: int, reps: int = 20) -> dict:
    """The fit's dominant kernel: the batched persistent factorisation inside every gp_loglik of
    a sweep, in its log-likelihood mode (pp_kernel<true>: Cholesky with the forward solve
    z = L^-1 w and the reduction to ll in the same launch, no L^-1).  One gp_loglik per
    speculative group at that group's batch ((2^g - 1) P problems at n = 512), at the fitted
    model's parameter values, timed ``reps`` times with the library's event pair around the
    factorisation (GP_PROF_POTRF) and with torch events around whole calls;
    flop = batch (n^3/3 + n^2)."""
    from gladsgp_amd import kernels
    sm = model._sampler()
    n, d, P, dev = sm.n, sm.d, sm.P, sm.dev
    pv = model.params.values()
    bu = np.asarray(pv["betaU"], dtype=np.float64).reshape(d + 1, P)
    lamUz = np.asarray(pv["lamUz"], dtype=np.float64).reshape(P)
    lamWs = np.asarray(pv["lamWs"], dtype=np.float64).reshape(P)
    lamWOs = float(np.asarray(pv["lamWOs"]).reshape(-1)[0])
    lam = model.LamSim.cpu().numpy().reshape(P)
    per_call = {}
    sizes = [(2 ** len(g) - 1) * P for g in sm.groups]
    for B in sorted(set(sizes)):
        k = B // P
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
        beta = t(np.tile(bu[1:].T, (k, 1)))
        sv = t(np.tile(1.0 / lamUz, k))
        dl = t(np.tile(1.0 / lamWs + 1.0 / (lamWOs * lam), k))
        w = sm.w.repeat(k, 1).contiguous()
        ws = kernels.LoglikWorkspace(n, B, dev)
        out = torch.empty(B, dtype=torch.float64, device=dev)
        for _ in range(3):
            kernels.loglik(sm.X, beta, sv, dl, w, ws, out)
        torch.cuda.synchronize()
        _capi.call("gp_profile_enable", 4 * reps)
        _capi.call("gp_profile_reset")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            kernels.loglik(sm.X, beta, sv, dl, w, ws, out)
        e1.record()
        torch.cuda.synchronize()
        cnt, tot = read_prof(_capi.PROF_POTRF)
        _capi.call("gp_profile_enable", 0)
        ws.check_status()
        per_call[B] = {"factorisation_ms": tot / max(cnt, 1),
                       "loglik_call_ms": e0.elapsed_time(e1) / reps}
    sweep_ms = 1e3 * mcmc_s / sweeps
    fact_per_sweep = sum(per_call[B]["factorisation_ms"] for B in sizes)
    Bmax = max(sizes)
    fl = Bmax * (n ** 3 / 3.0 + float(n) ** 2)
    ach = fl / (per_call[Bmax]["factorisation_ms"] * 1e-3) / 1e12
    return {"kernel": f"pp_kernel<true> (gp_loglik's batched Cholesky + in-chain forward "
                      f"solve, {Bmax} problems at n = {n})", "bound": "mfma",
            "achieved": round(ach, 3),
            "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(ach / FP64_MFMA_PEAK_TFLOPS, 4), "traffic": None,
            "avg_launch_ms": round(per_call[Bmax]["factorisation_ms"], 4),
            "flop_per_launch": fl,
            "calls_per_sweep": {str(B): sizes.count(B) for B in sorted(set(sizes))},
            "per_call_ms": {str(B): {k: round(v, 4) for k, v in c.items()}
                            for B, c in per_call.items()},
            "factorisation_share_of_sweep": round(fact_per_sweep / sweep_ms, 4),
            "sweep_ms": round(sweep_ms, 4),
            "work_note": "batch x (n^3/3 potrf + n^2 forward solve) per call; the chain of "
                         "n/64 dependent diagonal steps bounds it, not the flops (DESIGN §4.3); "
                         "timed outside the sampler's HIP graphs at the fitted parameters"}


def cpu_baseline_fit(model, cfg, n: int, P: int, sweeps: int, cpu_sweeps: int,
                     ny_frac: float) -> dict:
    """The oracle on the host for the fit: (1) PCA -- standardise + randomized_svd(y_std, 25,
    k=0, q=1) (gp_ref) on the first ``ny_frac`` of the field's nodes, extrapolated linearly in
    ny (every step of the PCA is linear in ny); (2) MCMC -- oracle/mcmc_ref.run_chain (the
    restated sweep with the restated likelihood: P scipy Cholesky solves per update) at the
    fitted model's inputs and step sizes for ``cpu_sweeps`` sweeps, extrapolated to the fit's
    ``sweeps``.  OpenBLAS on the pool's CPU share."""
    from gladsgp_amd import mcmc
    from oracle import gp_ref, mcmc_ref
    Yf = np.load(cfg.Y_physical, mmap_mode="r")              # (ny, n) float32, as stored
    ny = Yf.shape[0]
    nyc = max(1000, int(ny * ny_frac))
    y = np.ascontiguousarray(Yf[:nyc, :n].T)                 # (n, nyc) float32
    t0 = time.perf_counter()
    _, _, ys = gp_ref.standardize(y)
    np.random.seed(0)
    om = np.random.normal(size=(nyc, 25)).astype(np.float32)
    gp_ref.randomized_svd(ys.astype(np.float32), 25, k=0, q=1, omega=om)
    t_pca = (time.perf_counter() - t0) * ny / nyc
    del y, ys
    sd_ = model.data.sim_data
    X = sd_.t_dev.cpu().numpy()
    w = model.w_hat.cpu().numpy().T.copy()                  # (P, n)
    lam = model.LamSim.cpu().numpy().reshape(P)
    pr = model.params
    d = X.shape[1]
    spec = {k: (getattr(pr, k).dist, getattr(pr, k).params, getattr(pr, k).bounds,
                getattr(pr, k).mcmcStepType) for k in pr.names}
    state = {"betaU": np.asarray(pr.betaU.val, dtype=np.float64).reshape(d + 1, P),
             "lamUz": np.asarray(pr.lamUz.val, dtype=np.float64).reshape(P),
             "lamWs": np.asarray(pr.lamWs.val, dtype=np.float64).reshape(P),
             "lamWOs": float(np.asarray(pr.lamWOs.val).reshape(-1)[0])}
    steps = {k: getattr(pr, k).mcmcStepParam for k in pr.names}
    U = np.random.default_rng(7).random((cpu_sweeps, mcmc.uniforms_per_sweep(d, P)))
    t1 = time.perf_counter()
    mcmc_ref.run_chain(X, w, lam, spec, state, steps, U)
    t_sweep = (time.perf_counter() - t1) / cpu_sweeps
    t_mcmc = t_sweep * sweeps
    return {"value": t_pca + t_mcmc, "unit": "s", "cores": _CPU_THREADS, "kind": "port",
            "pca_s": t_pca, "mcmc_s": t_mcmc, "sweep_ms": 1e3 * t_sweep,
            "sample": (f"oracle numpy fp64, OpenBLAS {_CPU_THREADS} threads on {cpu_model()}: "
                       f"PCA (gp_ref.standardize + randomized_svd p=25) on {nyc} of {ny} nodes "
                       f"extrapolated linearly in ny; oracle/mcmc_ref.run_chain (P = {P} scipy "
                       f"Cholesky likelihoods per update, n = {n}) for {cpu_sweeps} sweeps "
                       f"({1e3 * t_sweep:.1f} ms each) extrapolated to the fit's {sweeps}")}


def main_fit(args):
    """The reference's fit_models at its own timing configuration (src/model.py:152-245,
    timing.csv:9): n=512 runs, d=8, a 1,347,945-node field (float32 like the reference), PCA
    basis from randomized_svd(p=25), P=8 PC GPs, tune_step_sizes(100, 5) + do_mcmc(512).
    One GPU; the model and timing files go to a temporary directory.  With --warmup > 0 (the
    default) an identical fit runs first in the same process and `value` is the second one's
    timing.csv PCA + MCMC seconds; the first's are reported as breakdown.cold."""
    import shutil
    import tempfile
    import types
    from gladsgp_amd import model as gmodel
    dev = torch.device("cuda", 0)
    n, d, P, ny = 512, 8, args.fit_pcs, args.ny
    rng = np.random.default_rng(0)
    t = rng.random((n, d))
    nm = 12
    modes = (rng.standard_normal((nm, ny)) * (0.6 ** np.arange(nm))[:, None]).astype(np.float32)
    coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, d) + k) for k in range(nm)], 1)
    Y = (coef.astype(np.float32) @ modes)
    Y += 1e-3 * rng.standard_normal(Y.shape, dtype=np.float32)
    tmp = tempfile.mkdtemp(prefix="gladsgp_fit_")
    try:
        np.savetxt(os.path.join(tmp, "X.csv"), t, delimiter=",",
                   header=",".join(f"x{i}" for i in range(d)), comments="")
        np.save(os.path.join(tmp, "Y.npy"), Y.T)          # the reference stores (ny, n)
        del Y
        cfg = types.SimpleNamespace(X_standard=os.path.join(tmp, "X.csv"),
                                    Y_physical=os.path.join(tmp, "Y.npy"), data_dir=tmp,
                                    exp="bench")
        # warm-up (--warmup > 0): one identical fit first, in the same process -- its PCA
        # phase carries the process's first-use costs (HIP context and code-object loads, the
        # caching allocator's first 8 GB, numpy's first draws: 0.50 vs 0.25 s for init_model,
        # profiles/r05/r05_pca_cold.log / r05_pca_warm.log); reported as `cold_s`, not `value`
        cold = None
        runs = 2 if args.warmup > 0 else 1
        for run in range(runs):
            t0 = time.perf_counter()
            models = gmodel.fit_models(cfg, [n], [P], dtype=np.float32, recompute=True,
                                       device=dev, seed=0)
            torch.cuda.synchronize()
            total = time.perf_counter() - t0
            tim = np.loadtxt(os.path.join(tmp, "models", "timing.csv"), delimiter=",")
            if run + 1 < runs:
                cold = {"pca_s": float(tim[2]), "mcmc_s": float(tim[3]),
                        "value": float(tim[2]) + float(tim[3])}
        sweeps = 100 * 5 + 100 + 512      # burn-in + 5 tuning levels + samples
        pca_s, mcmc_s = float(tim[2]), float(tim[3])
        roof = fit_roofline(models[-1], mcmc_s, sweeps)
        cpu = None
        if not args.no_cpu:
            cpu = cpu_baseline_fit(models[-1], cfg, n, P, sweeps, args.fit_cpu_sweeps,
                                   args.fit_cpu_ny_frac)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    value = pca_s + mcmc_s
    ref = REF_FIT_PCA_S + REF_FIT_MCMC_S if (P == 8 and ny == 1347945) else None
    line = {
        "metric": "GladsGP fit seconds (PCA + Metropolis MCMC), n=512 d=8 P=8 "
                  "ny=1,347,945 (timing.csv:9)",
        "value": value, "unit": "s", "n_gpus": 1, "steps": 1, "warmup": runs - 1,
        "ms_per_step": value * 1e3, "higher_is_better": False, "scaling": "strong",
        "vs_baseline": (value / ref) if ref else None, "dtype": "f64",
        "data": "synthetic low-rank field of the reference's shape (float32 in, like the "
                "reference), seeded",
        "config": {"workload": "fit_models: standardise + randomized_svd(p=25) + K basis + "
                               "pc_prec + tune_step_sizes(100,5) + do_mcmc(512)",
                   "n_train": n, "d": d, "pcs": P, "ny": ny,
                   "value_is": ("the second of two identical fits in one process (warm: "
                                "HIP context, code objects, allocator pools and host RNG "
                                "already initialised); the first is breakdown.cold"
                                if runs > 1 else "a single cold fit")},
        "breakdown": {"pca_s": pca_s, "mcmc_s": mcmc_s, "ref_pca_s": REF_FIT_PCA_S,
                      "ref_mcmc_s": REF_FIT_MCMC_S, "mcmc_ms_per_sweep": 1e3 * mcmc_s / sweeps,
                      "wall_s": total, "cold": cold},
        "roofline": roof, "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    try:
        main()
    finally:
        import torch.distributed as _tdist
        if _tdist.is_available() and _tdist.is_initialized():
            _tdist.destroy_process_group()
