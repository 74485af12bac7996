#!/usr/bin/env python
"""bench.py — GP posterior predictions/sec, fp64, C3 (n=4096 train, m=100k test, d=8).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A step is one full pass of the hot path for one GP on one GPU, from hyperparameters to
answers: ARD-SE Gram (n x n) -> blocked MFMA Cholesky + L^-1 -> fused cross-covariance /
TRMM / mean+variance over that rank's m = 100k test points.  Within a step the
cross-covariance (independent of the factorisation) is built on a second HIP stream while
the latency-bound Cholesky runs (``--serial`` disables that); steps never overlap.  Inputs are HBM-resident before
the timed region.  Ranks are independent test-point shards of one trained GP (weak scaling:
every rank predicts its own 100k points; no collective inside a step), so
value = N * 100k * K / max-over-ranks(time).

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
import platform
import sys
import time

_CPU_THREADS = min(16, os.cpu_count() or 1)
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


def c3_inputs(rank: int, n: int, m: int, d: int):
    """SURVEY §8d C3 recipe (seeded).  Rank r predicts rows [r m, (r+1) m) of rng(2)'s stream."""
    X = np.random.default_rng(0).random((n, d))
    a = np.random.default_rng(1).uniform(0, 1, d)
    y = np.sin(2 * np.pi * X @ a) + 0.1 * np.sum(X * X, axis=1)
    beta = np.random.default_rng(3).uniform(0.5, 5.0, d)
    Xs = np.random.default_rng(2).random(((rank + 1) * m, d))[rank * m:]
    return X, y, beta, Xs, 1.0, 1e-6


def c4_inputs(n: int, m: int, d: int, P: int):
    """SURVEY §8d C4 recipe: X = rng(0), beta_j = rng(10+j), w_j = rng(100+j), X* = rng(2)."""
    X = np.random.default_rng(0).random((n, d))
    beta = np.stack([np.random.default_rng(10 + j).uniform(0.5, 5.0, d) for j in range(P)])
    W = np.stack([np.random.default_rng(100 + j).standard_normal(n) for j in range(P)])
    Xs = np.random.default_rng(2).random((m, d))
    return X, W, beta, Xs, np.ones(P), np.full(P, 1e-6)


def cpu_baseline(X, y, beta, Xs, s, delta, budget_s: float):
    """numpy fp64 oracle (Gram -> cholesky -> chunked cross-cov + solve_triangular) on host."""
    from oracle import gp_ref
    import scipy.linalg as sla
    t0 = time.perf_counter()
    G = gp_ref.gram_ardse(X, beta, s, delta)
    L = np.linalg.cholesky(G)
    alpha = sla.cho_solve((L, True), y)
    t_fact = time.perf_counter() - t0
    chunk, done, t_pred = 2000, 0, 0.0
    means, vars_ = [], []
    while done < Xs.shape[0] and (t_fact + t_pred) < budget_s:
        t1 = time.perf_counter()
        Ks = gp_ref.cross_ardse(Xs[done:done + chunk], X, beta, s)
        mu = Ks @ alpha
        V = sla.solve_triangular(L, Ks.T, lower=True, check_finite=False)
        var = s - np.einsum("ij,ij->j", V, V)
        t_pred += time.perf_counter() - t1
        means.append(mu)
        vars_.append(var)
        done += Ks.shape[0]
    m = Xs.shape[0]
    t_full = t_fact + t_pred / done * m
    # "reference-faithful": re-factorise per batch of 4 points (assess_all_models.py:481-489)
    t2 = time.perf_counter()
    G4 = gp_ref.gram_ardse(X, beta, s, delta)
    L4 = np.linalg.cholesky(G4)
    a4 = sla.cho_solve((L4, True), y)
    K4 = gp_ref.cross_ardse(Xs[:4], X, beta, s)
    _ = K4 @ a4, sla.solve_triangular(L4, K4.T, lower=True)
    t4 = time.perf_counter() - t2
    return {
        "value": m / t_full, "unit": "predictions/s", "cores": _CPU_THREADS, "kind": "port",
        "sample": (f"oracle/gp_ref numpy fp64 (OpenBLAS, {_CPU_THREADS} threads, "
                   f"{platform.processor() or platform.machine()}): full n={X.shape[0]} "
                   f"Gram+Cholesky ({t_fact:.2f} s) + predict on the first {done} of {m} test "
                   f"points ({t_pred:.2f} s), extrapolated linearly to m={m}"),
        "reference_faithful_value": 4.0 / t4,
        "reference_faithful_sample": ("re-factorise per batch of 4 test points as "
                                      "assess_all_models.py:481-489 does: one batch timed "
                                      f"({t4:.2f} s)"),
    }, np.concatenate(means), np.concatenate(vars_)


def read_prof(pid):
    import ctypes
    cnt, tot, mx = ctypes.c_int(0), ctypes.c_double(0), ctypes.c_double(0)
    _capi.call("gp_profile_read", pid, ctypes.addressof(cnt), ctypes.addressof(tot),
               ctypes.addressof(mx))
    return cnt.value, max(tot.value, 1e-9)   # events off (GPFIT_BENCH_NOEVENTS=1): no data


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--m", type=int, default=100000, help="test points per GPU")
    ap.add_argument("--d", type=int, default=8)
    ap.add_argument("--m-chunk", type=int, default=0)
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds for the CPU leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--workload", choices=("c3", "c4", "fit"), default="c3")
    ap.add_argument("--ny", type=int, default=1347945, help="fit: field size per run")
    ap.add_argument("--fit-pcs", type=int, default=8, help="fit: principal components")
    ap.add_argument("--serial", action="store_true",
                    help="c3: one stream, no overlap at all (gram, potrf, predict in order)")
    ap.add_argument("--pipeline", action="store_true",
                    help="c3: alternate two streams so the next step's factorisation runs "
                         "under the current TRMM (measured no gain: the TRMM holds every CU "
                         "slot and the factorisation's launches wait behind it)")
    ap.add_argument("--pcs", type=int, default=32, help="c4: number of PC GPs")
    ap.add_argument("--c4-path", choices=("fit_predict", "predict"), default="predict",
                    help="c4: gram -> potrf -> gp_predict (default), or one gp_fit_predict per "
                         "step (measured 1-3%% slower at C4: its cross-covariance, 5x the "
                         "batched potrf, stretches the potrf and the TRMM waits for all of it)")
    args = ap.parse_args()
    if args.workload == "c4":
        return main_c4(args)
    if args.workload == "fit":
        return main_fit(args)

    ctx = gdist.init_from_env("cuda")
    dev = ctx.device
    n, m, d = args.n, args.m, args.d
    X, y, beta, Xs, s, delta = c3_inputs(ctx.rank, n, m, d)
    Xd = torch.as_tensor(X, device=dev)
    Xsd = torch.as_tensor(Xs, device=dev)
    yd = torch.as_tensor(y, device=dev).reshape(1, n)
    bd = torch.as_tensor(beta, device=dev).reshape(1, d)
    sd = torch.tensor([s], dtype=torch.float64, device=dev)
    dd = torch.tensor([delta], dtype=torch.float64, device=dev)
    # Default: one gp_fit_predict per step on the current stream (its cross-covariance runs
    # on a library stream while the factorisation runs).  --pipeline alternates two streams
    # and two buffer sets so step t+1's Gram + factorisation + cross-covariance run under step
    # t's TRMM; every step still does all of its own work inside the timed region.
    nslot = 2 if (args.pipeline and not args.serial) else 1
    streams = ([torch.cuda.current_stream(dev)] if nslot == 1 else
               [torch.cuda.Stream(device=dev) for _ in range(nslot)])
    wss = [kernels.PredictWorkspace() for _ in range(nslot)]
    outs = [(torch.empty((1, m), dtype=torch.float64, device=dev),
             torch.empty((1, m), dtype=torch.float64, device=dev)) for _ in range(nslot)]
    mean, var = outs[0]
    counter = [0]

    def step():
        sl = counter[0] % nslot
        counter[0] += 1
        if args.serial:
            G = kernels.gram(Xd, bd, sd, dd)
            ch = kernels.cholesky_inverse(G)
            kernels.predict(ch, Xd, Xsd, bd, sd, sd, yd, m_chunk=args.m_chunk,
                            workspace=wss[sl], out=outs[sl])
            return ch
        with torch.cuda.stream(streams[sl]):
            _, _, ch = kernels.fit_predict(Xd, Xsd, bd, sd, dd, sd, yd, m_chunk=args.m_chunk,
                                           workspace=wss[sl], out=outs[sl])
        return ch

    for _ in range(args.warmup):
        ch = step()
    torch.cuda.synchronize()
    ch.check()
    if os.environ.get("GPFIT_BENCH_NOEVENTS") != "1":
        _capi.call("gp_profile_enable", 64 * (args.steps + 1))
    _capi.call("gp_profile_reset")

    gdist.barrier(ctx)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    gdist.barrier(ctx)
    elapsed = time.perf_counter() - t0
    elapsed = gdist.max_over_ranks(ctx, elapsed)

    prof = {k: read_prof(v) for k, v in (("trmm", _capi.PROF_TRMM), ("gram", _capi.PROF_GRAM),
                                         ("potrf", _capi.PROF_POTRF),
                                         ("cross", _capi.PROF_CROSS))}
    _capi.call("gp_profile_enable", 0)

    if ctx.rank != 0:
        return
    K = args.steps
    value = ctx.world * m * K / elapsed
    # algorithmic work: trmm n^2 + mean/var 4n flop per prediction
    tr_cnt, tr_ms = prof["trmm"]
    tr_flops = float(m) * K * (n * n + 4 * n)
    tr_tfs = tr_flops / (tr_ms * 1e-3) / 1e12
    traffic, traffic_src = None, None
    tf = os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json")
    tj = json.load(open(tf)) if os.path.exists(tf) else {}
    chunk = args.m_chunk or 16384   # the library's default test-point chunk for one GP
    if tj and n == 4096 and chunk == tj.get("m_chunk"):
        kt = tj["kernels"].get("trmm_pair_kernel") or tj["kernels"]["trmm_reduce_kernel"]
        traffic = kt["bytes_per_launch"]
        traffic_src = "profiles/r01/pmc_traffic.json (FETCH_SIZE x2 + WRITE_SIZE, per launch)"
    roof = {"kernel": "trmm_pair_kernel", "bound": "mfma", "achieved": round(tr_tfs, 3),
            "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(tr_tfs / FP64_MFMA_PEAK_TFLOPS, 4),
            "traffic": traffic, "traffic_source": traffic_src, "launches": tr_cnt,
            "avg_launch_ms": round(tr_ms / max(tr_cnt, 1), 4),
            "flop_per_launch": tr_flops / max(tr_cnt, 1),
            "work_note": "n^2 + 4n flop per prediction (lower-triangular L^-1 K*^T + mean/var)"}
    g_cnt, g_ms = prof["gram"]
    g_bytes = (4.0 * n * (n + 1) + 8.0 * n * d) * g_cnt   # lower triangle written + X read
    p_cnt, p_ms = prof["potrf"]
    p_flops = 2.0 * n ** 3 / 3.0 * p_cnt
    c_cnt, c_ms = prof["cross"]
    npad = kernels.padded_n(n)
    c_bytes = 8.0 * npad * m * K
    aux = {
        "gram": {"bound": "hbm", "achieved": round(g_bytes / (g_ms * 1e-3) / 1e9, 1),
                 "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(g_bytes / (g_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                 "avg_launch_ms": round(g_ms / max(g_cnt, 1), 4)},
        "potrf_inv": {"bound": "mfma", "achieved": round(p_flops / (p_ms * 1e-3) / 1e12, 3),
                      "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                      "frac": round(p_flops / (p_ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS, 4),
                      "avg_call_ms": round(p_ms / max(p_cnt, 1), 4),
                      "work_note": "potrf n^3/3 + triangular inverse n^3/3"},
        "cross": {"bound": "hbm", "achieved": round(c_bytes / (c_ms * 1e-3) / 1e9, 1),
                  "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": round(c_bytes / (c_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                  "ms_per_step": round(c_ms / K, 4)},
        "trmm_ms_per_step": round(tr_ms / K, 4),
    }
    line = {
        "metric": METRIC, "value": value, "unit": "predictions/s", "n_gpus": ctx.world,
        "steps": K, "warmup": args.warmup, "ms_per_step": elapsed / K * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (SURVEY §8d C3 recipe: seeded uniform design, sin target)",
        "config": {"workload": "C3 single-output ARD-SE GP: Gram + Cholesky/L^-1 + predict",
                   "n_train": n, "m_test_per_gpu": m, "d": d,
                   "parallelism": f"test-point shards x{ctx.world}, redundant factorisation",
                   "pipeline": ("serial" if args.serial else
                                "gp_fit_predict (cross-covariance overlapped with the "
                                "factorisation)" if nslot == 1 else
                                "gp_fit_predict, 2 alternating streams (next factorisation "
                                "under the current TRMM)")},
        "roofline": roof, "roofline_aux": aux, "cpu_baseline": None,
    }
    if ctx.world == 1 and not args.no_cpu:
        cb, mu_ref, var_ref = cpu_baseline(X, y, beta, Xs, s, delta, args.cpu_budget)
        k = mu_ref.shape[0]
        mu_g = mean[0, :k].cpu().numpy()
        var_g = var[0, :k].cpu().numpy()
        cb["parity_vs_gpu"] = {"points": int(k),
                               "max_abs_dmean": float(np.max(np.abs(mu_g - mu_ref))),
                               "max_abs_dvar": float(np.max(np.abs(var_g - var_ref)))}
        line["cpu_baseline"] = cb
    print(json.dumps(line), flush=True)


def main_c4(args):
    from gladsgp_amd.emulator import assemble_units
    ctx = gdist.init_from_env("cuda")
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

    def step():
        if bl and args.c4_path == "fit_predict":
            # one gp_fit_predict over this rank's PCs: the cross-covariance of every chunk runs
            # on a library stream under the batched factorisation
            kernels.fit_predict(Xd, Xsd, Bl, Sl, Dl, Sl, Wl, m_chunk=args.m_chunk, workspace=ws,
                                out=(mean, var))
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
    if ctx.rank != 0:
        return
    K = args.steps
    value = P * m * K / elapsed
    tr_flops = float(bl) * m * K * (n * n + 4 * n)
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
                   "path": args.c4_path},
        "roofline": {"kernel": "trmm_pair_kernel (rank 0's PCs)", "bound": "mfma",
                     "achieved": round(tr_tfs, 3), "peak": FP64_MFMA_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(tr_tfs / FP64_MFMA_PEAK_TFLOPS, 4),
                     "traffic": None, "launches": tr_cnt,
                     "avg_launch_ms": round(tr_ms / max(tr_cnt, 1), 4)},
        "roofline_aux": {"potrf_inv_ms_per_step": round(p_ms / K, 4)},
        "cpu_baseline": None,
    }
    assert out is not None and out[0].shape == (P, m)
    print(json.dumps(line), flush=True)


# reference fit timings (timing.csv:9, n=512 P=8: PCA incl. load/standardise,
# tune_step_sizes(100, 5) + do_mcmc(512))
REF_FIT_PCA_S = 31.673
REF_FIT_MCMC_S = 1405.595


def main_fit(args):
    """The reference's fit_models at its own timing configuration (src/model.py:152-245,
    timing.csv:9): n=512 runs, d=8, a 1,347,945-node field (float32 like the reference), PCA
    basis from randomized_svd(p=25), P=8 PC GPs, tune_step_sizes(100, 5) + do_mcmc(512).
    One GPU; the model and timing files go to a temporary directory."""
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
        t0 = time.perf_counter()
        gmodel.fit_models(cfg, [n], [P], dtype=np.float32, recompute=True, device=dev, seed=0)
        torch.cuda.synchronize()
        total = time.perf_counter() - t0
        tim = np.loadtxt(os.path.join(tmp, "models", "timing.csv"), delimiter=",")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    pca_s, mcmc_s = float(tim[2]), float(tim[3])
    value = pca_s + mcmc_s
    ref = REF_FIT_PCA_S + REF_FIT_MCMC_S if (P == 8 and ny == 1347945) else None
    sweeps = 100 * 5 + 100 + 512      # burn-in + 5 tuning levels + samples
    line = {
        "metric": "GladsGP fit seconds (PCA + Metropolis MCMC), n=512 d=8 P=8 "
                  "ny=1,347,945 (timing.csv:9)",
        "value": value, "unit": "s", "n_gpus": 1, "steps": 1, "warmup": 0,
        "ms_per_step": value * 1e3, "higher_is_better": False, "scaling": "strong",
        "vs_baseline": (value / ref) if ref else None, "dtype": "f64",
        "data": "synthetic low-rank field of the reference's shape (float32 in, like the "
                "reference), seeded",
        "config": {"workload": "fit_models: standardise + randomized_svd(p=25) + K basis + "
                               "pc_prec + tune_step_sizes(100,5) + do_mcmc(512)",
                   "n_train": n, "d": d, "pcs": P, "ny": ny},
        "breakdown": {"pca_s": pca_s, "mcmc_s": mcmc_s, "ref_pca_s": REF_FIT_PCA_S,
                      "ref_mcmc_s": REF_FIT_MCMC_S, "mcmc_ms_per_sweep": 1e3 * mcmc_s / sweeps,
                      "wall_s": total},
        "roofline": None, "cpu_baseline": None,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
