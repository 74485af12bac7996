"""GPU, two ranks on the one GPU of the test box (gloo process group, collectives staged
through the host; the driver's 8-GPU runs use RCCL with the same code path): the sharded
paths of SURVEY §8e end to end, each rank computing on cuda:0.

* multivariate emulator: EmulatorPrediction(ctx=...) deals the (sample, PC) GPs round-robin,
  gathers to rank 0 and reassembles — equal to the unsharded prediction bit for bit;
* field reconstruction: get_y(ctx=...) splits K by output columns after broadcasting w;
  gathered, it equals the unsharded get_y, and each rank's block (gather=False) its columns;
* strong-scaled single-output GP (bench C3): rank r predicts shard_range(m, r, 2) with
  gp_fit_predict and gather_cols reassembles (2, m) — bit-identical to one rank doing all m.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ensemble(n=72, ny=640, d=5, seed=8):
    rng = np.random.default_rng(seed)
    t = rng.random((n, d))
    modes = rng.standard_normal((5, ny)) * (0.5 ** np.arange(5))[:, None]
    coef = np.stack([np.sin(2 * np.pi * t @ rng.uniform(0, 1, d) + k) for k in range(5)], 1)
    return t, 2.0 + coef @ modes + 1e-2 * rng.standard_normal((n, ny))


def _worker(rank, world, port, results, tmpdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gladsgp_amd import dist as gdist
    from gladsgp_amd import kernels
    from gladsgp_amd import model as gm
    from gladsgp_amd.emulator import EmulatorPrediction
    ctx = gdist.init_from_env("cuda", backend="gloo", device_index=0)
    out = {}
    try:
        dev = ctx.device
        t, y = _ensemble()
        np.random.seed(0)                  # the same Omega on both ranks
        data, model = gm.init_model(t, y, "dist", 4, data_dir=os.path.join(tmpdir, str(rank)),
                                    device=dev, verbose=False)
        rng = np.random.default_rng(1)
        S, P = 3, 4
        samples = {"betaU": rng.uniform(0.2, 3.0, (S, (t.shape[1] + 1) * P)),
                   "lamUz": rng.uniform(0.5, 3.0, (S, P)),
                   "lamWs": rng.uniform(200, 3000, (S, P)),
                   "lamWOs": rng.uniform(50, 500, (S, 1))}
        t_pred = np.random.default_rng(2).random((29, t.shape[1]))
        shard = EmulatorPrediction(model=model, samples=samples, t_pred=t_pred, ctx=ctx)
        y_sh = shard.get_y()                       # gathered to rank 0
        y_blk = shard.get_y(gather=False)          # this rank's column block
        c0, c1 = shard.y_cols
        full = EmulatorPrediction(model=model, samples=samples, t_pred=t_pred)
        y_full = full.get_y()
        out["blk"] = bool(np.allclose(y_blk, y_full[:, :, c0:c1], rtol=1e-13, atol=1e-12))
        out["cols"] = (c0, c1)
        if rank == 0:
            out["w"] = bool(np.array_equal(shard.w, full.w) and
                            np.array_equal(shard.var, full.var))
            out["y"] = bool(np.allclose(y_sh, y_full, rtol=1e-13, atol=1e-12))
        else:
            out["w"] = shard.w is None
            out["y"] = y_sh is None
        # strong-scaled single GP over the test points (bench C3 at small size)
        n, m, d = 700, 5003, 8
        X = np.random.default_rng(0).random((n, d))
        yv = np.sin(X @ np.random.default_rng(1).uniform(0, 1, d))
        beta = np.random.default_rng(3).uniform(0.5, 5, d)
        Xs = np.random.default_rng(2).random((m, d))
        lo, hi = gdist.shard_range(m, rank, world)
        counts = [b - a for a, b in (gdist.shard_range(m, r, world) for r in range(world))]
        T = lambda a: torch.as_tensor(np.ascontiguousarray(a), device=dev)  # noqa: E731
        buf = torch.empty((2, hi - lo), dtype=torch.float64, device=dev)
        with kernels.FitPredictContext(dev) as fctx:
            kernels.fit_predict(T(X), T(Xs[lo:hi]), T(beta), 1.0, 1e-6, 1.0, T(yv),
                                out=(buf[0:1], buf[1:2]), ctx=fctx)
            res = gdist.gather_cols(ctx, buf, counts)
            if rank == 0:
                mean, var, _ = kernels.fit_predict(T(X), T(Xs), T(beta), 1.0, 1e-6, 1.0, T(yv),
                                                   ctx=fctx)
                out["c3"] = bool(torch.equal(res[0], mean[0]) and torch.equal(res[1], var[0]))
            else:
                out["c3"] = res is None
        torch.cuda.synchronize()
    except Exception as exc:  # report, do not hang the peer
        out["error"] = repr(exc)
    finally:
        results[rank] = out
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_ranks_sharded_paths(tmp_path):
    world = 2
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), results, str(tmp_path)), nprocs=world,
             join=True)
    for r in range(world):
        res = dict(results[r])
        assert "error" not in res, res.get("error")
        assert res["w"] and res["y"] and res["blk"] and res["c3"], res
    assert results[0]["cols"][1] == results[1]["cols"][0]


def _pipe_worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    import time
    import types
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    from gladsgp_amd import dist as gdist
    ctx = gdist.init_from_env("cuda", backend="gloo", device_index=0)
    try:
        X, y, beta, Xs, s, delta = bench.c3_inputs(640, 40000, 8)
        args = types.SimpleNamespace(warmup=2, steps=3, m_chunk=0)

        def timed(fn, steps):
            gdist.barrier(ctx)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            torch.cuda.synchronize()
            gdist.barrier(ctx)
            return gdist.max_over_ranks(ctx, time.perf_counter() - t0)

        pipe = bench.c3_pipelined(args, ctx, X, y, beta, Xs, s, delta, timed)
        results[rank] = {"counts": pipe["counts"], "check": pipe["check"]}
    except Exception as exc:  # noqa: BLE001 - reported to the parent
        import traceback
        results[rank] = {"error": traceback.format_exc()}
    finally:
        dist.destroy_process_group()


def test_two_ranks_pipelined_c3():
    """bench.py's N > 1 schedule: rank 0 factorises GP k+1 and broadcasts L^-1 while both ranks
    predict GP k on their blocks (consecutive GPs differ); the function itself checks the last
    step's gathered (mean, var) against a direct single-rank computation of that GP."""
    world = 2
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_pipe_worker, args=(world, _free_port(), results), nprocs=world, join=True)
    for r in range(world):
        res = dict(results[r])
        assert "error" not in res, res.get("error")
    counts = results[0]["counts"]
    assert sum(counts) == 40000 and len(counts) == 2 and 0 < counts[0] <= counts[1]
    chk = results[0]["check"]
    assert chk["gp"] == 4 and chk["max_abs_dmean"] <= 1e-12 and chk["max_abs_dvar"] <= 1e-12, chk
