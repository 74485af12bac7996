"""GPU, RCCL (torch.distributed backend "nccl") at world size 1: every collective branch of the
sharded paths run through a real one-rank RCCL communicator on the box's one GPU.

The multi-rank GPU tests (test_gpu_dist.py) put two ranks on one GPU, which RCCL does not
support, so they use gloo (host-staged).  Here the branches that only run over RCCL on the
driver's 8-GPU node execute for real: ``sharded._wire_bcast`` (async broadcast),
``PipelinedPredictor``'s double-buffered broadcast + ``pending.wait()``, ``dist.barrier(
device_ids=)``, ``gather`` / ``all_gather`` on device tensors, ``NativeComm`` (libgpfit's own
RCCL communicator) and ``EmulatorPrediction(ctx=)`` / ``get_y(ctx=)``.  Every result must be
bit-identical to the single-process call (a one-rank collective copies, it never computes).
Consumers these branches serve: assess_all_models.py:471,489 and sensitivity_indices.py:85-96
(multi-GP prediction), time_predictions.py:73-79 (single-output GP).
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


def _worker(rank, port, results, tmpdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0",
                      WORLD_SIZE="1", LOCAL_RANK="0")
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gladsgp_amd import dist as gdist
    from gladsgp_amd import kernels
    from gladsgp_amd import model as gm
    from gladsgp_amd.emulator import EmulatorPrediction
    from gladsgp_amd.sharded import PipelinedPredictor, calibrate, predict_sharded
    out = {}
    try:
        ctx = gdist.init_from_env("cuda", force_group=True)
        out["backend"] = (ctx.backend, dist.get_backend(), ctx.world, ctx.distributed)
        dev = ctx.device
        gdist.barrier(ctx)                                     # dist.barrier(device_ids=[0])
        out["max"] = gdist.max_over_ranks(ctx, 3.25) == 3.25   # all_reduce on a device tensor
        # gather / all-gather of device tensors (one rank: exact copies)
        g = torch.Generator(device="cpu").manual_seed(5)
        a = torch.randn((7, 33), generator=g, dtype=torch.float64).to(dev)
        ok = torch.equal(gdist.gather_cols(ctx, a, [33]), a)
        ok &= torch.equal(gdist.gather_rows(ctx, a, [7]), a)
        ok &= torch.equal(gdist.all_gather_rows(ctx, a, [7]), a)
        b = a.clone()
        gdist.broadcast_(ctx, b)
        ok &= torch.equal(b, a)
        out["collectives"] = bool(ok)
        # libgpfit's own RCCL communicator (gp_comm_*): id over the torch group, bcast, gather
        comm = gdist.NativeComm(ctx)
        try:
            c = a.clone()
            comm.bcast_(c)
            gat = comm.gather(a)
            torch.cuda.synchronize()
            out["native"] = bool(torch.equal(c, a) and gat.shape == (1, 7, 33) and
                                 torch.equal(gat[0], a))
        finally:
            comm.close()

        # single-output GP (C3 shape at small size): predict_sharded + PipelinedPredictor
        n, m, d = 640, 40000, 8
        X = np.random.default_rng(0).random((n, d))
        av = np.random.default_rng(1).uniform(0, 1, d)
        y = np.sin(2 * np.pi * X @ av) + 0.1 * np.sum(X * X, axis=1)
        beta = np.random.default_rng(3).uniform(0.5, 5.0, d)
        Xs = np.random.default_rng(2).random((m, d))
        T = lambda v: torch.as_tensor(np.ascontiguousarray(v), device=dev)  # noqa: E731
        Xd, Xsd, yd = T(X), T(Xs), T(y).reshape(1, n)
        sd = torch.tensor([1.0], dtype=torch.float64, device=dev)
        dd = torch.tensor([1e-6], dtype=torch.float64, device=dev)
        betas = [T(beta * (1.0 + 1e-3 * k)).reshape(1, d) for k in range(3)]
        direct = []
        for k in range(3):
            ch = kernels.cholesky_inverse(kernels.gram(Xd, betas[k], sd, dd))
            ch.check()
            direct.append(kernels.predict(ch, Xd, Xsd, betas[k], sd, sd, yd))
        fp = kernels.fit_predict(Xd, Xsd, betas[0], sd, dd, sd, yd)
        modes = {}
        with kernels.FitPredictContext(dev) as fctx:
            r = predict_sharded(ctx, Xd, Xsd, betas[0], sd, dd, sd, yd, mode="redundant",
                                fctx=fctx)
            modes["redundant"] = bool(torch.equal(r[0], fp[0][0]) and
                                      torch.equal(r[1], fp[1][0]))
        r = predict_sharded(ctx, Xd, Xsd, betas[1], sd, dd, sd, yd, mode="broadcast")
        modes["broadcast"] = bool(torch.equal(r[0], direct[1][0][0]) and
                                  torch.equal(r[1], direct[1][1][0]))
        out["modes"] = modes
        t_fact, t_point = calibrate(ctx, Xd, Xsd, betas[0], sd, dd, sd, yd)
        out["calib"] = bool(t_fact > 0 and t_point > 0)
        gps = [(b_, sd, dd, sd) for b_ in betas]
        pp = PipelinedPredictor(ctx, Xd, Xsd, yd, calib_gp=gps[0])
        pp.start(gps[0])
        res = [pp.step(gps[k + 1] if k + 1 < 3 else None).clone() for k in range(3)]
        pp.finish()
        out["pipe_counts"] = pp.counts
        out["pipe"] = [bool(torch.equal(res[k][0], direct[k][0][0]) and
                            torch.equal(res[k][1], direct[k][1][0])) for k in range(3)]
        # the ranks >= 1 path forced on the one rank: prediction straight from the broadcast
        # payload (tile-packed L^-1 read in place, z shipped: no unpack, no trmv launched --
        # kernels.predict is handed z, so gp_predict_ex skips its trmv)
        seen = []
        real_predict = kernels.predict

        def spy(chol, *a, **kw):
            seen.append((type(chol).__name__, kw.get("z") is not None))
            return real_predict(chol, *a, **kw)

        kernels.predict = spy
        try:
            pr = PipelinedPredictor(ctx, Xd, Xsd, yd, counts=[m], receiver_path=True)
            pr.start(gps[0])
            res_r = [pr.step(gps[k + 1] if k + 1 < 3 else None).clone() for k in range(3)]
            pr.finish()
        finally:
            kernels.predict = real_predict
        out["pipe_receiver"] = [bool(torch.equal(res_r[k][0], direct[k][0][0]) and
                                     torch.equal(res_r[k][1], direct[k][1][0]))
                                for k in range(3)]
        out["receiver_calls"] = seen
        # a failed factorisation raises through the broadcast (rank 0's info travels with it)
        dbad = torch.tensor([-2.0], dtype=torch.float64, device=dev)
        try:
            predict_sharded(ctx, Xd, Xsd, betas[2], sd, dbad, sd, yd, mode="broadcast",
                            counts=[m])
            out["raised"] = False
        except ValueError:
            out["raised"] = True

        # multivariate emulator: (sample, PC) units dealt over the one rank, gathered by RCCL
        t, yy = _ensemble()
        np.random.seed(0)
        data, model = gm.init_model(t, yy, "rccl", 4, data_dir=tmpdir, device=dev,
                                    verbose=False)
        rng = np.random.default_rng(1)
        S, P = 3, 4
        samples = {"betaU": rng.uniform(0.2, 3.0, (S, (t.shape[1] + 1) * P)),
                   "lamUz": rng.uniform(0.5, 3.0, (S, P)),
                   "lamWs": rng.uniform(200, 3000, (S, P)),
                   "lamWOs": rng.uniform(50, 500, (S, 1))}
        t_pred = np.random.default_rng(2).random((29, t.shape[1]))
        sh = EmulatorPrediction(model=model, samples=samples, t_pred=t_pred, ctx=ctx)
        full = EmulatorPrediction(model=model, samples=samples, t_pred=t_pred)
        out["emu_w"] = bool(np.array_equal(sh.w, full.w) and np.array_equal(sh.var, full.var))
        out["emu_y"] = bool(np.array_equal(sh.get_y(), full.get_y()))
        sh.w = sh.w.astype(np.float32)
        full.w = full.w.astype(np.float32)
        ys, yf = sh.get_y(), full.get_y()
        out["emu_y32"] = bool(ys.dtype == np.float32 and np.array_equal(ys, yf))
        # scalar GP, forced test-point sharding (one unit, one rank)
        pts = EmulatorPrediction(model=model, samples=samples, t_pred=t_pred, ctx=ctx,
                                 shard="points")
        out["emu_points"] = bool(np.array_equal(pts.w, full.mean) and
                                 np.array_equal(pts.var, full.var))
        torch.cuda.synchronize()
    except Exception:  # noqa: BLE001 - reported to the parent
        import traceback
        out["error"] = traceback.format_exc()
    finally:
        results[rank] = out
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_world1_every_collective_branch(tmp_path):
    """A one-rank RCCL process group: the sharded single-GP modes, the pipelined predictor, the
    raw collectives, libgpfit's NativeComm and the emulator's unit / point sharding all equal the
    single-process results bit for bit, and a non-PD GP still raises through the broadcast."""
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(_free_port(), results, str(tmp_path)), nprocs=1, join=True)
    res = dict(results[0])
    assert "error" not in res, res.get("error")
    assert res["backend"] == ("nccl", "nccl", 1, True), res["backend"]
    assert res["max"] and res["collectives"] and res["native"], res
    assert all(res["modes"].values()), res["modes"]
    assert res["calib"] and res["pipe_counts"] == [40000], res
    assert all(res["pipe"]), res["pipe"]
    assert all(res["pipe_receiver"]), res["pipe_receiver"]
    assert res["receiver_calls"] == [("PackedLinv", True)] * 3, res["receiver_calls"]
    assert res["raised"], res
    assert res["emu_w"] and res["emu_y"] and res["emu_y32"] and res["emu_points"], res
