"""CPU (gloo, world_size 2): the multi-rank plumbing of the sharded emulator — unit dealing,
contiguous test-point shards, broadcast, gather-to-rank-0 reassembly and max-over-ranks
timing — exercised with real process groups on 127.0.0.1."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from gladsgp_amd import dist as gdist
    from gladsgp_amd.emulator import assemble_units
    ctx = gdist.init_from_env("cpu")
    try:
        assert ctx.distributed and ctx.backend == "gloo"
        # broadcast of inputs from rank 0
        x = torch.arange(12, dtype=torch.float64) if rank == 0 else torch.zeros(12, dtype=torch.float64)
        gdist.broadcast_(ctx, x)
        ok_b = bool(torch.equal(x, torch.arange(12, dtype=torch.float64)))
        # units dealt round-robin (S=3 samples x P=5 PCs = 15 units); each rank computes
        # a recognisable value per unit, rank 0 reassembles unit order
        n_units, m = 15, 4
        mine = gdist.shard_units(n_units, rank, world)
        mean_l = torch.tensor([[u * 10.0 + k for k in range(m)] for u in mine], dtype=torch.float64)
        var_l = -mean_l
        out = assemble_units(ctx, mean_l.reshape(len(mine), m), var_l.reshape(len(mine), m), n_units)
        if rank == 0:
            mean_u, var_u = out
            ref = torch.tensor([[u * 10.0 + k for k in range(m)] for u in range(n_units)],
                               dtype=torch.float64)
            ok_g = bool(torch.equal(mean_u, ref) and torch.equal(var_u, -ref))
        else:
            ok_g = out is None
        t = gdist.max_over_ranks(ctx, 1.0 + rank)
        # strong-scaled single-output GP (bench C3): contiguous test-point blocks
        # of (mean, var) as (2, m_r), gathered to rank 0 in rank order
        m_tot = 1001
        lo, hi = gdist.shard_range(m_tot, rank, world)
        counts = [b - a for a, b in (gdist.shard_range(m_tot, r, world) for r in range(world))]
        j = torch.arange(lo, hi, dtype=torch.float64)
        blk = torch.stack([j * 2.0, -j])
        full = gdist.gather_cols(ctx, blk, counts)
        if rank == 0:
            ref = torch.arange(m_tot, dtype=torch.float64)
            ok_s = bool(full.shape == (2, m_tot) and torch.equal(full[0], 2 * ref)
                        and torch.equal(full[1], -ref))
        else:
            ok_s = full is None
        # field reconstruction: all-gather of w rows, then a column block of K per rank
        S_m, P, ny = 5, 3, 17
        rows = gdist.shard_units(S_m, rank, world)
        w_loc = torch.tensor([[10.0 * u + q for q in range(P)] for u in rows],
                             dtype=torch.float64).reshape(len(rows), P)
        rc = [len(gdist.shard_units(S_m, r, world)) for r in range(world)]
        w_all = gdist.all_gather_rows(ctx, w_loc, rc)
        order = np.concatenate([gdist.shard_units(S_m, r, world) for r in range(world)])
        w_ref = torch.tensor([[10.0 * u + q for q in range(P)] for u in order],
                             dtype=torch.float64)
        ok_a = bool(torch.equal(w_all, w_ref))
        c0, c1 = gdist.shard_range(ny, rank, world)
        Kfull = torch.arange(P * ny, dtype=torch.float64).reshape(P, ny)
        y_loc = w_all @ Kfull[:, c0:c1]            # stands in for the device GEMM
        ycnt = [b - a for a, b in (gdist.shard_range(ny, r, world) for r in range(world))]
        y = gdist.gather_cols(ctx, y_loc.contiguous(), ycnt)
        ok_y = bool(torch.equal(y, w_all @ Kfull)) if rank == 0 else y is None
        results[rank] = (ok_b, ok_g, t, ok_s, ok_a, ok_y)
    finally:
        dist.destroy_process_group()


def test_shard_helpers():
    from gladsgp_amd import dist as gdist
    assert gdist.shard_units(10, 0, 4) == [0, 4, 8]
    assert gdist.shard_units(10, 3, 4) == [3, 7]
    parts = [gdist.shard_range(10, r, 3) for r in range(3)]
    assert parts == [(0, 4), (4, 7), (7, 10)]
    assert sum(sorted(sum((gdist.shard_units(17, r, 8) for r in range(8)), []))) == sum(range(17))


@pytest.mark.timeout(120)
def test_gloo_world2_broadcast_gather_max():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_worker, args=(world, port, results), nprocs=world, join=True)
    for r in range(world):
        ok_b, ok_g, t, ok_s, ok_a, ok_y = results[r]
        assert ok_b and ok_g and ok_s and ok_a and ok_y
        assert t == 2.0


def test_split_counts():
    from gladsgp_amd.sharded import split_counts
    assert split_counts(100, 1, 40.0) == [100]
    for m, world, extra in ((100000, 8, 9200.0), (40000, 2, 3000.0), (10, 4, 0.0),
                            (7, 8, 0.0), (100, 3, 1e9)):
        c = split_counts(m, world, extra)
        assert len(c) == world and sum(c) == m and min(c) >= 0
        assert max(c[1:]) - min(c[1:]) <= 1
        assert c[0] <= max(c[1:])
    # rank 0's share is shortened by the extra work in points (C3 at 8 GPUs: ~9.2k points)
    c = split_counts(100000, 8, 9200.0)
    assert abs((c[0] + 9200.0) - c[1]) <= 8


def _points_worker(rank, world, port, results):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from gladsgp_amd import dist as gdist
    from gladsgp_amd.emulator import assemble_points
    from gladsgp_amd.sharded import LinvPacker
    ctx = gdist.init_from_env("cpu")
    try:
        # test-point sharding of U units (EmulatorPrediction shard="points"): every rank holds
        # all units on its block of the m points; rank 0 reassembles (U, m)
        U, m = 3, 11
        lo, hi = gdist.shard_range(m, rank, world)
        j = torch.arange(lo, hi, dtype=torch.float64)
        mean_l = torch.stack([100.0 * u + j for u in range(U)])
        out = assemble_points(ctx, mean_l, -mean_l, m)
        if rank == 0:
            ref = torch.stack([100.0 * u + torch.arange(m, dtype=torch.float64)
                               for u in range(U)])
            ok_p = bool(torch.equal(out[0], ref) and torch.equal(out[1], -ref))
        else:
            ok_p = out is None
        # L^-1 broadcast tile-packed (sharded.LinvPacker: column c from row 16 floor(c/16) on),
        # with z and rank 0's factorisation info, so every rank can raise alike; rebuilt exactly
        # (gp_pack_linv / gp_unpack_linv run on the GPU; here the documented layout, host-side)
        npad = 128
        full = torch.tril(torch.arange(1.0, npad * npad + 1, dtype=torch.float64)
                          .reshape(npad, npad)).T.contiguous().reshape(1, npad, npad)
        pk = LinvPacker(npad, torch.device("cpu"))
        order = LinvPacker.order(npad)
        packed = pk.buffer(torch.device("cpu"))
        zz = torch.arange(npad, dtype=torch.float64) * 0.5
        if rank == 0:
            packed[: pk.elems] = full.reshape(-1)[order]
            pk.z(packed).copy_(zz)
            packed[pk.info_off:] = 3.0
        gdist.broadcast_(ctx, packed)
        got = torch.zeros((1, npad, npad), dtype=torch.float64)
        got.view(-1).index_copy_(0, order, packed[: pk.elems])
        q = npad // 16
        ok_l = (bool(torch.equal(got, full)) and pk.elems == npad * npad - 128 * q * (q - 1)
                and order.numel() == pk.elems and bool(torch.equal(pk.z(packed), zz))
                and pk.info(packed).tolist() == [3])
        results[rank] = (ok_p, ok_l)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_gloo_world2_point_shards_and_packed_linv():
    world = 2
    mgr = mp.Manager()
    results = mgr.dict()
    mp.spawn(_points_worker, args=(world, _free_port(), results), nprocs=world, join=True)
    for r in range(world):
        assert results[r] == (True, True), results[r]


@pytest.mark.timeout(240)
def test_bench_gpus_flag_launches_ranks():
    """``python bench.py --gpus 2`` with no launcher starts two ranks itself (a child
    torch.distributed.run; --dry-run: gloo on the host, no GPU work) and rank 0's JSON reports
    n_gpus = 2; a process group smaller than --gpus is refused (non-zero exit)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--dry-run"], capture_output=True, text=True, env=env, timeout=200)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["dry_run"] is True
    env1 = dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--dry-run"], capture_output=True, text=True, env=env1, timeout=200)
    assert r.returncode != 0 and "2 but 1 ranks" in r.stderr


@pytest.mark.timeout(240)
@pytest.mark.parametrize("mode", ["wall_limit", "pg_timeout"])
def test_bench_stalled_rank_fails_loudly(mode):
    """A rank that never reaches a collective must not hang ``bench.py --gpus 2``: either the
    process group's timeout (dist.init_from_env, ~0.6 x --wall-limit under the launcher) makes
    the waiting rank raise, or the launcher's wall limit kills the ranks' process group and
    prints a JSON error line; both exit non-zero well inside the limit."""
    import json
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT",
                        "GPFIT_PG_TIMEOUT_S")}
    if mode == "wall_limit":
        env["GPFIT_PG_TIMEOUT_S"] = "900"          # only the wall limit can end it
        limit = 20
    else:
        limit = 30                                  # process-group timeout 18 s
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--dry-run", "--stall-rank", "1", "--wall-limit", str(limit)],
                       capture_output=True, text=True, env=env, timeout=200)
    elapsed = time.perf_counter() - t0
    assert r.returncode != 0, r.stdout[-2000:]
    assert elapsed < limit + 40, elapsed
    if mode == "wall_limit":
        assert r.returncode == 124
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout
        rec = json.loads(lines[0])
        assert rec["value"] is None and "wall-limit" in rec["error"] and rec["n_gpus"] == 2
    else:
        assert elapsed < limit, elapsed


def test_balanced_split_minimises_the_slowest_rank():
    """sharded.balanced_split against brute force on a staircase prediction time (the TRMM's
    residency rounds: 4096 points per round, a partial round at 0.65 of a full one)."""
    import math

    from gladsgp_amd.sharded import balanced_split

    def T(p):
        full, part = divmod(p, 4096)
        return 0.875e-3 * full + (0.57e-3 if part else 0.0) + 0.05e-3 * (p > 0)

    for m, world, t_fact in ((100000, 8, 2.0e-3), (100000, 2, 2.0e-3), (100000, 4, 1.9e-3),
                             (40000, 2, 0.3e-3), (5000, 8, 2.0e-3), (100000, 8, 40e-3)):
        c = balanced_split(m, world, t_fact, T)
        assert len(c) == world and sum(c) == m and min(c) >= 0
        assert c[0] % 128 == 0 or c[0] == m
        assert max(c[1:]) - min(c[1:]) <= 1

        def cost(m0):
            m1 = math.ceil((m - m0) / (world - 1))
            return max(t_fact + T(m0), T(m1))

        best = min(cost(m0) for m0 in range(0, m + 1, 128))
        assert cost(c[0]) <= best + 1e-12, (m, world, c, cost(c[0]), best)
    assert balanced_split(777, 1, 1.0, T) == [777]


def test_init_from_env_multi_rank_needs_master_port(monkeypatch):
    """WORLD_SIZE > 1 without MASTER_PORT fails at once (each rank picking its own free port
    would hang the rendezvous); only the one-rank force_group rehearsal picks a port itself."""
    from gladsgp_amd import dist as gdist
    for k in ("MASTER_PORT", "MASTER_ADDR"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "1")
    with pytest.raises(RuntimeError, match="MASTER_PORT"):
        gdist.init_from_env("cpu", backend="gloo")
