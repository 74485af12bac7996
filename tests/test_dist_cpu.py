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
