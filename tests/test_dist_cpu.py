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
        results[rank] = (ok_b, ok_g, t)
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
        ok_b, ok_g, t = results[r]
        assert ok_b and ok_g
        assert t == 2.0
