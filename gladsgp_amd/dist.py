"""One process per GPU over torch.distributed (backend "nccl" = RCCL on ROCm, "gloo" on CPU).

The GP emulator shards without a data-path exchange:
  * multivariate emulator (C4/C5): the P x S independent (sample, PC) GPs are dealt
    round-robin to ranks; inputs are broadcast once from rank 0, per-rank (mean, var) blocks are
    gathered to rank 0 once at the end;
  * single-output GP (C2/C3): every rank factorises the same n x n Gram redundantly (~3 ms at
    n = 4096) and predicts its contiguous block of the test points; the (mean, var) blocks are
    gathered to rank 0 (``gather_cols``);
  * field reconstruction (get_y): the basis K is split by output columns, the PC weights are
    all-gathered (``all_gather_rows``) and every rank reconstructs its column block.

The reference has no distributed code at all (SLURM job arrays of the external
simulator only), so there is no call pattern to mirror; collectives here are the minimum the
sharding needs: one broadcast of the inputs and one gather of the outputs.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class Context:
    rank: int
    world: int
    local_rank: int
    device: torch.device
    backend: str | None

    @property
    def distributed(self) -> bool:
        return self.backend is not None


def init_from_env(device_type: str | None = None, backend: str | None = None,
                  device_index: int | None = None, force_group: bool = False,
                  timeout_s: float | None = None) -> Context:
    """Join the process group described by RANK/WORLD_SIZE/MASTER_* (torchrun), if any.

    Defaults: one GPU per rank (cuda:LOCAL_RANK) over RCCL.  ``backend="gloo"`` with
    ``device_index`` lets several ranks share one GPU (the multi-rank GPU tests on a 1-GPU box;
    collectives then stage through the host).  ``force_group``: join a process group even at
    world size 1 (RCCL accepts a one-rank communicator), so every collective branch of the
    sharded paths runs exactly as it does on N GPUs -- the one-GPU rehearsal of the RCCL code
    path (``bench.py --force-nccl``, ``tests/test_gpu_rccl.py``).

    ``timeout_s`` bounds the rendezvous and every collective of the group (default
    ``GPFIT_PG_TIMEOUT_S`` or 180 s, well under a driver's 600 s bench limit): a rank that never
    arrives makes the others raise instead of waiting out torch's default (10-30 min)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        idx = local_rank if device_index is None else device_index
        torch.cuda.set_device(idx)
        device = torch.device("cuda", idx)
    else:
        device = torch.device("cpu")
    if world > 1 or force_group:
        backend = backend or ("nccl" if device_type == "cuda" else "gloo")
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                if world > 1:
                    # every rank picking its own free port would leave rank 0 listening on one
                    # port and the others dialling others until the rendezvous times out
                    raise RuntimeError(
                        f"init_from_env: WORLD_SIZE={world} but MASTER_PORT is not set; launch "
                        "with torchrun / torch.distributed.run or export MASTER_PORT on every "
                        "rank")
                # the one-rank rehearsal (force_group): nobody else has to find this port
                os.environ["MASTER_PORT"] = str(_free_port())
            kw = {"device_id": device} if backend == "nccl" else {}
            if timeout_s is None:
                timeout_s = float(os.environ.get("GPFIT_PG_TIMEOUT_S", "180"))
            dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
    else:
        backend = None
    return Context(rank, world, local_rank, device, backend)


def _free_port() -> int:
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def barrier(ctx: Context) -> None:
    if ctx.distributed:
        if ctx.device.type == "cuda" and ctx.backend == "nccl":
            dist.barrier(device_ids=[ctx.local_rank])
        else:
            dist.barrier()


def max_over_ranks(ctx: Context, value: float) -> float:
    if not ctx.distributed:
        return value
    t = _wire(ctx, torch.tensor([value], dtype=torch.float64, device=ctx.device))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def broadcast_(ctx: Context, t: torch.Tensor, src: int = 0) -> torch.Tensor:
    """In-place broadcast of ``t`` from ``src`` (RCCL over xGMI on the GPU path)."""
    if ctx.distributed:
        w = _wire(ctx, t)
        dist.broadcast(w, src=src)
        if w is not t:
            t.copy_(w)
    return t


def shard_units(n_units: int, rank: int, world: int) -> list[int]:
    """Round-robin deal of independent units (PC GPs, samples) to ranks."""
    return list(range(rank, n_units, world))


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [a, b) of n items for ``rank`` (balanced to within one item)."""
    q, r = divmod(n, world)
    a = rank * q + min(rank, r)
    return a, a + q + (1 if rank < r else 0)


def _wire(ctx: Context, t: torch.Tensor) -> torch.Tensor:
    """Tensor as the backend moves it: gloo (the CPU test backend, also used to run two ranks
    on one GPU) only carries host tensors; RCCL carries device tensors in place."""
    return t.cpu() if (ctx.backend == "gloo" and t.is_cuda) else t


def gather_rows(ctx: Context, local: torch.Tensor, counts: list[int]) -> torch.Tensor | None:
    """Gather variable-length row blocks (dim 0) to rank 0; returns the concatenation there.

    Blocks are padded to the largest count so a single equal-shape ``gather`` serves RCCL and
    gloo alike (only rank 0 receives: one message per rank over xGMI, no all-to-all);
    rank 0 trims and concatenates, the other ranks get None.
    """
    if not ctx.distributed:
        return local
    mx = max(counts)
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if local.shape[0]:
        pad[: local.shape[0]] = local
    pad = _wire(ctx, pad)
    bufs = [torch.empty_like(pad) for _ in range(ctx.world)] if ctx.rank == 0 else None
    dist.gather(pad, gather_list=bufs, dst=0)
    if ctx.rank != 0:
        return None
    return torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0).to(local.device)


def gather_cols(ctx: Context, local: torch.Tensor, counts: list[int]) -> torch.Tensor | None:
    """Gather variable-length column blocks (last dim) to rank 0, concatenated in rank order.

    The strong-scaled single-output GP: rank r holds (mean, var) of its contiguous
    test-point block ``shard_range(m, r, N)`` as a (2, m_r) tensor; rank 0 receives (2, m).
    One padded equal-shape ``gather`` (RCCL / gloo); other ranks get None.
    """
    if not ctx.distributed:
        return local
    mx = max(counts)
    lead = tuple(local.shape[:-1])
    pad = torch.zeros(lead + (mx,), dtype=local.dtype, device=local.device)
    pad[..., : local.shape[-1]] = local
    pad = _wire(ctx, pad)
    bufs = [torch.empty_like(pad) for _ in range(ctx.world)] if ctx.rank == 0 else None
    dist.gather(pad, gather_list=bufs, dst=0)
    if ctx.rank != 0:
        return None
    return torch.cat([b[..., :c] for b, c in zip(bufs, counts)], dim=-1).to(local.device)


def all_gather_rows(ctx: Context, local: torch.Tensor, counts: list[int]) -> torch.Tensor:
    """Every rank receives the rank-order concatenation of variable-length row blocks (dim 0)
    — the all-gather of the PC weights w before the sharded field reconstruction (§8e)."""
    if not ctx.distributed:
        return local
    mx = max(counts)
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    if local.shape[0]:
        pad[: local.shape[0]] = local
    pad = _wire(ctx, pad)
    bufs = [torch.empty_like(pad) for _ in range(ctx.world)]
    dist.all_gather(bufs, pad)
    return torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0).to(local.device)


class NativeComm:
    """RCCL communicator owned by libgpfit (``gp_comm_*``, include/gpfit.h): the C-ABI route
    for the one broadcast + one gather the sharded emulator needs.

    The 128-byte RCCL id is made on rank 0 and travels over the existing torch.distributed
    group (any backend); at world size 1 no group is needed.
    """

    def __init__(self, ctx: Context):
        import ctypes

        from . import _capi
        self.ctx = ctx
        if not _capi.lib().gp_comm_available():
            raise _capi.GPFitUnavailable("librccl cannot be loaded: gp_comm_* unavailable")
        uid = (ctypes.c_char * 128)()
        if ctx.rank == 0:
            _capi.call("gp_comm_unique_id", ctypes.addressof(uid))
        if ctx.distributed:
            dev = ctx.device if ctx.backend == "nccl" else torch.device("cpu")
            t = torch.tensor(list(uid.raw), dtype=torch.uint8, device=dev)
            dist.broadcast(t, src=0)
            ctypes.memmove(uid, bytes(t.cpu().tolist()), 128)
        self._handle = ctypes.c_void_p()
        _capi.call("gp_comm_init", ctx.world, ctx.rank, ctypes.addressof(uid),
                   ctypes.addressof(self._handle))

    def _stream(self) -> int:
        return torch.cuda.current_stream(self.ctx.device).cuda_stream

    def bcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        """In-place broadcast of a contiguous device tensor from ``root``."""
        from . import _capi
        assert t.is_cuda and t.is_contiguous()
        _capi.call("gp_bcast", self._handle.value, t.data_ptr(), t.numel() * t.element_size(),
                   root, self._stream())
        return t

    def gather(self, t: torch.Tensor, root: int = 0) -> torch.Tensor | None:
        """Equal-shape tensors from every rank, stacked on ``root`` (None elsewhere)."""
        from . import _capi
        assert t.is_cuda and t.is_contiguous()
        out = (torch.empty((self.ctx.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
               if self.ctx.rank == root else None)
        _capi.call("gp_gather", self._handle.value, t.data_ptr(), t.numel() * t.element_size(),
                   out.data_ptr() if out is not None else None, root, self._stream())
        return out

    def close(self) -> None:
        from . import _capi
        if self._handle.value:
            _capi.call("gp_comm_destroy", self._handle.value)
            self._handle.value = None
