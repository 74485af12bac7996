"""One process per GPU over torch.distributed (backend "nccl" = RCCL on ROCm, "gloo" on CPU).

The GP emulator shards without a data-path exchange:
  * multivariate emulator (C4/C5): the P x S independent (sample, PC) GPs are dealt
    round-robin to ranks; inputs are broadcast once from rank 0, per-rank (mean, var) blocks are
    gathered to rank 0 once at the end;
  * single-output GP (C2/C3): every rank factorises the same n x n Gram redundantly (~1 ms at
    n = 4096) and predicts its own block of test points.

The reference has no distributed code at all (SLURM job arrays of the external
simulator only), so there is no call pattern to mirror; collectives here are the minimum the
sharding needs: one broadcast of the inputs and one gather of the outputs.
"""
from __future__ import annotations

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


def init_from_env(device_type: str | None = None) -> Context:
    """Join the process group described by RANK/WORLD_SIZE/MASTER_* (torchrun), if any."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if device_type == "cuda":
        torch.cuda.set_device(local_rank)
        device = torch.device("cuda", local_rank)
    else:
        device = torch.device("cpu")
    backend = None
    if world > 1:
        backend = "nccl" if device_type == "cuda" else "gloo"
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            kw = {"device_id": device} if device_type == "cuda" else {}
            dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
    return Context(rank, world, local_rank, device, backend)


def barrier(ctx: Context) -> None:
    if ctx.distributed:
        if ctx.device.type == "cuda":
            dist.barrier(device_ids=[ctx.local_rank])
        else:
            dist.barrier()


def max_over_ranks(ctx: Context, value: float) -> float:
    if not ctx.distributed:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=ctx.device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def broadcast_(ctx: Context, t: torch.Tensor, src: int = 0) -> torch.Tensor:
    """In-place broadcast of ``t`` from ``src`` (RCCL over xGMI on the GPU path)."""
    if ctx.distributed:
        dist.broadcast(t, src=src)
    return t


def shard_units(n_units: int, rank: int, world: int) -> list[int]:
    """Round-robin deal of independent units (PC GPs, samples) to ranks."""
    return list(range(rank, n_units, world))


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous block [a, b) of n items for ``rank`` (balanced to within one item)."""
    q, r = divmod(n, world)
    a = rank * q + min(rank, r)
    return a, a + q + (1 if rank < r else 0)


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
    bufs = [torch.empty_like(pad) for _ in range(ctx.world)] if ctx.rank == 0 else None
    dist.gather(pad, gather_list=bufs, dst=0)
    if ctx.rank != 0:
        return None
    return torch.cat([b[:c] for b, c in zip(bufs, counts)], dim=0)


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
