"""One-process-per-GPU harness (torch.distributed over RCCL on the box, gloo in CPU tests).

The LRS-PnP hot path shards without a data-path exchange: independent cubes (or
tiles) go one per rank, so the only collectives are timing/metric reductions:
  * barrier around the timed region,
  * MAX of the per-rank elapsed time (the job's wall time),
  * gather of per-rank scalars (MPSNR, convergence) to rank 0.
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class Ctx:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device | None = None

    @property
    def distributed(self) -> bool:
        return self.world > 1


def init_from_env(backend: str = "nccl") -> Ctx:
    """Read RANK/WORLD_SIZE/LOCAL_RANK (torchrun) and join the process group when world > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = None
    if backend == "nccl":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    if world > 1 and not dist.is_initialized():
        kw = {"device_id": dev} if (backend == "nccl" and dev is not None) else {}
        dist.init_process_group(backend, **kw)
    return Ctx(rank, world, local, dev)


def shard_units(n_units: int, ctx: Ctx) -> range:
    """Contiguous share of n_units for this rank (weak scaling uses one unit per rank)."""
    base, extra = divmod(n_units, ctx.world)
    start = ctx.rank * base + min(ctx.rank, extra)
    return range(start, start + base + (1 if ctx.rank < extra else 0))


def timed_steps(step, steps: int, warmup: int, ctx: Ctx, sync=None) -> float:
    """Run `warmup` untimed then `steps` timed calls of step(); barrier + sync on both sides;
    returns the MAX elapsed seconds over ranks."""
    sync = sync or (torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None))
    for _ in range(warmup):
        step()
    sync()
    if ctx.distributed:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if ctx.distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    return max_over_ranks(elapsed, ctx)


def max_over_ranks(x: float, ctx: Ctx) -> float:
    if not ctx.distributed:
        return x
    dev = ctx.device if (ctx.device is not None and dist.get_backend() == "nccl") else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_scalars(values: list[float], ctx: Ctx) -> list[list[float]] | None:
    """All ranks' scalar lists, on rank 0 (None elsewhere)."""
    if not ctx.distributed:
        return [list(values)]
    out = [None] * ctx.world
    dist.all_gather_object(out, list(values))
    return out if ctx.rank == 0 else None
