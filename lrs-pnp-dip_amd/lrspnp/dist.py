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
    elif torch.cuda.is_available():
        # gloo rehearsal: ranks spread over the visible GPUs (LOCAL_RANK mod count), so on a
        # 1-GPU box they share cuda:0 and on a multi-GPU node each rank still gets its own card
        torch.cuda.set_device(local % torch.cuda.device_count())
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


# ---- one cube over several ranks: pixel-row slabs ("single cube") -----------------
#
# The unfolded cube X (P x B, p = i + H j) is cut into row slabs aligned to the block size. With
# slidingDis == bb (every reference main: main_LRS_PnP.py:237-238) the blocks of a slab are exactly
# the cube's blocks over those rows (get_image_block, main_LRS_PnP.py:73-107: the extra block row
# at P - bb when bb does not divide P belongs to the last slab), so the sparse coding, col2im and
# X / dual updates are slab-local. The only coupled step is the SVT: its Gram is the sum of the
# slabs' Grams (B x B fp64, one all-reduce per outer iteration), after which every rank runs the
# same eigensolver and applies U = Z (I - E) to its own rows.


def slab_rows(P: int, bb: int, rank: int, world: int) -> tuple[int, int]:
    """[p0, p1) of rank's slab: whole block rows of bb pixels, split as evenly as possible; the
    last slab also takes the P % bb tail rows (whose appended block starts at P - bb)."""
    nfull = P // bb
    if nfull < world:
        raise ValueError(f"{P} rows in blocks of {bb} give {nfull} block rows, fewer than {world} ranks")
    base, extra = divmod(nfull, world)
    r0 = rank * base + min(rank, extra)
    r1 = r0 + base + (1 if rank < extra else 0)
    return r0 * bb, (P if rank == world - 1 else r1 * bb)


class SlabComm:
    """Sum-all-reduce of device tensors for a row-slab shard, stream-ordered.

    nccl (RCCL over xGMI on the box): the collective is enqueued behind `stream`'s work and
    later work on `stream` waits for it; the host does not block. gloo (CPU tests, or several
    ranks sharing one GPU): the tensor is staged through host memory after `stream` drains."""

    def __init__(self, ctx: Ctx):
        self.ctx = ctx

    def allreduce_(self, t: torch.Tensor, stream) -> None:
        if not self.ctx.distributed:
            return
        if dist.get_backend() == "nccl":
            with torch.cuda.stream(stream):
                dist.all_reduce(t)
            return
        if t.is_cuda:
            stream.synchronize()
            h = t.cpu()
            dist.all_reduce(h)
            with torch.cuda.stream(stream):
                t.copy_(h)
        else:
            dist.all_reduce(t)


def slab_solver(Y, M, D, cfg, ctx: Ctx, device="cuda"):
    """This rank's LrsPnP over its row slab of the whole-cube inputs Y, M (P x B, host arrays);
    returns (solver, (p0, p1))."""
    from .solver import LrsPnP
    if cfg.sliding != cfg.bb:
        raise ValueError("row-slab sharding needs slidingDis == bb")
    P = Y.shape[0]
    p0, p1 = slab_rows(P, cfg.bb, ctx.rank, ctx.world)
    comm = SlabComm(ctx) if ctx.distributed else None
    return LrsPnP(Y[p0:p1], M[p0:p1], D, cfg, device=device, comm=comm), (p0, p1)


def gather_rows(X: torch.Tensor, ctx: Ctx):
    """The whole unfolded matrix from the ranks' row slabs, on rank 0 (numpy; None elsewhere).
    Outside any timed region.  A tensor gather (slabs padded to the largest, sizes exchanged
    first): RCCL on the device under nccl, host tensors under gloo; no pickling."""
    import numpy as np
    if not ctx.distributed:
        return X.detach().cpu().numpy()
    nccl = dist.get_backend() == "nccl"
    dev = X.device if nccl else torch.device("cpu")
    rows = torch.tensor([X.shape[0]], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(rows) for _ in range(ctx.world)]
    dist.all_gather(sizes, rows)
    sizes = [int(v.item()) for v in sizes]
    mx = max(sizes)
    mine = torch.zeros((mx,) + tuple(X.shape[1:]), dtype=X.dtype, device=dev)
    mine[: X.shape[0]].copy_(X.detach())
    parts = [torch.empty_like(mine) for _ in range(ctx.world)] if ctx.rank == 0 else None
    dist.gather(mine, parts, dst=0)
    if ctx.rank != 0:
        return None
    return np.concatenate([p[:n].cpu().numpy() for p, n in zip(parts, sizes)], axis=0)


# ---- one cube, task-parallel DIP ("DIP on GPU 0, sparse coding sharded over the rest") --
#
# In the DIP mains the two proxes of an outer iteration read the same iterate (sparse coding: X +
# lambda_1 / mu_1, …1-LiP.py:362-392; DIP: X + lambda_2 / mu_2, :399-411), so they are independent:
# rank 0 trains the DIP (batch 1, not data-parallel), ranks 1..W-1 code contiguous block ranges.
# Every rank keeps the whole (replicated) cube state; per outer iteration rank 0 broadcasts U
# (P x B floats) and the workers' Phi rows are all-gathered (nb x n_pad floats), after which every
# rank applies the same deterministic ADMM update.  With one rank it is the ordinary step.


class DipTaskSplit:
    def __init__(self, Y, M, D, cfg, ctx: Ctx, image_shape, device="cuda"):
        from .solver import LrsPnP
        if cfg.lowrank != "dip":
            raise ValueError("DipTaskSplit needs a DIP configuration (LrsPnPConfig.dip_1lip / dip_pro)")
        self.ctx = ctx
        # only rank 0 trains the DIP: the workers keep the cube state but build no network engine
        self.s = LrsPnP(Y, M, D, cfg, device=device, image_shape=image_shape,
                        dip_engine=ctx.rank == 0 or ctx.world == 1)
        nb, W = self.s.nb, ctx.world
        self.ranges = [(0, 0)] * W
        if W > 1:
            base, extra = divmod(nb, W - 1)
            b = 0
            for r in range(1, W):
                c = base + (1 if r - 1 < extra else 0)
                self.ranges[r] = (b, b + c)
                b += c
        self.maxc = max(b1 - b0 for b0, b1 in self.ranges) if W > 1 else nb
        n_pad = self.s.phi.shape[1]
        self.mine = torch.zeros((self.maxc, n_pad), dtype=torch.float32, device=self.s.phi.device)
        self.buf = None
        self.comm_stream = torch.cuda.Stream(device=self.s.phi.device) if W > 1 else None

    def _gather_phi(self, comm):
        """The workers' Phi rows to every rank.  Under nccl it is enqueued on the comm stream as soon
        as this rank's rows exist, so on rank 0 it runs beside the DIP training."""
        s, ctx = self.s, self.ctx
        b0, b1 = self.ranges[ctx.rank]
        n_pad = s.phi.shape[1]
        if dist.get_backend() == "nccl":
            if self.buf is None:
                self.buf = torch.empty((ctx.world * self.maxc, n_pad), dtype=torch.float32, device=s.phi.device)
            with torch.cuda.stream(comm):
                if b1 > b0:
                    self.mine[: b1 - b0].copy_(s.phi[b0:b1])
                dist.all_gather_into_tensor(self.buf, self.mine)
            return self.buf.view(ctx.world, self.maxc, n_pad)
        comm.synchronize()
        if b1 > b0:
            self.mine[: b1 - b0].copy_(s.phi[b0:b1])
        hs = [torch.empty((self.maxc, n_pad), dtype=torch.float32) for _ in range(ctx.world)]
        dist.all_gather(hs, self.mine.cpu())
        return hs

    def _broadcast_u(self, comm):
        s = self.s
        if dist.get_backend() == "nccl":
            with torch.cuda.stream(comm):
                dist.broadcast(s.U, src=0)
        else:
            comm.synchronize()
            h = s.U.cpu()
            dist.broadcast(h, src=0)
            s.U.copy_(h)

    def step(self):
        s, ctx = self.s, self.ctx
        main = torch.cuda.current_stream()
        if ctx.world == 1:
            return s.step()
        comm = self.comm_stream
        if ctx.rank == 0:
            lr = s.lowrank_stream
            lr.wait_stream(main)
            comm.wait_stream(main)
            if dist.get_backend() == "nccl":
                # the RCCL all-gather is enqueued first so it runs beside the DIP training (rank 0
                # contributes no rows); the multi-rank overlap is unmeasured on hardware
                parts = self._gather_phi(comm)
                s.low_rank_dip(lr)
            else:
                # gloo's gather blocks the host until the workers finish: train the DIP first, so it
                # still overlaps the workers' sparse coding
                s.low_rank_dip(lr)
                parts = self._gather_phi(comm)
            comm.wait_stream(lr)
        else:
            b0, b1 = self.ranges[ctx.rank]
            s.sparse_coding_range(b0, b1, stream=main)
            comm.wait_stream(main)
            parts = self._gather_phi(comm)
        self._broadcast_u(comm)
        main.wait_stream(comm)
        for r, (c0, c1) in enumerate(self.ranges):
            if c1 > c0:
                s.phi[c0:c1].copy_(parts[r][: c1 - c0], non_blocking=True)
        s.admm(main)
