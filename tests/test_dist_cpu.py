"""The N>1 harness on CPU: world_size-2 gloo process group on 127.0.0.1 (bench.py's path without
the GPU): sharding, barrier-bracketed timing with MAX over ranks, scalar gather."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "lrs-pnp-dip_amd")]
    import time

    import torch.distributed as dist

    from lrspnp import dist as D
    ctx = D.init_from_env("gloo")
    units = list(D.shard_units(8, ctx))
    calls = []

    def step():
        calls.append(1)
        time.sleep(0.01 * (rank + 1))     # rank 1 is the slow one

    el = D.timed_steps(step, steps=3, warmup=1, ctx=ctx, sync=lambda: None)
    got = D.gather_scalars([float(rank), float(len(units))], ctx)
    q.put((rank, units, el, len(calls), got))
    dist.destroy_process_group()


def test_gloo_world2_harness():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, u0, e0, c0, g0), (r1, u1, e1, c1, g1) = res
    assert u0 == [0, 1, 2, 3] and u1 == [4, 5, 6, 7]
    assert c0 == c1 == 4
    assert e0 == e1 and e0 >= 0.06              # MAX over ranks: both see rank 1's 3 x 20 ms
    assert g0 == [[0.0, 4.0], [1.0, 4.0]] and g1 is None


def test_shard_units_uneven():
    from lrspnp.dist import Ctx, shard_units
    parts = [list(shard_units(10, Ctx(rank=r, world=4))) for r in range(4)]
    assert parts == [[0, 1, 2], [3, 4, 5], [6, 7], [8, 9]]


# ---- one cube in pixel-row slabs (lrspnp.dist.slab_rows / SlabComm) -------------

@pytest.mark.parametrize("P,bb,world", [(40000, 8, 2), (40000, 8, 8), (1296, 36, 2), (38416, 36, 8),
                                        (1300, 36, 3), (203, 8, 4), (64, 8, 8)])
def test_slab_blocks_are_the_cube_blocks(P, bb, world):
    """The blocks of the slabs (shifted by p0) are exactly get_image_block's blocks of the cube
    (main_LRS_PnP.py:73-107), each once, including the appended P - bb row."""
    import numpy as np

    from lrspnp import dist as D
    from lrspnp import ops
    B = 198
    rows, cols = ops.block_grid(P, B, bb, bb)
    want = sorted(zip(rows.tolist(), cols.tolist()))
    got, edge = [], 0
    for r in range(world):
        p0, p1 = D.slab_rows(P, bb, r, world)
        assert p0 == edge and p1 - p0 >= bb and p0 % bb == 0
        edge = p1
        lr, lc = ops.block_grid(p1 - p0, B, bb, bb)
        got += list(zip((lr + p0).tolist(), lc.tolist()))
    assert edge == P
    assert sorted(got) == want and len(got) == len(set(got)) == rows.size


def _slab_svt_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [repo, os.path.join(repo, "lrs-pnp-dip_amd")]
    import numpy as np
    import torch.distributed as dist

    from lrspnp import dist as D
    ctx = D.init_from_env("gloo")
    rng = np.random.default_rng(3)
    Z = (rng.standard_normal((200, 6)) @ rng.standard_normal((6, 30)) + 0.1 * rng.standard_normal((200, 30)))
    Z = Z.astype(np.float32)
    p0, p1 = D.slab_rows(Z.shape[0], 8, rank, world)
    Zs = Z[p0:p1].astype(np.float64)
    G = torch.from_numpy(Zs.T @ Zs)
    D.SlabComm(ctx).allreduce_(G, None)            # the cube's Gram from the slabs' Grams
    lam, V = np.linalg.eigh(G.numpy())
    s = np.sqrt(np.maximum(lam, 0.0))
    tau = 1.1
    f = np.where(s > tau, (s - tau) / np.where(s > 0, s, 1.0), 0.0)
    Us = (Zs @ (V * f) @ V.T).astype(np.float32)  # SVT of the slab rows: Z V diag(f) V^T
    full = D.gather_rows(torch.from_numpy(Us), ctx)
    q.put((rank, None if full is None else full.tolist(), Z.tolist(), tau))
    dist.destroy_process_group()


def test_gloo_world2_slab_svt_matches_oracle():
    """Row-slab SVT (per-rank Gram, sum all-reduce, the same eig on every rank, local apply)
    equals the oracle's whole-matrix SVT (main_LRS_PnP.py:118-124)."""
    import numpy as np

    from oracle import oracle as O
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_slab_svt_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in range(world)), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full, Z, tau = np.array(res[0][1], np.float32), np.array(res[0][2], np.float32), res[0][3]
    assert res[1][1] is None
    ref = O.svt(Z, tau)
    assert np.linalg.norm(full - ref) / np.linalg.norm(ref) < 1e-5
