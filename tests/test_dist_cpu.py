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
