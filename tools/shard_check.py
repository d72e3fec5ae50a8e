"""Row-slab sharding of one cube vs the whole-cube solver, on the GPU (run under torchrun).

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P \
        tools/shard_check.py [--backend gloo] [--cube 96x64x40] [--steps 3]

Every rank solves its pixel-row slab (lrspnp.dist.slab_solver; the SVT Gram is all-reduced each
outer iteration); rank 0 also runs the unsharded LrsPnP on the same cube and prints one JSON line
with the relative L2 differences of X, lambda_1, lambda_2 and the convergence norms. With
--backend gloo several ranks can share one GPU (the test path on the 1-GPU box).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--cube", default="96x64x40")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--bb", type=int, default=8)
    ap.add_argument("--nit", type=int, default=20)
    ap.add_argument("--dip", type=int, default=0, help="> 0: task-parallel DIP (DIP steps per outer iteration)")
    a = ap.parse_args()
    from lrspnp import LrsPnP, LrsPnPConfig
    from lrspnp import dist as D
    from lrspnp.data import mask_matrix, synthetic_cube, synthetic_dictionary, unfold
    if a.backend == "gloo":
        torch.cuda.set_device(0)
    ctx = D.init_from_env(a.backend)
    H, W, B = (int(v) for v in a.cube.split("x"))
    obs, clean, mask = synthetic_cube(H, W, B, seed=5)
    Y, M = unfold(obs), mask_matrix(mask, B)
    Dct = synthetic_dictionary(a.bb * a.bb, 256, 0)
    if a.dip:
        return dip_split(a, ctx, H, W, Y, M, Dct)
    cfg = LrsPnPConfig(bb=a.bb, sliding=a.bb, Nit=a.nit)
    s, (p0, p1) = D.slab_solver(Y, M, Dct, cfg, ctx)
    for _ in range(a.steps):
        s.step()
    conv = s.convergence()
    X, L1, L2 = (D.gather_rows(t, ctx) for t in (s.X, s.L1, s.L2))
    if ctx.rank == 0:
        r = LrsPnP(Y, M, Dct, cfg)
        for _ in range(a.steps):
            r.step()
        rel = lambda u, v: float(np.linalg.norm(u - v.cpu().numpy()) / max(np.linalg.norm(v.cpu().numpy()), 1e-30))
        out = {"world": ctx.world, "cube": a.cube, "steps": a.steps, "rel_X": rel(X, r.X), "rel_L1": rel(L1, r.L1),
               "rel_L2": rel(L2, r.L2), "conv_sharded": conv, "conv_whole": r.convergence(),
               "X_bitwise_equal": bool(np.array_equal(X, r.X.cpu().numpy()))}
        print(json.dumps(out), flush=True)
    if ctx.distributed:
        torch.distributed.destroy_process_group()


def dip_split(a, ctx, H, W, Y, M, Dct):
    """Task-parallel DIP (lrspnp.dist.DipTaskSplit) vs the one-rank DIP solver on rank 0."""
    from lrspnp import LrsPnP, LrsPnPConfig
    from lrspnp import dist as D
    from lrspnp.dip import DipConfig
    cfg = LrsPnPConfig.dip_1lip(bb=a.bb, sliding=a.bb, Nit=a.nit, dip=DipConfig(num_iter=a.dip, early_stop=False))
    t = D.DipTaskSplit(Y, M, Dct, cfg, ctx, image_shape=(H, W))
    for _ in range(a.steps):
        t.step()
    torch.cuda.synchronize()
    if ctx.rank == 0:
        r = LrsPnP(Y, M, Dct, cfg, image_shape=(H, W))
        for _ in range(a.steps):
            r.step()
        torch.cuda.synchronize()
        rel = lambda u, v: float((u - v).norm() / max(float(v.norm()), 1e-30))
        out = {"world": ctx.world, "cube": a.cube, "steps": a.steps, "dip_steps": a.dip, "rel_X": rel(t.s.X, r.X),
               "rel_L1": rel(t.s.L1, r.L1), "rel_L2": rel(t.s.L2, r.L2), "rel_U": rel(t.s.U, r.U),
               "X_bitwise_equal": bool(torch.equal(t.s.X, r.X)), "ranges": t.ranges}
        print(json.dumps(out), flush=True)
    if ctx.distributed:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
