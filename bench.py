"""Benchmark: LRS-PnP outer ADMM iterations/sec on the BASELINE.json configs[1] workload.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--cube 200x200x198] [--bb 8] [--nit 80]

One "step" = one outer ADMM iteration of main_LRS_PnP.py (:250-366) over a whole synthetic
200x200x198 cube: im2col of X + L1/mu1, fused masked ISTA + PnP-NLM prox over all 125,000 8x8
blocks (Nit = 80, K = 256), SVT low-rank prox (concurrent stream), col2im + X + dual updates.
Inputs are resident in HBM before the timed region.

Multi-GPU (torchrun): one independent cube per rank (seed = rank), no data-path collective
(weak scaling); barrier + synchronize around the K timed steps, MAX over ranks;
value = (ranks * K) / max_time.  With --split-cube: ONE cube (seed 0) in pixel-row slabs, one per
rank, with an fp64 all-reduce of the B x B SVT Gram per iteration (strong scaling, value =
K / max_time; lrspnp.dist.slab_solver).

Rank 0 prints one JSON line, including
  roofline    : the dominant kernel (lrs_ista_f32 / k_ista_b3) — algorithmic fp32-GEMM FLOPs per
                launch (Nit*nb*4*n*K + nb*2*n*K) / mean launch time (HIP events on its stream), vs
                the 157.3 TFLOP/s fp32 MFMA peak (the products are fp32-accurate split-bf16 MFMA;
                the kernel itself is bound by the fp64 NLM VALU); `traffic` from
                profiles/ PMC summary when present;
  cpu_baseline: the oracle (C restatement + numpy alpha/SVT, OpenMP) timed on a bounded sample
                of the same workload on this host (N = 1, rank 0 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "lrs-pnp-dip_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md chip table
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cube", default="200x200x198")
    ap.add_argument("--bb", type=int, default=8)
    ap.add_argument("--nit", type=int, default=80)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group: nccl (= RCCL, one GPU per rank) or gloo (rehearsal: ranks may share a GPU)")
    ap.add_argument("--split-cube", action="store_true",
                    help="one cube over all ranks in pixel-row slabs (strong scaling; SVT Gram all-reduce)")
    ap.add_argument("--workload", default="pnp", choices=["pnp", "dip", "dip-pro"],
                    help="pnp: BASELINE configs[1] (the headline); dip: configs[2], LRS-PnP-DIP(1-Lip) on a "
                         "196x196x198 cube (the 200x200 cube cropped to a size the U-Net maps onto itself); "
                         "dip-pro: configs[3], LRS-PnP-DIP with the skip net on a 512x512x224 cube")
    ap.add_argument("--dip-steps", type=int, default=100, help="DIP steps per outer iteration (ES off, §8d)")
    return ap.parse_args()


def make_problem(H, W, B, bb, K, seed):
    from lrspnp.data import load_fixture, mask_matrix, synthetic_cube, synthetic_dictionary, unfold
    base = load_fixture("data_img5.npz")["lrs_mask"]
    obs, clean, mask = synthetic_cube(H, W, B, seed=seed, base_mask=base)
    return unfold(obs), mask_matrix(mask, B), synthetic_dictionary(bb * bb, K, 0), clean


def cpu_baseline(Y, M, D, bb, nit, budget_s):
    """Oracle timed on a bounded sample of the same workload (host cores)."""
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    os.environ["OMP_NUM_THREADS"] = str(threads)
    P, B = Y.shape
    rows, cols = O.block_grid(P, B, bb, bb)
    nb = rows.size
    rng = np.random.default_rng(0)
    # per-block cost: alpha (numpy float32 SVD of the pruned dictionary, as ista() does per call)
    # + the C ISTA (GEMVs + NLM) — grow the sample until the budget is used
    blocks = O.im2col(Y, bb, rows, cols)
    obs = (blocks != 0).astype(np.uint8)
    done, t_ista, t_alpha = 0, 0.0, 0.0
    batch = 256
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < budget_s * 0.7 and done < nb:
        idx = rng.choice(nb, batch, replace=False)
        t0 = time.perf_counter()
        al = np.empty(batch, np.float32)
        th = np.empty(batch, np.float64)
        for k, j in enumerate(idx):
            al[k], th[k] = O.ista_alpha_h(D[obs[j].astype(bool)], 0.1, "spec2")
        t1 = time.perf_counter()
        O.ista_batch(blocks[idx], obs[idx], D, al, th, nit)
        t2 = time.perf_counter()
        t_alpha += t1 - t0
        t_ista += t2 - t1
        done += batch
    per_block = (t_alpha + t_ista) / done
    t0 = time.perf_counter()
    U = O.svt(Y, 1 / 0.9)                                   # the reference's float32 LAPACK SVT
    t_svt = time.perf_counter() - t0
    X = Y.copy()
    PHI = np.zeros((nb, bb * bb), np.float32)
    t0 = time.perf_counter()
    O.lib().oracle_admm_update(P, B, bb, nb, rows, cols, PHI, Y, M, U, X, X, 0.5, np.float32(0.15),
                               np.float32(0.9), X.copy(), X.copy(), X.copy(), None, None)
    t_admm = time.perf_counter() - t0
    t_iter = per_block * nb + t_svt + t_admm
    return {"value": 1.0 / t_iter, "unit": "outer_iters/s", "cores": threads, "kind": "port",
            "sample": f"{done} of {nb} blocks (alpha+ISTA, Nit={nit}) extrapolated x{nb / done:.1f}, "
                      f"+ full SVT ({t_svt:.2f}s) + full ADMM update ({t_admm:.3f}s); "
                      f"est. {t_iter:.1f}s per outer iteration"}


def dip_flops_per_step(net):
    """Algorithmic MFMA FLOPs of one DIP training step of a DipNet: conv forward + dW + dX (no dX
    for a conv reading the network input)."""
    sh = [net.in_shape] + list(net.shapes)
    tot = 0
    for i, nd in enumerate(net.nodes):
        if nd.kind != 0:
            continue
        co, ho, wo = sh[i + 1]
        f = 2 * co * sh[nd.in0][0] * nd.k * nd.k * ho * wo
        tot += f * (2 if nd.in0 == 0 else 3)
    return tot


def main_dip(args):
    import torch

    from lrspnp import LrsPnP, LrsPnPConfig
    from lrspnp import dist as D
    from lrspnp.dip import DipConfig
    from lrspnp.metrics import mpsnr
    ctx = D.init_from_env(args.backend)
    pro = args.workload == "dip-pro"
    H = W = 512 if pro else 196
    B = 224 if pro else 198
    bb = 36 if args.bb == 8 else args.bb
    Y, M, Dct, clean = make_problem(H, W, B, bb, args.K, seed=ctx.rank)
    dcfg = DipConfig(num_iter=args.dip_steps, early_stop=False, net="skip" if pro else "unet1lip")
    cfg = (LrsPnPConfig.dip_pro if pro else LrsPnPConfig.dip_1lip)(bb=bb, sliding=bb, dip=dcfg)
    s = LrsPnP(Y, M, Dct, cfg, image_shape=(H, W))
    clean_d = torch.from_numpy(clean).cuda()
    mp0 = mpsnr(s.X, clean_d)
    # DIP training time per outer iteration: events on the low-rank stream around the DIP call
    ev = []
    orig = s.low_rank_dip

    def timed(stream):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        orig(stream)
        e1.record(stream)
        ev.append((e0, e1))

    s.low_rank_dip = timed
    elapsed = D.timed_steps(s.step, args.steps, args.warmup, ctx)
    dip_ms = float(np.mean([a.elapsed_time(b) for a, b in ev[args.warmup:]]))
    mp1 = mpsnr(s.X, clean_d)
    flops = dip_flops_per_step(s.dip.net) * args.dip_steps
    achieved = flops / (dip_ms * 1e-3) / 1e12
    out = {
        "metric": METRIC, "value": ctx.world * args.steps / elapsed, "unit": "outer_iters/s",
        "n_gpus": ctx.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32 (MFMA) + f64 (NLM, BN/sigma statistics)",
        "data": f"synthetic (seeded low-rank {H}x{W}x{B} cube per rank, random-init DIP net per outer iteration)",
        "config": {"workload": (f"LRS-PnP-DIP(pro) {H}x{W}x{B}, {bb}x{bb} blocks, K={args.K}, Nit=100 fro4 ISTA, "
                                f"DIP skip net (5x128 ch, 128 skips) {args.dip_steps} Adam steps, ES off "
                                "(BASELINE configs[3])") if pro else
                               (f"LRS-PnP-DIP(1-Lip) 196x196x198, {bb}x{bb} blocks, K={args.K}, Nit=100 fro4 ISTA, "
                                f"DIP my_Lipschitz_Unet (198->128->198 ch) {args.dip_steps} Adam steps, ES off "
                                "(BASELINE configs[2])"), "blocks": s.nb,
                   "parallelism": f"{ctx.world} independent cube(s), one per GPU"},
        "roofline": {"bound": "mfma", "kernel": "DIP training (conv GEMMs + BN/sigma/Adam kernels)",
                     "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP32_MFMA_PEAK_TFLOPS, "traffic": None,
                     "flops_per_outer_iter": flops, "dip_ms_per_outer_iter": dip_ms},
        "mpsnr": {"input": mp0, "after_steps": mp1, "steps_run": args.warmup + args.steps},
    }
    if ctx.rank == 0:
        print(json.dumps(out), flush=True)


def main():
    args = parse()
    if args.workload in ("dip", "dip-pro"):
        return main_dip(args)
    import torch

    from lrspnp import dist as D
    ctx = D.init_from_env(args.backend)
    from lrspnp import LrsPnP, LrsPnPConfig, ops
    from lrspnp.metrics import mpsnr

    H, W, B = (int(v) for v in args.cube.split("x"))
    split = args.split_cube
    # one cube per rank (seed = rank), or with --split-cube one cube (seed 0) in row slabs
    Y, M, Dct, clean = make_problem(H, W, B, args.bb, args.K, seed=0 if split else ctx.rank)
    cfg = LrsPnPConfig(bb=args.bb, sliding=args.bb, Nit=args.nit, variant="spec2")
    t0 = time.perf_counter()
    if split:
        s, _ = D.slab_solver(Y, M, Dct, cfg, ctx)
    else:
        s = LrsPnP(Y, M, Dct, cfg)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    clean_d = torch.from_numpy(clean).cuda()

    def cube_mpsnr():
        if not split:
            return mpsnr(s.X, clean_d)
        X = D.gather_rows(s.X, ctx)
        return mpsnr(torch.from_numpy(X).cuda(), clean_d) if X is not None else float("nan")

    mp0 = cube_mpsnr()

    # dominant-kernel timing: HIP events on the stream the ISTA kernel is launched on
    ev = []
    orig_ista = ops.ista
    timing = [False]

    def timed_ista(*a, **k):
        st = k.get("stream") or torch.cuda.current_stream()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        out = orig_ista(*a, **k)
        e1.record(st)
        if timing[0]:
            ev.append((e0, e1))
        return out

    ops.ista = timed_ista

    def step():
        if not timing[0] and warm_done[0] >= args.warmup:
            timing[0] = True
        warm_done[0] += 1
        s.step()

    warm_done = [0]
    elapsed = D.timed_steps(step, args.steps, args.warmup, ctx)
    ops.ista = orig_ista
    ista_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    mp1 = cube_mpsnr()
    world, rank = ctx.world, ctx.rank
    mps = [[mp0, mp1]] if split else D.gather_scalars([mp0, mp1], ctx)   # split: one cube, MPSNR on rank 0

    n, K, nb = args.bb * args.bb, args.K, s.nb
    flops = args.nit * nb * 4 * n * K + nb * 2 * n * K
    achieved = flops / (ista_ms * 1e-3) / 1e12
    traffic = None
    prof = os.path.join(REPO, "profiles", "ista_pmc_traffic.json")
    if os.path.exists(prof):
        try:
            traffic = json.load(open(prof)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    out = {
        "metric": METRIC,
        "value": (1 if split else world) * args.steps / elapsed,
        "unit": "outer_iters/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if split else "weak",
        "vs_baseline": None,
        "dtype": "f32 (MFMA) + f64 (NLM prox, Gram/eig)",
        "data": "synthetic (seeded low-rank cube per rank, tiled low_rank_sparsity_mask, seeded K=256 dictionary)",
        "config": {"workload": f"LRS-PnP (no DIP) {args.cube} cube, {args.bb}x{args.bb} blocks, K={K}, "
                               f"Nit={args.nit} inner ISTA, SVT low-rank prox (BASELINE configs[1])",
                   "blocks": int(ops.block_grid(Y.shape[0], B, args.bb, args.bb)[0].size),
                   "parallelism": (f"1 cube in {world} pixel-row slab(s), fp64 Gram all-reduce per iteration"
                                   if split else f"{world} independent cube(s), one per GPU")},
        "roofline": {"bound": "mfma", "kernel": "k_ista_ln2 (lrs_ista_f32)", "achieved": achieved,
                     "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": achieved / FP32_MFMA_PEAK_TFLOPS,
                     "traffic": traffic, "flops_per_launch": flops, "ms_per_launch": ista_ms},
        "setup_s": setup_s,
        "mpsnr": {"input": mp0, "after_steps": mp1, "steps_run": args.warmup + args.steps,
                  "per_rank": mps},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(Y, M, Dct, args.bb, args.nit, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as tdist
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
