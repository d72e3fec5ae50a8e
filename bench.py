"""Benchmark: LRS-PnP-DIP outer ADMM iterations/sec (BASELINE.json `metric`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload dip|pnp|dip-pro]

One "step" = one outer ADMM iteration over a whole synthetic cube, inputs resident in HBM:

  dip (default, BASELINE configs[2]) — main_LRS_PnP_DIP_1-LiP.py:347-520 on the seeded
      200x200x198 cube cropped to 196x196x198 (the largest size <= 200 that my_Lipschitz_Unet maps
      onto itself: 16a-12): im2col of X + L1/mu1, fused masked ISTA + NLM prox
      over 6,408 36x36 blocks (Nit 100, alpha = 4||H||_F^2), and — concurrently, on a second
      stream — the DIP low-rank prox: a fresh 1-Lipschitz U-Net (198 -> 128 -> 198 channels)
      trained for 100 Adam steps (lr 0.1, ES off: SURVEY.md §8d fixes N_dip = 100 for timing),
      then col2im + closed-form X + dual updates (get_DIP_out :208-264, X update :420-453).
  pnp (configs[1]) — main_LRS_PnP.py:250-366 on the 200x200x198 cube: 125,000 8x8 blocks,
      Nit 80, alpha = ||H||_2^2, SVT low-rank prox.
  dip-pro (configs[3]; with N ranks configs[4]) — main_LRS_PnP_DIP_pro.py on 512x512x224:
      50,974 36x36 blocks, the skip network DIP.

Multi-GPU (one process per GPU, RCCL): one independent cube per rank (seed = rank), no data-path
collective; barrier + synchronize around the K timed steps, MAX over ranks;
value = ranks * K / max_time ("weak").  `--gpus N` without a torchrun environment starts N ranks
itself (a child torch.distributed.run, before any GPU call); a rank count that differs from
--gpus is an error.  --split-cube runs ONE cube over the ranks ("strong"): pnp in pixel-row slabs
with an fp64 all-reduce of the B x B SVT Gram per iteration; dip / dip-pro task-parallel (DIP on
rank 0, the sparse coding's blocks over the other ranks, U broadcast + Phi all-gathered).

Rank 0 prints one JSON line with
  roofline     : the dominant stage — the DIP training of one outer iteration (dip workloads) or
                 the ISTA kernel (pnp): algorithmic MFMA FLOPs / time from HIP events on the stream
                 it runs on, vs the 157.3 TFLOP/s f32 MFMA peak; `traffic` = HBM bytes from the
                 committed rocprofv3 PMC pass (profiles/r06/traffic.json), per the same unit;
                 `peak_split_bf16` / `frac_split_bf16`: the same work against the split-bf16
                 matrix-core ceiling (6 bf16 MFMAs per fp32-accurate product).
                 `roofline.kernels` adds the sparse-coding kernel (k_ista_rs / k_ista_ln2) per launch.
  cpu_baseline : the oracle timed on this host (rank 0, N = 1): the C ISTA restatement on a bounded
                 block sample + (dip) the plain-torch DIP restatement (oracle/dip_ref.py) for a few
                 steps, both extrapolated to a full outer iteration, + the full ADMM update.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "lrs-pnp-dip_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
FP32_MFMA_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md chip table (f32 MFMA = f32 vector peak)
# The split-bf16 kernels (the DIP convs, k_ista_ln2) compute each fp32-accurate product as 6
# v_mfma_f32_16x16x32_bf16 (16 cycles per SIMD each, MI355X_MICROARCH.md cycle constants): 1024 FLOP
# per clock per SIMD x 4 x 256 CUs x 2.4 GHz = 2,517 TFLOP/s of bf16, / 6 = the ceiling of fp32-accurate
# work on the bf16 matrix cores.
SPLIT_BF16_PEAK_TFLOPS = 2516.6 / 6
TRAFFIC_FILE = os.path.join(REPO, "profiles", "r06", "traffic.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed outer iterations (default 3 dip, 10 pnp)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed outer iterations (default 1 dip, 2 pnp)")
    ap.add_argument("--workload", default="dip", choices=["dip", "pnp", "dip-pro"])
    ap.add_argument("--cube", default=None, help="HxWxB (default: the workload's cube)")
    ap.add_argument("--bb", type=int, default=None)
    ap.add_argument("--nit", type=int, default=None)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--dip-steps", type=int, default=100, help="DIP steps per outer iteration (ES off, §8d)")
    ap.add_argument("--early-stop", action="store_true",
                    help="the reference's early stopping on (buffer 30, patience 60, at most --dip-cap steps: "
                         "main_LRS_PnP_DIP_1-LiP.py:221-223,242-264,345): DIP steps vary per outer iteration")
    ap.add_argument("--dip-cap", type=int, default=5000, help="--early-stop: the step cap (the reference's dip_iter)")
    ap.add_argument("--data", default="synthetic", choices=["synthetic", "native"],
                    help="native: the reference's own 36x36x128 image (data_img5: noisy_img5 / clean_img5 + "
                         "low_rank_sparsity_mask, tests/golden/data_img5.npz), the only real-data size it runs")
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--ista-slices", type=int, default=None,
                    help="DIP workloads: launches the sparse coding's Nit is split over (LrsPnPConfig.ista_slices_dip)")
    ap.add_argument("--ista-max-wg", type=int, default=None,
                    help="workgroups of the sparse-coding kernel beside the DIP (default LrsPnPConfig's; 0 = unbounded)")
    ap.add_argument("--lowrank-priority", type=int, default=None,
                    help="priority of the low-rank (DIP) stream (LrsPnPConfig.lowrank_priority; negative = higher)")
    ap.add_argument("--ista-dip-order", default=None, choices=["beside", "before"],
                    help="DIP workloads: sparse coding beside the DIP training or before it (LrsPnPConfig.ista_dip_order)")
    ap.add_argument("--ista-patterns", default=None, choices=["auto", "on", "off"],
                    help="sparse coding on per-pattern masked Grams (LrsPnPConfig.ista_patterns)")
    ap.add_argument("--mask", default="tiled", choices=["tiled", "random"],
                    help="tiled: the 36x36 low_rank_sparsity_mask tiled over the cube (SURVEY.md §8d; the blocks "
                         "share a few observation patterns); random: the same 5.1 %% of missing pixels drawn "
                         "independently (every block its own pattern: the row-split sparse-coding kernel)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process group: nccl (= RCCL, one GPU per rank) or gloo (rehearsal: rank r on GPU "
                         "r mod the visible count, so ranks share cuda:0 on a 1-GPU box)")
    ap.add_argument("--split-cube", action="store_true",
                    help="one cube over all ranks (strong scaling): pnp in pixel-row slabs; dip task-parallel "
                         "(DIP on rank 0, sparse coding over the others)")
    a = ap.parse_args()
    dip = a.workload != "pnp"
    if a.steps is None:
        a.steps = 3 if dip else 10
    if a.warmup is None:
        a.warmup = 1 if dip else 2
    return a


def ensure_ranks(args):
    """--gpus N: under torchrun the world size must equal N; without a torchrun environment,
    N > 1 re-launches this script under torch.distributed.run as a CHILD process (nothing has
    touched the GPU yet) and exits with its code."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if args.gpus <= 1:
            return
        port = os.environ.get("MASTER_PORT", str(29500 + (os.getpid() % 1000)))
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", "--master-port", port, os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    if int(world) != args.gpus:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}\n")
        sys.exit(2)


def make_problem(H, W, B, bb, K, seed, mask="tiled", data="synthetic"):
    from lrspnp.data import load_fixture, mask_matrix, synthetic_cube, synthetic_dictionary, unfold
    if data == "native":   # the reference mains' own image and mask (tests/test_gpu_e2e_dip.py)
        d = load_fixture("data_img5.npz")
        return (unfold(d["noisy"][0]), mask_matrix(d["lrs_mask"], d["noisy"].shape[1]),
                synthetic_dictionary(bb * bb, K, 0), d["clean"][0])
    base = load_fixture("data_img5.npz")["lrs_mask"] if mask == "tiled" else None
    obs, clean, mask = synthetic_cube(H, W, B, seed=seed, base_mask=base)
    return unfold(obs), mask_matrix(mask, B), synthetic_dictionary(bb * bb, K, 0), clean


def load_traffic(key, profiled=True):
    """HBM bytes of the committed PMC pass (profiles/r06/traffic.json); None for a configuration
    other than the profiled default one."""
    if not profiled:
        return None
    try:
        return json.load(open(TRAFFIC_FILE)).get(key)
    except Exception:
        return None


class StreamTimer:
    """HIP events around a call, on the stream the call's kernels are launched on."""

    def __init__(self):
        self.ev = []
        self.on = False

    def wrap(self, fn, stream_of):
        import torch

        def timed(*a, **k):
            st = stream_of(a, k)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            out = fn(*a, **k)
            e1.record(st)
            if self.on:
                self.ev.append((e0, e1))
            return out
        return timed

    def mean_ms(self):
        return float(np.mean([a.elapsed_time(b) for a, b in self.ev])) if self.ev else float("nan")


# ------------------------------------------------------------------------------------------------
# CPU baseline (oracle), rank 0 at N = 1 only
# ------------------------------------------------------------------------------------------------
def host_cpus():
    """The host's CPUs: the machine's count, the CPUs this process may run on (affinity), the cgroup's
    CPU quota (cpu.max, None when unlimited) and the model name (/proc/cpuinfo)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return nproc, aff, quota, model


def _threads():
    """Threads of the CPU baseline: every CPU this process may use -- the affinity set, bounded by the
    cgroup quota -- unless OMP_NUM_THREADS fixes the share (the GPU pool sets it to the box's per-GPU
    CPU share and asks that it be left as it is)."""
    nproc, aff, quota, _ = host_cpus()
    avail = min(aff, int(quota)) if quota else aff
    t = int(os.environ.get("OMP_NUM_THREADS", "0")) or max(1, avail)
    os.environ["OMP_NUM_THREADS"] = str(t)
    return t


def nproc_cmd():
    """What `nproc` prints here (GNU: the usable CPUs, OMP_NUM_THREADS honoured), None without it."""
    import shutil
    exe = shutil.which("nproc")
    if not exe:
        return None
    try:
        return int(subprocess.run([exe], capture_output=True, text=True, timeout=10).stdout.strip())
    except (OSError, ValueError, subprocess.SubprocessError):
        return None


def host_fields(threads):
    machine, aff, quota, model = host_cpus()
    return {"cores": threads, "nproc": nproc_cmd(), "machine_cpus": machine, "affinity_cpus": aff,
            "cgroup_cpu_quota": quota, "cpu_model": model, "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_sparse_coding(Y, D, bb, nit, variant, budget_s):
    """Seconds per outer iteration of the oracle's sparse coding (alpha per block as the reference
    computes it inside ista(), + the C ISTA), from a growing random block sample."""
    from oracle import oracle as O
    P, B = Y.shape
    rows, cols = O.block_grid(P, B, bb, bb)
    nb = rows.size
    rng = np.random.default_rng(0)
    blocks = O.im2col(Y, bb, rows, cols)
    obs = (blocks != 0).astype(np.uint8)
    done, t_alpha, t_ista, batch = 0, 0.0, 0.0, 64 if bb > 8 else 256
    per_block = []   # seconds per block of each sampled batch (the extrapolation's spread)
    t_start = time.perf_counter()
    while (time.perf_counter() - t_start < budget_s or done < 2 * batch) and done < nb:
        idx = rng.choice(nb, batch, replace=False)
        t0 = time.perf_counter()
        al = np.empty(batch, np.float32)
        th = np.empty(batch, np.float64)
        for k, j in enumerate(idx):
            al[k], th[k] = O.ista_alpha_h(D[obs[j].astype(bool)], 0.1, variant)
        t1 = time.perf_counter()
        O.ista_batch(blocks[idx], obs[idx], D, al, th, nit)
        t_ista += time.perf_counter() - t1
        t_alpha += t1 - t0
        per_block.append((time.perf_counter() - t0) / batch)
        done += batch
    pb = np.asarray(per_block)
    se = float(pb.std(ddof=1) / np.sqrt(pb.size) * nb) if pb.size > 1 else float("nan")
    return (t_alpha + t_ista) / done * nb, done, nb, t_alpha / done * nb, se


def cpu_admm(Y, M, bb):
    from oracle import oracle as O
    P, B = Y.shape
    rows, cols = O.block_grid(P, B, bb, bb)
    nb = rows.size
    X = Y.copy()
    PHI = np.zeros((nb, bb * bb), np.float32)
    t0 = time.perf_counter()
    O.lib().oracle_admm_update(P, B, bb, nb, rows, cols, PHI, Y, M, Y, X, X, 0.5, np.float32(0.15),
                               np.float32(0.9), X.copy(), X.copy(), X.copy(), None, None)
    return time.perf_counter() - t0


def cpu_baseline_pnp(Y, M, D, bb, nit, budget_s):
    from oracle import oracle as O
    threads = _threads()
    t_sc, done, nb, t_alpha, se_sc = cpu_sparse_coding(Y, D, bb, nit, "spec2", budget_s * 0.7)
    t0 = time.perf_counter()
    O.svt(Y, 1 / 0.9)                                       # the reference's float32 LAPACK SVT
    t_svt = time.perf_counter() - t0
    t_admm = cpu_admm(Y, M, bb)
    t_iter = t_sc + t_svt + t_admm
    return {"value": 1.0 / t_iter, "unit": "outer_iters/s", **host_fields(threads), "kind": "port",
            # the GPU path computes alpha once per observation pattern, outside the timed steps
            "value_alpha_hoisted": 1.0 / (t_iter - t_alpha),
            # 95 % interval of the extrapolated time from the spread of the sampled batches
            "ci95_rel": 1.96 * se_sc / t_iter,
            "sample": f"{done} of {nb} blocks (alpha+ISTA, Nit={nit}) extrapolated x{nb / done:.1f} "
                      f"({t_sc:.1f}s, of which per-block alpha {t_alpha:.1f}s), + full SVT ({t_svt:.2f}s) + "
                      f"full ADMM update ({t_admm:.3f}s); est. {t_iter:.1f}s per outer iteration"}


def cpu_baseline_dip(solver, Y, M, D, bb, nit, dip_steps, budget_s):
    import torch

    from oracle import dip_ref
    threads = _threads()
    torch.set_num_threads(threads)
    t_sc, done, nb, t_alpha, se_sc = cpu_sparse_coding(Y, D, bb, nit, "fro4", budget_s * 0.4)
    net = solver.dip.net
    x = solver.dip_in.detach().cpu()
    target = solver.dip_target.detach().cpu()
    mask = solver.dip_mask.detach().cpu()
    tr = dip_ref.RefTrainer(net.nodes, net.params.detach().cpu())
    tr.step(x, target, mask)                                # warm (allocator, thread pool)
    steps, t_dip, st = 0, 0.0, []
    t_start = time.perf_counter()
    while time.perf_counter() - t_start < budget_s * 0.5 or steps < 2:
        t0 = time.perf_counter()
        tr.step(x, target, mask)
        st.append(time.perf_counter() - t0)
        t_dip += st[-1]
        steps += 1
    per_step = t_dip / steps
    se_dip = float(np.std(st, ddof=1) / np.sqrt(len(st))) * dip_steps
    t_admm = cpu_admm(Y, M, bb)
    t_iter = t_sc + per_step * dip_steps + t_admm
    return {"value": 1.0 / t_iter, "unit": "outer_iters/s", **host_fields(threads), "kind": "port",
            # the GPU path computes alpha once per observation pattern, outside the timed steps
            "value_alpha_hoisted": 1.0 / (t_iter - t_alpha),
            # 95 % interval of the extrapolated time: the sampled batches' and DIP steps' spreads
            "ci95_rel": 1.96 * float(np.sqrt(se_sc ** 2 + se_dip ** 2)) / t_iter,
            "sample": f"sparse coding: {done} of {nb} blocks (alpha+ISTA, Nit={nit}, oracle C) extrapolated "
                      f"x{nb / done:.1f} = {t_sc:.1f}s (of which per-block alpha {t_alpha:.1f}s, as the reference "
                      f"computes it inside ista; value_alpha_hoisted leaves it out); DIP: {steps} training steps of the torch-CPU restatement "
                      f"(oracle/dip_ref.py: conv/BN/LeakyReLU, full-SVD sigma_max per conv, Adam) at "
                      f"{per_step:.2f}s/step x {dip_steps:g} = {per_step * dip_steps:.1f}s; full ADMM update "
                      f"{t_admm:.3f}s; est. {t_iter:.1f}s per outer iteration"}


# ------------------------------------------------------------------------------------------------
def dip_flops_per_step(net):
    """Algorithmic MFMA FLOPs of one DIP training step: conv forward + dW + dX (no dX for a conv
    that reads the network input)."""
    sh = [net.in_shape] + list(net.shapes)
    tot = 0
    for i, nd in enumerate(net.nodes):
        if nd.kind != 0:
            continue
        co, ho, wo = sh[i + 1]
        f = 2 * co * sh[nd.in0][0] * nd.k * nd.k * ho * wo
        tot += f * (2 if nd.in0 == 0 else 3)
    return tot


def dip_alg_bytes_per_step(net):
    """Algorithmic HBM bytes of one DIP training step: every tensor a layer must read
    or write once, fp32.  Per conv node with input x (Cin x Pin) and output z (Cout x P): forward x
    in, z out, BN(+act) z in, y out; backward BN gy and z in, dL/dz out, data gradient dL/dz in and
    dL/dx out (none for a conv on the network input), weight gradient dL/dz and x in: 3 Cin Pin +
    8 Cout P (2 Cin Pin fewer on the input, 2 Cout P fewer without BN); the loss head reads the
    output and target and writes dL/dz (3 C P), Adam reads p, g, m, v and writes p, m, v."""
    sh = [net.in_shape] + list(net.shapes)
    tot = 0
    for i, nd in enumerate(net.nodes):
        if nd.kind != 0:
            continue
        ci, hi, wi = sh[nd.in0]
        co, ho, wo = sh[i + 1]
        xin, out = ci * hi * wi, co * ho * wo
        tot += (xin if nd.in0 == 0 else 3 * xin) + (8 if nd.bn else 6) * out
    co, ho, wo = sh[-1]
    tot += 3 * co * ho * wo + 7 * net.n_params
    return 4 * tot


def ista_entry(name, ista_ms, flops, traffic_key, profiled=True):
    achieved = flops / (ista_ms * 1e-3) / 1e12
    return {"kernel": name, "bound": "mfma", "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / FP32_MFMA_PEAK_TFLOPS, "traffic": load_traffic(traffic_key, profiled),
            "flops_per_launch": flops, "ms_per_launch": ista_ms}


def main_dip(args, ctx):
    import torch

    from lrspnp import LrsPnP, LrsPnPConfig, ops
    from lrspnp import dist as D
    from lrspnp.dip import DipConfig
    from lrspnp.metrics import mpsnr
    pro = args.workload == "dip-pro"
    native = args.data == "native"
    if native and args.cube not in (None, "36x36x128"):
        raise SystemExit("bench.py: --data native is the reference's 36x36x128 image")
    H, W, B = ((36, 36, 128) if native else (int(v) for v in args.cube.split("x")) if args.cube else
               ((512, 512, 224) if pro else (196, 196, 198)))
    bb = args.bb or 36
    nit = args.nit or 100
    split = args.split_cube
    es = args.early_stop
    Y, M, Dct, clean = make_problem(H, W, B, bb, args.K, seed=0 if split else ctx.rank, mask=args.mask, data=args.data)
    # ES off: exactly --dip-steps per outer iteration; ES on: the reference's rule, at most
    # --dip-cap steps (get_DIP_out, main_LRS_PnP_DIP_1-LiP.py:221-264)
    dcfg = DipConfig(num_iter=args.dip_cap if es else args.dip_steps, early_stop=es, net="skip" if pro else "unet1lip")
    extra = {} if args.ista_max_wg is None else {"ista_max_wg_dip": args.ista_max_wg}
    if args.ista_slices is not None:
        extra["ista_slices_dip"] = args.ista_slices
    if args.lowrank_priority is not None:
        extra["lowrank_priority"] = args.lowrank_priority
    if args.ista_dip_order is not None:
        extra["ista_dip_order"] = args.ista_dip_order
    if args.ista_patterns is not None:
        extra["ista_patterns"] = args.ista_patterns
    cfg = (LrsPnPConfig.dip_pro if pro else LrsPnPConfig.dip_1lip)(bb=bb, sliding=bb, Nit=nit, dip=dcfg, **extra)
    # the per-solve setup of the sparse coding (alpha / h per observation pattern, and on the pattern
    # path every pattern's masked Gram): D and the masks are fixed for the whole solve, so it runs once
    # in the constructor, outside the timed steps; its device time is reported in the line's config
    setup_t = StreamTimer()
    setup_t.on = True
    orig_alpha, orig_prep = ops.ista_alpha, ops.ista_pat_prepare
    ops.ista_alpha = setup_t.wrap(orig_alpha, lambda a, k: k.get("stream") or torch.cuda.current_stream())
    ops.ista_pat_prepare = setup_t.wrap(orig_prep, lambda a, k: k.get("stream") or torch.cuda.current_stream())
    try:
        task = D.DipTaskSplit(Y, M, Dct, cfg, ctx, image_shape=(H, W)) if split else None
        s = task.s if split else LrsPnP(Y, M, Dct, cfg, image_shape=(H, W))
    finally:
        ops.ista_alpha, ops.ista_pat_prepare = orig_alpha, orig_prep
    clean_d = torch.from_numpy(clean).cuda()
    mp0 = mpsnr(s.X, clean_d)

    dip_t, ista_t = StreamTimer(), StreamTimer()
    s.low_rank_dip = dip_t.wrap(s.low_rank_dip, lambda a, k: a[0])
    orig_ista, orig_ista_pat = ops.ista, ops.ista_pat
    ops.ista = ista_t.wrap(orig_ista, lambda a, k: k.get("stream") or torch.cuda.current_stream())
    ops.ista_pat = ista_t.wrap(orig_ista_pat, lambda a, k: k.get("stream") or torch.cuda.current_stream())
    count = [0]

    def step():
        dip_t.on = ista_t.on = count[0] >= args.warmup
        count[0] += 1
        (task.step if split else s.step)()

    try:
        elapsed = D.timed_steps(step, args.steps, args.warmup, ctx)
    finally:
        ops.ista, ops.ista_pat = orig_ista, orig_ista_pat
    setup_ms = setup_t.mean_ms() * len(setup_t.ev)   # (events complete: timed_steps synchronised)
    mp1 = mpsnr(s.X, clean_d)
    # a time-sliced sparse coding (LrsPnPConfig.ista_slices_dip) is several back-to-back launches:
    # its time per outer iteration is their sum
    n_sl = len(ista_t.ev) / max(1, args.steps)
    dip_ms, ista_ms = dip_t.mean_ms(), ista_t.mean_ms() * n_sl
    if split and ctx.world > 1:   # rank 0 trained the DIP, ranks 1.. coded: take each stage from those ranks
        per = D.gather_scalars([dip_ms, ista_ms], ctx)
        if per is not None:
            dip_ms = per[0][0]
            ista_ms = float(np.nanmean([v[1] for v in per[1:]]))
    # DIP steps of the timed outer iterations (ES on: to the stop, each different)
    timed_runs = list(getattr(s, "dip_steps", []))[-args.steps:] if s.dip is not None else []
    n_dip = float(np.mean([n for n, _ in timed_runs])) if es and timed_runs else float(args.dip_steps)
    # (task-parallel workers build no DIP engine; rank 0, which prints the line, always has one)
    flops = dip_flops_per_step(s.dip.net) * n_dip if s.dip is not None else float("nan")
    profiled = not (args.cube or args.bb or args.nit or args.K != 256 or args.dip_steps != 100 or args.mask != "tiled"
                    or es or native)
    achieved = flops / (dip_ms * 1e-3) / 1e12
    n = bb * bb
    pat = getattr(s, "pat_plan", None) is not None
    # matrix-core work per launch: the row-split kernel's two products per iteration (+ Phi), or the
    # per-pattern path's b and Phi once and one K x K product per iteration (its Grams are formed
    # once per solve, lrs_ista_pat_prepare, outside the timed steps)
    ista_flops = (s.nb * (4 * n * args.K + nit * 2 * args.K ** 2) if pat else
                  nit * s.nb * 4 * n * args.K + s.nb * 2 * n * args.K)
    ista_name = (f"k_ista_pat (lrs_ista_pat_f32: {s.nb} blocks of {n} rows in {s.pat_ntiles} tiles of "
                 f"{s.npat} observation patterns, Nit {nit}" if pat else
                 f"k_ista_rs (lrs_ista_f32: {s.nb} blocks of {n} rows, Nit {nit}")
    net_desc = ("skip net (5 x 128 ch, 128-ch skips)" if pro else f"my_Lipschitz_Unet ({B}->128->{B} ch)")
    tag = "dip_pro" if pro else "dip"
    traffic = load_traffic(f"{tag}_hbm_bytes_per_outer_iter", profiled)
    alg_bytes = dip_alg_bytes_per_step(s.dip.net) * n_dip if s.dip is not None else None
    es_desc = (f"ES on (buffer 30, patience 60, cap {args.dip_cap}: {n_dip:.1f} DIP steps per timed outer iteration "
               f"on average)" if es else "ES off")
    data_desc = ("the reference's own 36x36x128 image (data_img5 noisy/clean, low_rank_sparsity_mask)" if native else
                 f"synthetic (seeded low-rank {H}x{W}x{B} cube per rank, "
                 + ("tiled low_rank_sparsity_mask" if args.mask == "tiled" else
                    "random mask with 5.1 % missing pixels (no repeated block patterns)") + ")")
    out = {
        "metric": METRIC, "value": (1 if split else ctx.world) * args.steps / elapsed, "unit": "outer_iters/s",
        "n_gpus": ctx.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong" if split else "weak",
        "vs_baseline": None, "dtype": "f32 (MFMA products fp32-accurate) + f64 (NLM prox, BN/sigma statistics)",
        "data": f"{data_desc}, seeded K={args.K} dictionary, random-init DIP net per outer iteration",
        "config": {"workload": (f"LRS-PnP-DIP(pro) skip net on the literal {H}x{W}x{B} cube (BASELINE configs[2] "
                                f"as written; the skip net maps any H x W)" if pro and (H, W, B) == (200, 200, 198) else
                                f"LRS-PnP-DIP(pro) {H}x{W}x{B} (BASELINE configs[3]; configs[4] = one such cube per "
                                f"GPU)" if pro else
                                f"LRS-PnP-DIP(1-Lip) on the reference's 36x36x128 image" if native else
                                f"LRS-PnP-DIP(1-Lip) on a {H}x{W}x{B} cube" if args.cube else
                                f"LRS-PnP-DIP(1-Lip) on the 200x200x198 cube cropped to {H}x{W}x{B} "
                                f"(BASELINE configs[2]; 196 = largest 16a-12 size <= 200 that the U-Net maps onto "
                                f"itself)") + f": {bb}x{bb} blocks ({s.nb}), K={args.K}, Nit={nit} fro4 ISTA + NLM "
                               f"prox; DIP {net_desc} "
                               + (f"{args.dip_steps} Adam steps per outer iteration, ES off" if not es else
                                  f"Adam to the early stop: {es_desc}"),
                   "blocks": s.nb,
                   "mask": args.mask, "observation_patterns": int(s.npat),
                   "sparse_coding_path": "k_ista_pat" if pat else "k_ista_rs",
                   "setup_ms_per_solve": setup_ms,
                   "setup": "per-pattern alpha/h (k_alpha) and, on the k_ista_pat path, the masked Grams "
                            "(k_pat_gram + dictionary images): once per solve, outside the timed steps",
                   "parallelism": (f"1 cube, task-parallel: DIP on rank 0, sparse coding over {ctx.world - 1} rank(s)"
                                   if split and ctx.world > 1 else f"{ctx.world} independent cube(s), one per GPU")},
        "roofline": {"bound": "mfma", "kernel": f"DIP training of one outer iteration ({n_dip:g} steps: conv "
                                                f"GEMMs, sigma_max, BN, loss, Adam kernels)",
                     "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP32_MFMA_PEAK_TFLOPS,
                     # the convs run on the bf16 matrix cores, 6 MFMAs per fp32-accurate product
                     "peak_split_bf16": SPLIT_BF16_PEAK_TFLOPS,
                     "frac_split_bf16": achieved / SPLIT_BF16_PEAK_TFLOPS,
                     "traffic": traffic,
                     "alg_bytes": alg_bytes,
                     "traffic_over_alg": (traffic / alg_bytes) if traffic and alg_bytes else None,
                     "flops_per_outer_iter": flops, "ms_per_outer_iter": dip_ms,
                     "kernels": [ista_entry(ista_name
                                            + (f" over {n_sl:.0f} warm-started launches" if n_sl > 1 else "") + ")",
                                            ista_ms, ista_flops, f"{tag}_ista_hbm_bytes_per_launch", profiled)]},
        "mpsnr": {"input": mp0, "after_steps": mp1, "outer_iterations_run": args.warmup + args.steps},
    }
    if es:
        out["early_stopping"] = {
            "dip_steps_per_outer_iter": [int(n) for n, _ in timed_runs],
            "stop_epochs": [None if e is None else int(e) for _, e in timed_runs],
            "mean_dip_steps": n_dip, "s_per_outer_iter": elapsed / args.steps,
            "dip_ms_per_step": dip_ms / n_dip,
            "reference": "main_LRS_PnP_DIP_1-LiP.py on its 36x36x128 data, 1st outer iteration: 28.4 s "
                         "(~165 DIP steps to the stop, 0.127 s per step; BASELINE.md:46)"}
    if ctx.rank == 0 and ctx.world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_dip(s, Y, M, Dct, bb, nit, n_dip, args.cpu_seconds)
    return out


def main_pnp(args, ctx):
    import torch

    from lrspnp import LrsPnP, LrsPnPConfig, ops
    from lrspnp import dist as D
    from lrspnp.metrics import mpsnr
    H, W, B = (int(v) for v in (args.cube or "200x200x198").split("x"))
    bb = args.bb or 8
    nit = args.nit or 80
    split = args.split_cube
    Y, M, Dct, clean = make_problem(H, W, B, bb, args.K, seed=0 if split else ctx.rank, mask=args.mask)
    cfg = LrsPnPConfig(bb=bb, sliding=bb, Nit=nit, variant="spec2")
    t0 = time.perf_counter()
    s = D.slab_solver(Y, M, Dct, cfg, ctx)[0] if split else LrsPnP(Y, M, Dct, cfg)
    torch.cuda.synchronize()
    setup_s = time.perf_counter() - t0
    clean_d = torch.from_numpy(clean).cuda()

    def cube_mpsnr():
        if not split:
            return mpsnr(s.X, clean_d)
        X = D.gather_rows(s.X, ctx)
        return mpsnr(torch.from_numpy(X).cuda(), clean_d) if X is not None else float("nan")

    mp0 = cube_mpsnr()
    ista_t = StreamTimer()
    orig_ista = ops.ista
    ops.ista = ista_t.wrap(orig_ista, lambda a, k: k.get("stream") or torch.cuda.current_stream())
    count = [0]
    track = []

    def step():
        ista_t.on = count[0] >= args.warmup
        count[0] += 1
        s.step()
        if count[0] <= min(2, args.warmup) and not split:
            track.append(mpsnr(s.X, clean_d))      # the first two iterates, for the oracle fixture below

    elapsed = D.timed_steps(step, args.steps, args.warmup, ctx)
    ops.ista = orig_ista
    mp1 = cube_mpsnr()
    world, rank = ctx.world, ctx.rank
    mps = [[mp0, mp1]] if split else D.gather_scalars([mp0, mp1], ctx)
    n, K = bb * bb, args.K
    flops = nit * s.nb * 4 * n * K + s.nb * 2 * n * K
    profiled = (H, W, B, bb, nit, K) == (200, 200, 198, 8, 80, 256) and args.mask == "tiled"
    entry = ista_entry("k_ista_ln2 (lrs_ista_f32)", ista_t.mean_ms(), flops, "pnp_ista_hbm_bytes_per_launch", profiled)
    roof = {k: entry[k] for k in ("bound", "kernel", "achieved", "peak", "unit", "frac", "traffic",
                                  "flops_per_launch", "ms_per_launch")}
    # k_ista_ln2's products are split-bf16 (6 bf16 MFMAs each); its NLM prox is fp64 VALU
    roof["peak_split_bf16"] = SPLIT_BF16_PEAK_TFLOPS
    roof["frac_split_bf16"] = entry["achieved"] / SPLIT_BF16_PEAK_TFLOPS
    out = {
        "metric": METRIC, "value": (1 if split else world) * args.steps / elapsed, "unit": "outer_iters/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong" if split else "weak", "vs_baseline": None,
        "dtype": "f32 (MFMA products fp32-accurate) + f64 (NLM prox, Gram/eig)",
        "data": "synthetic (seeded low-rank cube per rank, "
                + ("tiled low_rank_sparsity_mask" if args.mask == "tiled" else "random mask, 5.1 % missing pixels")
                + ", seeded K=256 dictionary)",
        "config": {"workload": f"LRS-PnP (no DIP) {H}x{W}x{B} cube, {bb}x{bb} blocks, K={K}, Nit={nit} inner ISTA, "
                               f"SVT low-rank prox ("
                               + ("BASELINE configs[1]" if (H, W, B) == (200, 200, 198) else
                                  "configs[1]'s workload on a cube of another size; 512x512x224 = the configs[3]/[4] "
                                  "cube" if (H, W, B) == (512, 512, 224) else "configs[1]'s workload, other cube")
                               + ")",
                   "blocks": s.nb,
                   "parallelism": (f"1 cube in {world} pixel-row slab(s), fp64 Gram all-reduce per iteration"
                                   if split else f"{world} independent cube(s), one per GPU")},
        "roofline": roof, "setup_s": setup_s,
        "mpsnr": {"input": mp0, "after_steps": mp1, "outer_iterations_run": args.warmup + args.steps,
                  "per_rank": mps},
    }
    fx = os.path.join(REPO, "tests", "golden", "cube200_oracle_2iter.npz")
    if track and (H, W, B, bb, nit, K) == (200, 200, 198, 8, 80, 256) and os.path.exists(fx):
        with np.load(fx, allow_pickle=False) as z:
            out["mpsnr"]["first_two_iterates"] = {"gpu": track[:2], "oracle": [float(v) for v in z["mpsnr"]],
                                                  "oracle_input": float(z["mpsnr_input"])}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_pnp(Y, M, Dct, bb, nit, args.cpu_seconds)
    return out


def main():
    args = parse()
    ensure_ranks(args)
    from lrspnp import dist as D
    ctx = D.init_from_env(args.backend)
    out = main_pnp(args, ctx) if args.workload == "pnp" else main_dip(args, ctx)
    if out["n_gpus"] != args.gpus:
        raise SystemExit(f"bench.py: ran on {out['n_gpus']} rank(s), --gpus {args.gpus}")
    if ctx.rank == 0:
        print(json.dumps(out), flush=True)
    if ctx.world > 1:
        import torch.distributed as tdist
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
