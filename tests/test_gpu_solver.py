"""End-to-end parity of the batched GPU solver.

* native 36x36x128 data (img5 + fourth_mask, K=256 seed-0 dictionary): two outer iterations of the
  unmodified main_LRS_PnP.py captured in tests/golden/lrs_pnp_2iter.npz.  Tolerance: 1e-5 relative
  L2 on X / lambda_1 / lambda_2, MPSNR identical to 2 dp (BASELINE.json north_star).
* BASELINE configs[1] shape (200x200x198, bb=8, nb=125000): size-independent properties — a sample
  of blocks re-solved by the oracle, determinism, finiteness, convergence norms.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return np.linalg.norm(a - b) / np.linalg.norm(b)


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True


def test_two_outer_iterations_vs_reference(gpu, golden):
    from lrspnp import LrsPnP, LrsPnPConfig
    from lrspnp.data import synthetic_dictionary, unfold, mask_matrix
    from lrspnp.metrics import mpsnr
    d = golden("data_img5.npz")
    g = golden("lrs_pnp_2iter.npz")
    Y = unfold(d["noisy_img5"][0])
    M = mask_matrix(d["fourth_mask"], 128)
    D = synthetic_dictionary(1296, 256, 0)
    s = LrsPnP(Y, M, D, LrsPnPConfig(bb=36, sliding=36, Nit=80, variant="spec2"))
    clean = torch.from_numpy(d["clean_img5"][0]).cuda()
    s.step()
    torch.cuda.synchronize()
    assert rel(s.X.cpu().numpy(), g["it1_X"]) < 1e-5
    assert rel(s.L1.cpu().numpy(), g["it1_L1"]) < 1e-5
    assert rel(s.L2.cpu().numpy(), g["it1_L2"]) < 1e-5
    assert rel(s.U.cpu().numpy(), g["it1_U"]) < 1e-5
    assert rel(s.phi.cpu().numpy()[:, :1296], g["it1_PHI"]) < 1e-5
    p1 = mpsnr(s.X, clean)
    s.step()
    torch.cuda.synchronize()
    assert rel(s.X.cpu().numpy(), g["it2_X"]) < 1e-5
    assert rel(s.L1.cpu().numpy(), g["it2_L1"]) < 1e-5
    assert rel(s.L2.cpu().numpy(), g["it2_L2"]) < 1e-5
    p2 = mpsnr(s.X, clean)
    assert round(p1, 2) == round(float(g["mpsnr"][0]), 2)
    assert round(p2, 2) == round(float(g["mpsnr"][1]), 2)


def test_config0_fifty_outer_iterations_vs_reference(gpu, golden):
    """BASELINE configs[0] as written: main_LRS_PnP.py's 50 outer iterations on
    low_rank_sparsity_noisy.mat + fourth_mask.mat (the reference itself, run by
    tests/golden/gen_golden.py cfg0).  X after iterations 1, 2 and 50 and lambda_1 / lambda_2 after
    50 to 1e-5 relative L2, the MPSNR of every one of the 50 iterations identical to 2 dp."""
    from lrspnp import LrsPnP, LrsPnPConfig
    from lrspnp.data import synthetic_dictionary, unfold, mask_matrix
    from lrspnp.metrics import mpsnr
    d = golden("data_img5.npz")
    g = golden("lrs_pnp_cfg0_50iter.npz")
    s = LrsPnP(unfold(d["noisy"][0]), mask_matrix(d["fourth_mask"], 128), synthetic_dictionary(1296, 256, 0),
               LrsPnPConfig(bb=36, sliding=36, Nit=80, variant="spec2"))
    clean = torch.from_numpy(d["clean"][0]).cuda()
    mps = []
    for it in range(50):
        s.step()
        mps.append(mpsnr(s.X, clean))
        if it in (0, 1):
            torch.cuda.synchronize()
            ref = g["X1"] if it == 0 else g["X2"]
            assert rel(s.X.cpu().numpy(), ref) < 1e-5, it
    torch.cuda.synchronize()
    assert rel(s.X.cpu().numpy(), g["X"]) < 1e-5
    assert rel(s.L1.cpu().numpy(), g["L1"]) < 1e-5
    assert rel(s.L2.cpu().numpy(), g["L2"]) < 1e-5
    assert np.array_equal(np.round(mps, 2), np.round(g["mpsnr"], 2)), (mps, g["mpsnr"])


def test_dip_variant_sparse_coding_matches_oracle(gpu, golden):
    """ISTA rule of the DIP mains (alpha = 4||H||_F^2, h = T, Nit = 100) on the native data."""
    from lrspnp import LrsPnP, LrsPnPConfig
    from lrspnp.data import synthetic_dictionary, unfold, mask_matrix
    d = golden("data_img5.npz")
    Y = unfold(d["noisy"][0])
    M = mask_matrix(d["lrs_mask"], 128)
    D = synthetic_dictionary(1296, 256, 0)
    s = LrsPnP(Y, M, D, LrsPnPConfig.dip_1lip(lowrank="svt"))   # the sparse-coding half only
    phi = s.sparse_coding().cpu().numpy()[:, :1296]
    o = O.LrsPnpOracle(Y, M, D, bb=36, sliding=36, gamma=0.5, mu1=0.1, mu2=0.1, Nit=100, variant="fro4")
    blocks = O.im2col(o.X + o.L1 / np.float32(0.1), 36, o.rows, o.cols)
    _, PHI = O.ista_batch(blocks, o.obs, D, o.alpha, o.thr, 100)
    assert rel(phi, PHI) < 1e-5
    assert np.allclose(s.alpha.cpu().numpy(), o.alpha, rtol=1e-6)


def test_config2_shape_properties(gpu):
    """200x200x198 cube, bb = 8 (125,000 blocks), Nit = 80: the bench workload."""
    from lrspnp import LrsPnP, LrsPnPConfig
    from lrspnp.data import synthetic_cube, synthetic_dictionary, unfold, mask_matrix, load_fixture
    base = load_fixture("data_img5.npz")["lrs_mask"]
    obs, clean, mask = synthetic_cube(200, 200, 198, seed=0, base_mask=base)
    Y, M = unfold(obs), mask_matrix(mask, 198)
    D = synthetic_dictionary(64, 256, 0)
    cfg = LrsPnPConfig(bb=8, sliding=8, Nit=80, variant="spec2")
    s = LrsPnP(Y, M, D, cfg)
    assert s.nb == 125000
    s.step()
    torch.cuda.synchronize()
    X1 = s.X.clone()
    assert torch.isfinite(X1).all()
    # oracle re-solve of a sample of blocks (same inputs: first iteration, L1 = 0)
    rng = np.random.default_rng(0)
    sample = rng.choice(s.nb, 48, replace=False)
    Yb = s.Yb.cpu().numpy()[sample]
    ob = s.obs.cpu().numpy()[sample]
    Xo, PHIo = O.ista_batch(Yb, ob, D, s.alpha.cpu().numpy()[sample], s.thr.cpu().numpy()[sample], 80)
    phi = s.phi.cpu().numpy()[sample, :64]
    for k in range(sample.size):
        assert rel(phi[k], PHIo[k]) < 1e-5
    # the alpha of every distinct observation pattern vs numpy's float32 SVD
    pats = s.obs_pat.cpu().numpy()
    ap = s.alpha_pat.cpu().numpy()
    for k in range(min(pats.shape[0], 40)):
        ra, _ = O.ista_alpha_h(D[pats[k, :64].astype(bool)], 0.1, "spec2")
        assert abs(int(ap[k].view(np.int32)) - int(np.float32(ra).view(np.int32))) <= 2
    # determinism: a fresh solver reproduces the iterate bit for bit
    s2 = LrsPnP(Y, M, D, cfg)
    s2.step()
    torch.cuda.synchronize()
    assert torch.equal(s2.X, X1)
    nx, n1, n2 = s.norms.cpu().numpy()
    assert np.isfinite([nx, n1, n2]).all() and nx > 0


def _bench_problem(H, W, B, bb):
    from lrspnp.data import load_fixture, mask_matrix, synthetic_cube, synthetic_dictionary, unfold
    base = load_fixture("data_img5.npz")["lrs_mask"]
    obs, clean, mask = synthetic_cube(H, W, B, seed=0, base_mask=base)
    return unfold(obs), mask_matrix(mask, B), synthetic_dictionary(bb * bb, 256, 0), clean


def test_config1_two_outer_iterations_vs_oracle_fixture(gpu, golden):
    """BASELINE configs[1] end to end at full size (200x200x198, bb 8, 125,000 blocks, Nit 80):
    two whole-cube outer iterations against the oracle's (tests/golden/gen_cube_oracle.py).
    Tolerances: 1e-5 relative L2 on the row-strided X subsample (lambda_1 / lambda_2: see below), MPSNR and
    every band's PSNR identical to 2 dp (north_star), the three state_convergence norms to 1e-4.
    The oracle's MPSNR also falls from iteration 1 to 2 (32.136 -> 32.108), as the bench's does."""
    from lrspnp import LrsPnP, LrsPnPConfig
    from lrspnp.metrics import psnr_bands
    g = golden("cube200_oracle_2iter.npz")
    Y, M, D, clean = _bench_problem(200, 200, 198, 8)
    s = LrsPnP(Y, M, D, LrsPnPConfig(bb=8, sliding=8, Nit=80, variant="spec2"))
    clean_d = torch.from_numpy(clean).cuda()
    rows = torch.from_numpy(g["rows"]).cuda()
    assert np.allclose(psnr_bands(s.X, clean_d).cpu().numpy(), g["psnr_input"], atol=5e-3)
    for it in range(2):
        s.step()
        torch.cuda.synchronize()
        Xr = g["X"][it]
        got = s.X.index_select(0, rows).cpu().numpy()
        assert rel(got, Xr) < 1e-5, (it, rel(got, Xr))
        # the duals are mu (X - Phi) and mu (X - U): differences ~100x smaller than X, so their
        # relative error is X's amplified by the cancellation (measured 1.2e-5 on lambda_2, the
        # float32-LAPACK vs fp64-Gram SVT rounding).  Bound them at X's scale: ||d lambda|| <= 1e-5 mu ||X||
        for name, mu, ref in (("L1", s.cfg.mu1, g["L1"][it]), ("L2", s.cfg.mu2, g["L2"][it])):
            got = getattr(s, name).index_select(0, rows).cpu().numpy()
            err = np.linalg.norm((got - ref).astype(np.float64))
            assert err < 1e-5 * mu * np.linalg.norm(Xr.astype(np.float64)) and rel(got, ref) < 5e-5, (it, name, rel(got, ref))
        p = psnr_bands(s.X, clean_d).cpu().numpy()
        assert np.array_equal(np.round(p, 2), np.round(g["psnr"][it], 2)) or np.abs(p - g["psnr"][it]).max() < 5e-4
        assert round(float(p.mean()), 2) == round(float(g["mpsnr"][it]), 2)
        assert np.allclose(s.convergence(), g["norms"][it], rtol=1e-4)


@pytest.mark.parametrize("patterns", ["auto", "off"])
def test_config2_sparse_coding_vs_oracle_fixture(gpu, golden, patterns):
    """BASELINE configs[2]'s sparse coding at full size (196x196x198, bb 36, 6,408 blocks, fro4,
    Nit 100): Phi and coefficients of every 53rd block of the first outer iteration against the
    oracle C ISTA at 1e-5 relative L2 (per block and overall), on the per-pattern Gram path the
    solver picks for this cube (27 observation patterns) and on the row-split kernel."""
    from lrspnp import LrsPnP, LrsPnPConfig
    g = golden("cube196_bb36_sc.npz")
    Y, M, D, _ = _bench_problem(196, 196, 198, 36)
    s = LrsPnP(Y, M, D, LrsPnPConfig.dip_1lip(lowrank="svt", ista_patterns=patterns))
    assert s.nb == 6408
    assert (s.pat_plan is not None) == (patterns == "auto") and s.npat < 64
    phi, coefs = s.sparse_coding(want_coefs=True)
    torch.cuda.synchronize()
    sel = torch.from_numpy(g["blocks"]).cuda()
    ph = phi.index_select(0, sel).cpu().numpy()[:, :1296]
    co = coefs.index_select(0, sel).cpu().numpy()
    assert rel(ph, g["phi"]) < 1e-5 and rel(co, g["coefs"]) < 1e-5
    for k in range(sel.numel()):
        assert rel(ph[k], g["phi"][k]) < 1e-5, k


@pytest.mark.parametrize("patterns", ["auto", "off"])
def test_config3_sparse_coding_vs_oracle_fixture(gpu, golden, patterns):
    """BASELINE configs[3]'s sparse coding at full size (512x512x224, bb 36, 50,974 blocks, fro4,
    Nit 100; main_LRS_PnP_DIP_pro.py:375-400): coefficients of every 53rd block and Phi of every
    212th against the oracle C ISTA at 1e-5 relative L2, per-pattern Gram path (24 patterns) and
    row-split kernel."""
    from lrspnp import LrsPnP, LrsPnPConfig
    g = golden("cube512_bb36_sc.npz")
    Y, M, D, _ = _bench_problem(512, 512, 224, 36)
    s = LrsPnP(Y, M, D, LrsPnPConfig.dip_pro(lowrank="svt", ista_patterns=patterns))
    assert (s.pat_plan is not None) == (patterns == "auto")
    assert s.nb == int(g["nb"]) == 50974
    phi, coefs = s.sparse_coding(want_coefs=True)
    torch.cuda.synchronize()
    co = coefs.index_select(0, torch.from_numpy(g["blocks"]).cuda()).cpu().numpy()
    ph = phi.index_select(0, torch.from_numpy(g["phi_blocks"]).cuda()).cpu().numpy()[:, :1296]
    assert rel(co, g["coefs"]) < 1e-5 and rel(ph, g["phi"]) < 1e-5
    for k in range(co.shape[0]):
        assert rel(co[k], g["coefs"][k]) < 1e-5, k


@pytest.mark.parametrize("world,cube,bb", [(2, "96x64x40", 8), (3, "100x60x37", 8), (3, "100x61x37", 8),
                                           (2, "38x38x40", 36)])
def test_row_slab_sharding_matches_whole_cube(gpu, world, cube, bb):
    """One cube in pixel-row slabs over `world` ranks (gloo, all on cuda:0): the
    sharded solver (slab-local sparse coding / col2im / updates, all-reduced fp64 SVT Gram)
    reproduces the whole-cube solver. Tolerance 1e-6 relative L2 after 3 outer iterations: the
    slabs sum the fp64 Gram in another order, everything else is the same per-block arithmetic.
    100x60 (P = 6000, a multiple of bb = 8) splits into ragged slabs of whole block rows and 37 bands
    give an odd Gram size; 100x61 (P = 6100, P % 8 = 4) and 38x38x40 with bb 36 (P = 1444, P % 36 = 4:
    the 200x200 / 196x196 configs' case) put the appended block row at P - bb, overlapping the
    previous block row, on the last rank."""
    import json
    import os
    import socket
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(repo, "tools", "shard_check.py"),
           "--backend", "gloo", "--cube", cube, "--steps", "3", "--bb", str(bb)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=100, cwd=repo)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    r = json.loads(line)
    assert r["world"] == world
    assert r["rel_X"] < 1e-6 and r["rel_L1"] < 1e-6 and r["rel_L2"] < 1e-6, r
    assert np.allclose(r["conv_sharded"], r["conv_whole"], rtol=1e-6, atol=1e-9), r


@pytest.mark.parametrize("world", [2, 3])
def test_task_parallel_dip_matches_one_rank(gpu, world):
    """One cube, task-parallel DIP (lrspnp.dist.DipTaskSplit): rank 0 trains the
    DIP, the other ranks code block ranges, U is broadcast and Phi all-gathered, every rank
    applies the same update.  Against the one-rank solver on rank 0 (gloo, all ranks on cuda:0):
    the kernels are deterministic, so the iterates agree to rounding (1e-6 relative L2) after 2
    outer iterations of 5 DIP steps each."""
    import json
    import os
    import socket
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(repo, "tools", "shard_check.py"),
           "--backend", "gloo", "--cube", "36x36x40", "--bb", "12", "--steps", "2", "--dip", "5", "--nit", "10"]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=150, cwd=repo)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert r["world"] == world
    assert r["rel_X"] < 1e-6 and r["rel_L1"] < 1e-6 and r["rel_L2"] < 1e-6 and r["rel_U"] < 1e-6, r


@pytest.mark.parametrize("H", [36, 132])
def test_lowrank_priority_same_iterates(gpu, H):
    """LrsPnPConfig.lowrank_priority only changes the queue priority of the DIP's streams (its
    training stream and the engine's weight-gradient side stream, which takes the same priority),
    not the arithmetic: two DIP solvers in one process, priority 0 and -1, same seeds, give the same
    iterates (1e-6 relative L2, the task-parallel test's bar) after 2 outer iterations.  The weight
    gradients run on the engine's side stream at both sizes; one net is then also trained on streams
    of the other priority (the side stream is re-created) with bit-identical results."""
    from lrspnp import LrsPnP, LrsPnPConfig
    from lrspnp.data import mask_matrix, synthetic_cube, synthetic_dictionary, unfold
    from lrspnp.dip import DipConfig
    W, B, bb = H, 40, 12
    obs, clean, mask = synthetic_cube(H, W, B, seed=5)
    Y, M = unfold(obs), mask_matrix(mask, B)
    Dct = synthetic_dictionary(bb * bb, 256, 0)
    out = []
    for prio in (0, -1):
        cfg = LrsPnPConfig.dip_1lip(bb=bb, sliding=bb, Nit=10, lowrank_priority=prio,
                                    dip=DipConfig(num_iter=5, early_stop=False))
        s = LrsPnP(Y, M, Dct, cfg, image_shape=(H, W))
        assert s.lowrank_stream.priority == prio and s.dip.net.stream.priority == prio
        for _ in range(2):
            s.step()
        torch.cuda.synchronize()
        out.append((s.X.clone(), s.U.clone()))
    (X0, U0), (X1, U1) = out
    assert float((X1 - X0).norm() / X0.norm()) < 1e-6
    assert float((U1 - U0).norm() / U0.norm()) < 1e-6
    if True:
        # the same engine (priority -1 so far) trained on priority-0 / -1 / 0 streams
        net = s.dip.net
        res = []
        for prio in (0, -1, 0):
            net.stream = torch.cuda.Stream(priority=prio)
            y = s.dip.run(s.dip_target, s.dip_in, s.dip_mask, seed=11, early_stop=False)
            torch.cuda.synchronize()
            res.append(y.clone())
        assert torch.equal(res[0], res[1]) and torch.equal(res[0], res[2])
