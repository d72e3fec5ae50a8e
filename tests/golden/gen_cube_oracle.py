"""Fixtures of the ORACLE at the benchmarked sizes (run in the build container, ~10 min on 8 cores).

    OMP_NUM_THREADS=8 python tests/golden/gen_cube_oracle.py

cube200_oracle_2iter.npz — BASELINE configs[1]: oracle.LrsPnpOracle (main_LRS_PnP.py:244-366
  restated: C ISTA + NLM over 125,000 8x8 blocks, Nit 80, numpy float32 SVT, C ADMM update) for two
  outer iterations on bench.py's seeded 200x200x198 cube: MPSNR and per-band PSNR of the input and
  of both iterates, the three state_convergence norms, and a row-strided subsample (every 97th
  pixel row, all bands) of X, lambda_1, lambda_2 after each iteration.
cube196_bb36_sc.npz — BASELINE configs[2]'s sparse coding: the oracle ISTA (fro4, Nit 100) of the
  first outer iteration over the 6,408 36x36 blocks of the 196x196x198 cube; Phi and coefficients
  of every 53rd block.
cube512_bb36_sc.npz — BASELINE configs[3]'s sparse coding (512x512x224, 50,974 blocks): the
  coefficients of every 53rd block and Phi of every 212th (python tests/golden/gen_cube_oracle.py
  cube512; the oracle runs only those blocks).

The oracle is itself pinned to the reference (tests/test_oracle.py, tests/golden/gen_golden.py);
nothing here imports /root/reference.
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]

import numpy as np  # noqa: E402

from lrspnp.data import load_fixture, mask_matrix, synthetic_cube, synthetic_dictionary, unfold  # noqa: E402
from oracle import oracle as O  # noqa: E402

ROW_STRIDE = 97
BLOCK_STRIDE = 53


def problem(H, W, B, bb, K=256, seed=0):
    base = load_fixture("data_img5.npz")["lrs_mask"]
    obs, clean, mask = synthetic_cube(H, W, B, seed=seed, base_mask=base)
    return unfold(obs), mask_matrix(mask, B), synthetic_dictionary(bb * bb, K, 0), clean


def norms(o, Xp, L1p, L2p):
    # state_convergence (main_LRS_PnP.py:23-25): ln ||new - old||_F of X, lambda_1, lambda_2
    f = lambda a, b: float(np.log(np.linalg.norm((a - b).astype(np.float64))))
    return [f(o.X, Xp), f(o.L1, L1p), f(o.L2, L2p)]


def cube200():
    Y, M, D, clean = problem(200, 200, 198, 8)
    o = O.LrsPnpOracle(Y, M, D, bb=8, sliding=8, Nit=80, variant="spec2")
    rows = np.arange(0, Y.shape[0], ROW_STRIDE)
    out = {"rows": rows, "psnr_input": O.psnr_bands(Y, clean)}
    out["mpsnr_input"] = np.float64(out["psnr_input"].mean())
    ps, mps, nr, Xs, L1s, L2s = [], [], [], [], [], []
    for it in range(2):
        t0 = time.time()
        Xp, L1p, L2p = o.X.copy(), o.L1.copy(), o.L2.copy()
        o.step()
        p = O.psnr_bands(o.X, clean)
        ps.append(p); mps.append(p.mean()); nr.append(norms(o, Xp, L1p, L2p))
        Xs.append(o.X[rows]); L1s.append(o.L1[rows]); L2s.append(o.L2[rows])
        print(f"cube200 iteration {it + 1}: MPSNR {p.mean():.6f}  ({time.time() - t0:.0f} s)", flush=True)
    out.update(psnr=np.stack(ps), mpsnr=np.array(mps), norms=np.array(nr), X=np.stack(Xs), L1=np.stack(L1s),
               L2=np.stack(L2s))
    np.savez_compressed(os.path.join(HERE, "cube200_oracle_2iter.npz"), **out)


def cube196_sc():
    Y, M, D, clean = problem(196, 196, 198, 36)
    P, B = Y.shape
    rows, cols = O.block_grid(P, B, 36, 36)
    blocks = O.im2col(Y, 36, rows, cols)
    obs = (blocks != 0).astype(np.uint8)
    nb = rows.size
    al = np.empty(nb, np.float32)
    th = np.empty(nb, np.float64)
    cache = {}
    for j in range(nb):
        k = obs[j].tobytes()
        if k not in cache:
            cache[k] = O.ista_alpha_h(D[obs[j].astype(bool)], 0.1, "fro4")
        al[j], th[j] = cache[k]
    t0 = time.time()
    X, PHI = O.ista_batch(blocks, obs, D, al, th, 100)
    print(f"cube196 sparse coding: {nb} blocks ({time.time() - t0:.0f} s)", flush=True)
    sel = np.arange(0, nb, BLOCK_STRIDE)
    np.savez_compressed(os.path.join(HERE, "cube196_bb36_sc.npz"), blocks=sel, phi=PHI[sel], coefs=X[sel])


def cube512_sc():
    """BASELINE configs[3]'s sparse coding (512x512x224, bb 36, 50,974 blocks, fro4, Nit 100): the
    oracle ISTA of every 53rd block only (blocks are independent), from the first outer iteration's
    input X = Y."""
    Y, M, D, clean = problem(512, 512, 224, 36)
    P, B = Y.shape
    rows, cols = O.block_grid(P, B, 36, 36)
    nb = rows.size
    sel = np.arange(0, nb, BLOCK_STRIDE)
    blocks = O.im2col(Y, 36, rows[sel], cols[sel])
    obs = (blocks != 0).astype(np.uint8)
    al = np.empty(sel.size, np.float32)
    th = np.empty(sel.size, np.float64)
    cache = {}
    for j in range(sel.size):
        k = obs[j].tobytes()
        if k not in cache:
            cache[k] = O.ista_alpha_h(D[obs[j].astype(bool)], 0.1, "fro4")
        al[j], th[j] = cache[k]
    t0 = time.time()
    X, PHI = O.ista_batch(blocks, obs, D, al, th, 100)
    print(f"cube512 sparse coding: {sel.size} of {nb} blocks ({time.time() - t0:.0f} s)", flush=True)
    # coefficients of all selected blocks, Phi of every 4th of them (fixture size)
    np.savez_compressed(os.path.join(HERE, "cube512_bb36_sc.npz"), blocks=sel, nb=np.int64(nb), coefs=X,
                        phi_blocks=sel[::4], phi=PHI[::4])


if __name__ == "__main__":
    which = sys.argv[1:] or ["cube196", "cube200"]
    if "cube512" in which:
        cube512_sc()
    if "cube196" in which:
        cube196_sc()
    if "cube200" in which:
        cube200()
