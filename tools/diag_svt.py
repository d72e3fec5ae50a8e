"""Diagnostic: SVT stage timings (isolated, synchronised) per eigensolver path, on the bench
workload's cube evolving through LRS-PnP outer iterations; U of the two paths compared.

    python tools/diag_svt.py [HxWxB] [iterations]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]
import numpy as np
import torch

from lrspnp import LrsPnP, LrsPnPConfig, ops
from lrspnp.data import load_fixture, mask_matrix, synthetic_cube, synthetic_dictionary, unfold

H, W, B = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "200x200x198").split("x"))
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
obs, clean, mask = synthetic_cube(H, W, B, seed=0, base_mask=load_fixture("data_img5.npz")["lrs_mask"])
s = LrsPnP(unfold(obs), mask_matrix(mask, B), synthetic_dictionary(64, 256, 0), LrsPnPConfig(bb=8, sliding=8, Nit=80))
wsj = ops.svt_workspace(s.P, s.B, "cuda")
Uj = torch.empty_like(s.U)
for it in range(iters):
    res = {}
    for method, ws, U in (("tri", s.svt_ws, s.U), ("jacobi", wsj, Uj)):
        warm = it > 0
        for rep in range(2):                      # second repetition is the timed one
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ops.svt_gram(s.X, s.L2, s.c2, ws, warm=warm, method=method)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ops.svt_finish(s.X, s.L2, s.c2, s.tau, ws, U, warm=warm, method=method)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
        st = ops.svt_state(ws, s.P, s.B)
        res[method] = (1e3 * (t1 - t0), 1e3 * (t2 - t1), st)
    d = (torch.linalg.norm(s.U - Uj) / torch.linalg.norm(Uj)).item()
    (g0, f0, st0), (g1, f1, st1) = res["tri"], res["jacobi"]
    print(f"iter {it}: tri gram {g0:6.3f} finish {f0:6.3f} ms path {st0[4]} | jacobi gram {g1:6.3f} "
          f"finish {f1:6.3f} ms sweeps {st1[3]} | rel(U_tri - U_jac) {d:.2e}", flush=True)
    s.step()
    torch.cuda.synchronize()
print("tridiagonal-path phases (us): load+tridiag, eigenvalues, inverse iteration, back-transform, "
      "certificate+orthogonalise, fallback+E:", [round(v, 1) for v in ops.svt_phase_us(s.svt_ws, s.P, s.B)])
