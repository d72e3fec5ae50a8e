"""Diagnostic: SVT stage timings (isolated, synchronised) and Jacobi rounds/sweeps per call,
on the bench workload's cube evolving through LRS-PnP outer iterations."""
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
obs, clean, mask = synthetic_cube(H, W, B, seed=0, base_mask=load_fixture("data_img5.npz")["lrs_mask"])
s = LrsPnP(unfold(obs), mask_matrix(mask, B), synthetic_dictionary(64, 256, 0), LrsPnPConfig(bb=8, sliding=8, Nit=80))
for it in range(6):
    warm = it > 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ops.svt_gram(s.X, s.L2, s.c2, s.svt_ws, warm=warm)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ops.svt_finish(s.X, s.L2, s.c2, s.tau, s.svt_ws, s.U, warm=warm)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    st = ops.svt_state(s.svt_ws, s.P, s.B)
    print(f"iter {it}: gram {1e3*(t1-t0):7.3f} ms  finish {1e3*(t2-t1):7.3f} ms  rounds {st[2]} sweeps {st[3]}")
    s.step()
    torch.cuda.synchronize()
