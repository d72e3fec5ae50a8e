"""Diagnostic: time ablated variants of the resident ISTA kernel (one process, interleaved)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]
import numpy as np
import torch

from lrspnp import _lib
from lrspnp.data import synthetic_dictionary

L = _lib.device_lib()
f = L.lrs_diag_ista_ablate_f32
vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
f.restype = i32
f.argtypes = [vp, vp, vp, i64, i64, i64, vp, vp, i32, i32, vp, vp]
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
Nit = int(sys.argv[2]) if len(sys.argv) > 2 else 80
rng = np.random.default_rng(0)
D = torch.from_numpy(synthetic_dictionary(64, 256, 0)).cuda()
Yb = torch.from_numpy((rng.standard_normal((nb, 64)) * 0.3).astype(np.float32)).cuda()
obs = torch.from_numpy((rng.random((nb, 64)) > 0.05).astype(np.uint8)).cuda()
alpha = torch.full((nb,), 5.0, device="cuda")
thr = torch.full((nb,), 3e-3, dtype=torch.float64, device="cuda")
phi = torch.empty((nb, 64), device="cuda")
P = lambda t: ctypes.c_void_p(t.data_ptr())
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
times = {0: [], 1: [], 2: []}
for rep in range(4):
    for ab in (0, 1, 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert f(P(Yb), P(obs), P(D), 64, 64, nb, P(alpha), P(thr), Nit, ab, P(phi), s) == 0
        e1.record()
        torch.cuda.synchronize()
        if rep:
            times[ab].append(e0.elapsed_time(e1))
names = {0: "full", 1: "no-NLM (MFMA+move)", 2: "no-MFMA (NLM+move)"}
for ab in (0, 1, 2):
    print(f"{names[ab]:22s} median {np.median(times[ab]):8.3f} ms  min {np.min(times[ab]):8.3f}")
