"""Diagnostic: time variants of the split-bf16 ISTA kernel (lrs_diag_ista_b3_variant), one process,
interleaved reps.  Usage: python tools/diag_b3.py [nb] [Nit] [variants, comma-separated]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lrspnp import _lib  # noqa: E402
from lrspnp.data import synthetic_dictionary  # noqa: E402

NAMES = {0: "baseline", 1: "no shuffles", 2: "no NLM", 3: "no MFMA", 4: "2 waves/SIMD", 5: "seq pair NLM", 9: "v9", 10: "ln2", 11: "ln2+gb", 12: "ln2 tile-major", 13: "+fold alpha", 14: "+fold+div1", 15: "+fold+div0",
         6: "variant6", 7: "variant7", 8: "variant8"}
L = _lib.device_lib()
f = L.lrs_diag_ista_b3_variant
vp, i64, i32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
f.restype = i32
f.argtypes = [vp, vp, vp, i64, i64, i64, vp, vp, i32, i32, vp, vp]
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
Nit = int(sys.argv[2]) if len(sys.argv) > 2 else 80
variants = [int(v) for v in sys.argv[3].split(",")] if len(sys.argv) > 3 else [0, 1, 2, 3, 4, 5]
rng = np.random.default_rng(0)
D = torch.from_numpy(synthetic_dictionary(64, 256, 0)).cuda()
Yb = torch.from_numpy((rng.standard_normal((nb, 64)) * 0.3).astype(np.float32)).cuda()
obs = torch.from_numpy((rng.random((nb, 64)) > 0.05).astype(np.uint8)).cuda()
alpha = torch.full((nb,), 5.0, device="cuda")
thr = torch.full((nb,), 3e-3, dtype=torch.float64, device="cuda")
phi = torch.empty((nb, 64), device="cuda")
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
times = {v: [] for v in variants}
ref = None
for rep in range(4):
    for v in variants:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert f(P(Yb), P(obs), P(D), 64, 64, nb, P(alpha), P(thr), Nit, v, P(phi), s) == 0
        e1.record()
        torch.cuda.synchronize()
        if rep:
            times[v].append(e0.elapsed_time(e1))
        if rep == 0 and v == variants[0]:
            ref = phi.clone()
        elif rep == 0:
            d = float((phi - ref).norm() / ref.norm())
            print(f"variant {v}: rel diff vs variant {variants[0]} {d:.3e}", flush=True)
for v in variants:
    print(f"{v} {NAMES[v]:>16s}: {np.median(times[v]):8.3f} ms", flush=True)
