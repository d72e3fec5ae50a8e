"""Diagnostic: SVT apply kernel time per rows-per-wave variant (dbg 1: 16, 2: 32, 0: 64 rows)."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]
import torch

from lrspnp import _lib, ops

L = _lib.device_lib()
f = L.lrs_diag_svt_apply
vp = ctypes.c_void_p
f.argtypes = [vp, vp, ctypes.c_float, ctypes.c_int64, ctypes.c_int64, vp, vp, ctypes.c_int, vp]
P, B = 40000, 198
X = torch.randn(P, B, device="cuda")
L2 = torch.randn(P, B, device="cuda")
U = torch.empty_like(X)
ws = ops.svt_workspace(P, B, "cuda")
s = vp(torch.cuda.current_stream().cuda_stream)
for dbg in (0, 1, 2, 0):
    ts = []
    for rep in range(6):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        assert f(vp(X.data_ptr()), vp(L2.data_ptr()), 1.0, P, B, vp(ws.data_ptr()), vp(U.data_ptr()), dbg, s) == 0
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"dbg {dbg}: {min(ts[1:]) * 1e3:.1f} us", flush=True)
