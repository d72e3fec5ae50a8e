"""Diagnostic: the in-register MATLAB-variant NLM prox vs the oracle, per vector and atom."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]
import numpy as np
import torch

from lrspnp import _lib
from oracle import oracle as O

L = _lib.device_lib()
f = L.lrs_diag_nlm_matlab
vp = ctypes.c_void_p
f.argtypes = [vp, vp, ctypes.c_int64, vp, vp]
rng = np.random.default_rng(0)
nb = 32
g = (rng.standard_normal((nb, 256)) * 0.1).astype(np.float32)
h = np.full(nb, 0.05)
gd, hd = torch.from_numpy(g).cuda(), torch.from_numpy(h).cuda()
out = torch.empty_like(gd)
assert f(vp(gd.data_ptr()), vp(hd.data_ptr()), nb, vp(out.data_ptr()), vp(torch.cuda.current_stream().cuda_stream)) == 0
o = out.cpu().numpy()
ref = np.stack([O.nlm_matlab_col(g[j], h[j]) for j in range(nb)])
d = np.abs(o - ref)
print("max abs diff", d.max(), "rel", d.max() / np.abs(ref).max())
bad = np.argwhere(d > 1e-6 * np.abs(ref).max())
print("bad (vector, atom) count", len(bad), "atoms:", sorted(set(bad[:, 1].tolist()))[:40])
