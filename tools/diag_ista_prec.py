"""ISTA kernel: f32-MFMA vs split-bf16 MFMA products, time and agreement on a bench-sized batch."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]
import numpy as np
import torch

from lrspnp import _lib, ops
from lrspnp.data import synthetic_dictionary

L = _lib.device_lib()
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
Nit = int(sys.argv[2]) if len(sys.argv) > 2 else 80
rng = np.random.default_rng(0)
D = torch.from_numpy(synthetic_dictionary(64, 256, 0)).cuda()
Yb = torch.from_numpy((rng.standard_normal((nb, 64)) * 0.3).astype(np.float32)).cuda()
obs = torch.from_numpy((rng.random((nb, 64)) > 0.05).astype(np.uint8)).cuda()
alpha, thr = ops.ista_alpha(D, obs[:1].contiguous(), 64, ops.ALPHA_SPEC2, 0.1)
alpha = alpha.expand(nb).contiguous()
thr = thr.expand(nb).contiguous()
out = {}
for prec in (0, 1, 0, 1, 0, 1):
    assert L.lrs_ista_set_precision(prec) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    phi, coefs = ops.ista(Yb, obs, D, 64, alpha, thr, Nit, ops.PROX_NLM, want_coefs=True)
    e1.record()
    torch.cuda.synchronize()
    out.setdefault(prec, []).append(e0.elapsed_time(e1))
    out[("phi", prec)] = phi.clone()
    out[("c", prec)] = coefs.clone()
L.lrs_ista_set_precision(1)
rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm())
print("f32 MFMA    ms", [round(t, 3) for t in out[0]])
print("split-bf16  ms", [round(t, 3) for t in out[1]])
print("rel L2 phi %.3e coefs %.3e" % (rel(out[("phi", 1)], out[("phi", 0)]), rel(out[("c", 1)], out[("c", 0)])))
