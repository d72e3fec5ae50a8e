"""Dump the configs[2] / configs[3] sparse coding (per-pattern Gram path) of the loaded library to an
.npz, so two builds can be compared bit for bit (A/B of output-preserving kernel changes).

    LRSPNP_LIB=<lib> python tools/pat_dump.py out.npz [cfg2|cfg3]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lrspnp import LrsPnP, LrsPnPConfig  # noqa: E402
from lrspnp.data import load_fixture, mask_matrix, synthetic_cube, synthetic_dictionary, unfold  # noqa: E402

out = sys.argv[1]
which = sys.argv[2] if len(sys.argv) > 2 else "cfg2"
H, W, B = (196, 196, 198) if which == "cfg2" else (512, 512, 224)
base = load_fixture("data_img5.npz")["lrs_mask"]
obs, clean, mask = synthetic_cube(H, W, B, seed=0, base_mask=base)
s = LrsPnP(unfold(obs), mask_matrix(mask, B), synthetic_dictionary(1296, 256, 0), LrsPnPConfig.dip_1lip(lowrank="svt"))
assert s.pat_plan is not None
phi, coefs = s.sparse_coding(want_coefs=True)
torch.cuda.synchronize()
np.savez(out, phi=phi.cpu().numpy(), coefs=coefs.cpu().numpy())
print("dumped", out, phi.shape)
