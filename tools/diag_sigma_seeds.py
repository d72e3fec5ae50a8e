"""sigma_max of every U-Net conv weight for several parameter seeds vs fp64 SVD (diagnostic)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
for p in ("../lrs-pnp-dip_amd", "../tests/golden", "../tests", ".."):
    sys.path.insert(0, os.path.join(HERE, p))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gen_dip_golden import flat_params  # noqa: E402
from lrspnp.dip import lipschitz_unet_units, sigma_max  # noqa: E402
import dip_ref  # noqa: E402

u = lipschitz_unet_units(128, 128, 128)
offs, _ = dip_ref.param_offsets(u, 128, 36, 36)
worst = []
for seed in list(range(20)) + [31, 1234]:
    flat = torch.from_numpy(flat_params(u, seed, 128, 36, 36))
    mats = []
    for i in range(len(u)):
        W, *_ = dip_ref.views(flat, u, i, offs, 128, 36, 36)
        mats.append(W.reshape(W.shape[0], -1).contiguous())
    sig, _ = sigma_max([m.cuda() for m in mats])
    ref = np.array([float(torch.linalg.svdvals(m.double())[0]) for m in mats])
    err = np.abs(sig.cpu().double().numpy() - ref) / ref
    sv = [torch.linalg.svdvals(m.double())[:2].numpy() for m in mats]
    gaps = [1 - s[1] / s[0] for s in sv]
    k = int(np.argmax(err))
    worst.append(err.max())
    print(f"seed {seed}: max rel err {err.max():.2e} at node {k} (gap {gaps[k]:.2e}); errs>1e-6 at",
          [(i, f"{e:.1e}", f"{gaps[i]:.1e}") for i, e in enumerate(err) if e > 1e-6], flush=True)
