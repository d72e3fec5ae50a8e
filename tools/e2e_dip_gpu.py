"""LRS-PnP-DIP end to end on the reference's own 36x36x128 data, as main_LRS_PnP_DIP_1-LiP.py /
main_LRS_PnP_DIP_pro.py run it (early stopping on, mu1 = mu2 = 0.1, Nit 100), over several DIP
init seeds: per outer iteration MPSNR / MSSIM / DIP steps -> JSON (compare with
tests/golden/dip_e2e_ref.npz, the reference's own runs).

    python tools/e2e_dip_gpu.py [--seeds 5] [--iters 4] [--out gpurun_out/e2e_dip.json]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "lrs-pnp-dip_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from lrspnp import LrsPnP, LrsPnPConfig  # noqa: E402
from lrspnp.data import mask_matrix, synthetic_dictionary, unfold  # noqa: E402
from lrspnp.metrics import fold, mpsnr, mssim  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--seeds", type=int, default=5)
ap.add_argument("--iters", type=int, default=4)
ap.add_argument("--out", default="gpurun_out/e2e_dip.json")
a = ap.parse_args()
d = np.load(os.path.join(HERE, "..", "tests", "golden", "data_img5.npz"))
Y, M = unfold(d["noisy"][0]), mask_matrix(d["lrs_mask"], 128)
D = synthetic_dictionary(1296, 256, 0)
clean = torch.from_numpy(d["clean"][0]).cuda()
res = {}
for net in ("1lip", "pro"):
    mk = LrsPnPConfig.dip_1lip if net == "1lip" else LrsPnPConfig.dip_pro
    rows = []
    for seed in range(a.seeds):
        s = LrsPnP(Y, M, D, mk(dip_seed=1000 * seed), image_shape=(36, 36))
        mp, ms = [], []
        for _ in range(a.iters):
            s.step()
            mp.append(float(mpsnr(s.X, clean)))
            ms.append(float(mssim(clean, fold(s.X, 36, 36))))   # pytorch_ssim.ssim(gt, generated) (:480)
        # training steps up to the returned output: the stop epoch + 1 (the reference's count of its
        # per-step prints), or all steps run when early stopping never fired
        steps = [int(e) + 1 if e is not None else int(n) for n, e in s.dip_steps]
        rows.append({"seed": seed, "mpsnr": mp, "mssim": ms, "dip_steps": steps})
        print(net, seed, np.round(mp, 4), np.round(ms, 4), steps, flush=True)
    res[net] = rows
os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
json.dump(res, open(a.out, "w"), indent=1)
