"""MPSNR trajectory of the ORACLE-driven LRS-PnP-DIP(1-Lip) outer loop on the bench's configs[2]
cube (run in the BUILD CONTAINER only, ~10 min per seed for 8 outer iterations on 6 cores):

    OMP_NUM_THREADS=6 python tests/golden/gen_dip196_traj.py 5 8 [out.npz]   # -> dip196_traj_ref.npz (5 seeds x 8)

The reference's main_LRS_PnP_DIP_1-LiP.py cannot run this cube: its my_Lipschitz_Unet hardcodes
128 bands (models/my_Lipschitz_Unet.py:33-101), and the cube has 198.  So the outer loop is the
oracle's restatement of the main (oracle.LrsPnpOracle: main_LRS_PnP.py:244-366 with the DIP mains'
parameters, …1-LiP.py:316-345 -- fro4 ISTA, Nit 100, mu1 = mu2 = 0.1, gamma 0.5), everything on the
host and nothing of lrspnp's device code:
  * sparse coding: the oracle's C ISTA + NLM prox over the 6,408 36x36 blocks (pinned to the
    reference's ista / skimage, tests/test_oracle.py);
  * the low-rank prox: get_DIP_out (…1-LiP.py:208-238, early stopping off, 100 Adam steps as the
    bench) on oracle/dip_ref.py's plain-torch U-Net (198 -> 128 -> 198 bands; pinned to the
    reference modules, tests/test_dip_ref.py), float32 CPU torch, full-SVD sigma_max per conv, a
    fresh net per outer iteration initialised as the reference's layers are (kaiming_uniform for
    the Lipschitz convs, the nn.Conv2d default for the others, BN gamma = 1, beta = 0) from
    torch.Generator(seed * 1000 + iteration); the input image and U follow the reference's reshapes
    (…1-LiP.py:404, :411);
  * the X / dual update: the oracle's C col2im + closed form (main_LRS_PnP.py:324-366).
Saved: seeds (S,), mpsnr (S, iters) after each outer iteration, mpsnr_input, loss_last (S, iters)
(the last DIP step's masked MSE) and the cube parameters.  tests/test_gpu_e2e_dip.py compares
lrspnp.LrsPnP's per-iteration mean MPSNR over its own seeds with these (DIP trajectories are not
reproducible, even by the reference: tests/test_dip_ref.py).
"""
import hashlib
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lrspnp.data import load_fixture, mask_matrix, synthetic_cube, synthetic_dictionary, unfold  # noqa: E402
from lrspnp.dip import lipschitz_unet_nodes  # noqa: E402
from oracle import dip_ref  # noqa: E402
from oracle import oracle as O  # noqa: E402

H = W = 196
B = 198
BB = 36
DIP_STEPS = 100
OUT = os.path.join(HERE, "dip196_traj_ref.npz")


def problem():
    """bench.py make_problem(196, 196, 198, 36, 256, seed=0)."""
    base = load_fixture("data_img5.npz")["lrs_mask"]
    obs, clean, mask = synthetic_cube(H, W, B, seed=0, base_mask=base)
    return unfold(obs), mask_matrix(mask, B), synthetic_dictionary(BB * BB, 256, 0), clean


def ref_init(nodes, gen):
    """Reference layer init in the engine's flat layout (dip_ref.param_offsets)."""
    offs, n = dip_ref.param_offsets(nodes, B, H, W)
    sh = dip_ref.shapes(nodes, B, H, W)
    flat = torch.zeros(n, dtype=torch.float32)
    for i, (d, (w, b, g, be)) in enumerate(zip(dip_ref.node_dicts(nodes), offs)):
        C = sh[i + 1][0]
        if w >= 0:
            fan = sh[d["in0"]][0] * d["k"] * d["k"]
            bound = np.sqrt(6.0 / fan) if d["winit"] == 1 else 1 / np.sqrt(fan)
            flat[w:w + C * fan] = (torch.rand(C * fan, generator=gen, dtype=torch.float64) * 2 - 1).float() * bound
            flat[b:b + C] = (torch.rand(C, generator=gen, dtype=torch.float64) * 2 - 1).float() / np.sqrt(fan)
        if g >= 0:
            flat[g:g + C] = 1.0
            flat[be:be + C] = 0.0
    return flat


class DipLowRank:
    """get_DIP_out(target, X + L2/mu2) with early stopping off: 100 steps, the last step's output."""

    def __init__(self, Y, M, seed):
        self.nodes = lipschitz_unet_nodes(B, B, 128)
        img = lambda Z: torch.from_numpy(np.ascontiguousarray(Z.T.reshape(Z.shape[1], W, H).transpose(0, 2, 1)))
        self.img = img
        self.target = img(Y)                                   # the observed cube as an image
        self.mask = img(M[:, :1]).reshape(-1)                  # mask_bkg: the pixel mask
        self.seed, self.calls, self.loss = seed, 0, []

    def __call__(self, Xlr):
        gen = torch.Generator().manual_seed(self.seed * 1000 + self.calls)
        self.calls += 1
        tr = dip_ref.RefTrainer(self.nodes, ref_init(self.nodes, gen), lr=0.1)
        x = self.img(Xlr)                                       # …1-LiP.py:404
        for _ in range(DIP_STEPS):
            out, loss, _ = tr.step(x, self.target, self.mask)
        self.loss.append(loss)
        U = out.numpy()[None].transpose(0, 1, 3, 2).reshape(B, -1).transpose(1, 0)   # :411
        return np.ascontiguousarray(U, dtype=np.float32)


_memo = {}
_ista = O.ista_batch


def ista_memo(Yb, OBS, *a, **k):
    """The first outer iteration's sparse coding is the same for every seed (X = Y): run it once."""
    key = hashlib.sha1(np.ascontiguousarray(Yb).tobytes()).hexdigest()
    if key not in _memo:
        _memo[key] = _ista(Yb, OBS, *a, **k)
    return _memo[key]


def main(seeds=5, iters=4, out=OUT):
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "8")))
    O.ista_batch = ista_memo
    Y, M, D, clean = problem()
    mp0 = float(O.psnr_bands(Y, clean).mean())
    res = {"seeds": [], "mpsnr": [], "loss_last": []}
    for seed in range(seeds):
        dip = DipLowRank(Y, M, seed)
        o = O.LrsPnpOracle(Y, M, D, bb=BB, sliding=BB, gamma=0.5, mu1=0.1, mu2=0.1, lambda_ista=0.1, Nit=100,
                           variant="fro4", lowrank=dip)
        mp = []
        for it in range(iters):
            t0 = time.time()
            o.step()
            mp.append(float(O.psnr_bands(o.X, clean).mean()))
            print(f"seed {seed} iteration {it + 1}: MPSNR {mp[-1]:.4f} (input {mp0:.4f}), last DIP loss "
                  f"{dip.loss[-1]:.6g}, {time.time() - t0:.0f}s", flush=True)
        res["seeds"].append(seed)
        res["mpsnr"].append(mp)
        res["loss_last"].append(dip.loss)
        np.savez(out, seeds=np.array(res["seeds"]), mpsnr=np.array(res["mpsnr"]),
                 loss_last=np.array(res["loss_last"]), mpsnr_input=np.float64(mp0),
                 cube=np.array([H, W, B, BB, 256, 100, DIP_STEPS]))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]), *(sys.argv[3:4] or [OUT]))
