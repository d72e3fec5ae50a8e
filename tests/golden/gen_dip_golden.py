"""Generate tests/golden/dip_golden.npz and skip_golden.npz from the reference's own
my_Lipschitz_Unet and skip() networks (run in the BUILD CONTAINER only; /root/reference never
reaches the GPU box).

    python tests/golden/gen_dip_golden.py

The reference module is imported from /root/reference/models (CPU torch, float32) and trained
exactly as get_DIP_out does (main_LRS_PnP_DIP_1-LiP.py:214-237): Adam(lr=0.1), loss =
MSE(target*mask, out*mask), `steps` iterations.  Its parameters are set from a seeded numpy
generator (the reference's own init draws from the unseeded torch RNG), so the fixture stores
the seed and the recipe, not the 1.6 M weights:
  per conv unit i: W_bar ~ U(-sqrt(6/fan_in), +) ; bias ~ U(-1/sqrt(fan_in), +)
  per BN: gamma_orig = 1 + 0.25 u (some > 1: the Lipschitz rescale c is exercised), beta_orig = 0.1 u
drawn in the engine's flat order (tests/dip_ref.param_offsets).  Inputs: data_img5 noisy cube as
target, lrs_mask as the mask, a seeded U(0,1) input (the reference feeds X + L2/mu2).
Saved (float32): out after each step (every 5th element), loss per step, per-parameter gradient
norms of step 0, sigma_max of each conv at step 0.  skip_golden.npz: the same for the skip net of
main_LRS_PnP_DIP_pro.py:215-221 (5 scales of 128 channels, 128-channel skips, reflection pad,
nearest upsample, Sigmoid) with nn.Conv2d-default-scaled weights; its parameters are loaded in
the reference's parameters() order, which is the engine's flat layout.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "lrs-pnp-dip_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

SEED = 1234
STEPS = 3
SUB = 5


def flat_params(nodes, seed, c0=128, H=36, W=36):
    """Seeded parameters in the engine's flat layout: conv W ~ U(+-sqrt(6/fan_in)) (kaiming a=0) or
    U(+-1/sqrt(fan_in)) (nn.Conv2d default) per node winit, bias ~ U(+-1/sqrt(fan_in)), gamma =
    1 + 0.25 u, beta = 0.1 u."""
    import dip_ref
    offs, n = dip_ref.param_offsets(nodes, c0, H, W)
    sh = dip_ref.shapes(nodes, c0, H, W)
    rng = np.random.default_rng(seed)
    flat = np.zeros(n, np.float32)
    for i, (d, (w, b, g, be)) in enumerate(zip(dip_ref.node_dicts(nodes), offs)):
        C = sh[i + 1][0]
        if w >= 0:
            fan = sh[d["in0"]][0] * d["k"] * d["k"]
            bound = np.sqrt(6.0 / fan) if d["winit"] == 1 else 1 / np.sqrt(fan)
            flat[w:w + C * fan] = rng.uniform(-bound, bound, C * fan)
            flat[b:b + C] = rng.uniform(-1 / np.sqrt(fan), 1 / np.sqrt(fan), C)
        if g >= 0:
            flat[g:g + C] = 1.0 + 0.25 * rng.uniform(-1, 1, C)
            flat[be:be + C] = 0.1 * rng.uniform(-1, 1, C)
    return flat


def problem(seed):
    d = np.load(os.path.join(HERE, "data_img5.npz"))
    target = d["noisy_img5"][0].astype(np.float32)            # (128, 36, 36)
    mask = d["lrs_mask"].astype(np.float32)                   # (36, 36)
    x = np.random.default_rng(seed + 1).uniform(0, 1, target.shape).astype(np.float32)
    return x, target, mask


def skip_golden():
    """The reference's skip() net with the pro settings (main_LRS_PnP_DIP_pro.py:215-221)."""
    from models.skip import skip   # the reference module itself
    from lrspnp.dip import skip_nodes
    import dip_ref

    torch.manual_seed(0)
    nodes = skip_nodes(128, 128)
    flat = flat_params(nodes, SEED + 1)
    net = skip(128, 128, num_channels_down=[128] * 5, num_channels_up=[128] * 5, num_channels_skip=[128] * 5,
               filter_size_up=3, filter_size_down=3, upsample_mode="nearest", filter_skip_size=1,
               need_sigmoid=True, need_bias=True, pad="reflection", act_fun="LeakyReLU")
    params = list(net.parameters())
    # the engine's flat layout is the reference's named_parameters() order (conv W, b, BN w, b)
    assert sum(p.numel() for p in params) == flat.size, (sum(p.numel() for p in params), flat.size)
    off = 0
    with torch.no_grad():
        for p in params:
            p.copy_(torch.from_numpy(flat[off:off + p.numel()]).view_as(p))
            off += p.numel()
    x, target, mask = problem(SEED + 1)
    X, T, M = torch.from_numpy(x)[None], torch.from_numpy(target)[None], torch.from_numpy(mask)[None, None]
    opt = torch.optim.Adam(net.parameters(), 0.1)
    mse = torch.nn.MSELoss()
    outs, losses, gnorm = [], [], None
    for it in range(STEPS):
        opt.zero_grad()
        out = net(X)
        loss = mse(T * M, out * M)
        loss.backward()
        if it == 0:
            gnorm = [float(p.grad.norm()) for p in params]
        opt.step()
        outs.append(out.detach()[0].numpy().reshape(-1)[::SUB].copy())
        losses.append(float(loss.detach()))
    np.savez_compressed(os.path.join(HERE, "skip_golden.npz"), seed=np.int64(SEED + 1), steps=np.int64(STEPS),
                        sub=np.int64(SUB), out_sub=np.stack(outs).astype(np.float32),
                        loss=np.array(losses, np.float64), grad_norms=np.array(gnorm, np.float64))
    print("skip losses", losses)


def main():
    sys.path.insert(0, "/root/reference")
    skip_golden()
    from models.my_Lipschitz_Unet import my_Lipschitz_Unet   # the reference module itself
    from lrspnp.dip import UNET_REF_NAMES, lipschitz_unet_units
    import dip_ref

    torch.manual_seed(0)
    units = lipschitz_unet_units(128, 128, 128)
    flat = flat_params(units, SEED)
    offs, _ = dip_ref.param_offsets(units, 128)
    net = my_Lipschitz_Unet(num_input_channels=128, num_output_channels=128, ln_lambda=1, pad="reflection")
    sd = dict(net.named_parameters())
    with torch.no_grad():
        for i, (cp, bp) in enumerate(UNET_REF_NAMES):
            W, b, g, be = dip_ref.views(torch.from_numpy(flat), units, i, offs)
            sd[cp + ".weight_bar"].copy_(W)
            sd[cp + ".bias"].copy_(b)
            if bp:
                sd[bp + ".weight_orig"].copy_(g)
                sd[bp + ".bias_orig"].copy_(be)
    x, target, mask = problem(SEED)
    X = torch.from_numpy(x)[None]
    T = torch.from_numpy(target)[None]
    M = torch.from_numpy(mask)[None, None]
    opt = torch.optim.Adam(net.parameters(), 0.1)
    mse = torch.nn.MSELoss()
    outs, losses, gnorm = [], [], None
    sig = []
    for cp, _ in UNET_REF_NAMES:
        mod = dict(net.named_modules())[cp]
        w = mod.weight_bar.detach()
        sig.append(float(torch.svd(w.view(w.shape[0], -1), some=False, compute_uv=False)[1][0]))
    for it in range(STEPS):
        opt.zero_grad()
        out = net(X)
        loss = mse(T * M, out * M)
        loss.backward()
        if it == 0:
            gnorm = []
            for cp, bp in UNET_REF_NAMES:
                gnorm.append(float(sd[cp + ".weight_bar"].grad.norm()))
                gnorm.append(float(sd[cp + ".bias"].grad.norm()))
                if bp:
                    gnorm.append(float(sd[bp + ".weight_orig"].grad.norm()))
                    gnorm.append(float(sd[bp + ".bias_orig"].grad.norm()))
                else:
                    gnorm += [0.0, 0.0]
        opt.step()
        outs.append(out.detach()[0].numpy().reshape(-1)[::SUB].copy())
        losses.append(float(loss))
    np.savez_compressed(os.path.join(HERE, "dip_golden.npz"), seed=np.int64(SEED), steps=np.int64(STEPS),
                        sub=np.int64(SUB), out_sub=np.stack(outs).astype(np.float32),
                        loss=np.array(losses, np.float64), grad_norms=np.array(gnorm, np.float64),
                        sigma=np.array(sig, np.float64))
    print("losses", losses)
    print("sigma", np.round(sig, 5))


if __name__ == "__main__":
    main()
