"""Plain-PyTorch fp32 restatement of the 1-Lipschitz U-Net and its training step (test reference).

TEST INFRASTRUCTURE ONLY: the numerics tests compare the HIP engine (lrs_dipnet_*) against this
module, and tests/test_dip_ref.py pins this module against outputs of the reference's own
my_Lipschitz_Unet (tests/golden/dip_golden.npz, made by tests/golden/gen_dip_golden.py).

It follows, statement by statement:
  models/lipschitz_constraint_layer.py:36-44   sigma = svd(W.view(Co,-1))[0]; W = W_bar / max(1, sigma)
                                               (computed here in fp64, then rounded to float32)
  lipschitz_constraint_layer.py:65-78          ReflectionPad2d((k-1)//2) then Conv2d(pad 0)
  lipschitz_constraint_layer.py:88-101         c = max(max|gamma_orig|, 1); BN(gamma/c, beta/c), train mode
  lipschitz_constraint_layer.py:6-22           LeakyReLU(0.2)
  my_Lipschitz_Unet.py:71-94                   nn.Upsample(scale_factor=2, mode='nearest')
  main_LRS_PnP_DIP_1-LiP.py:215-237            Adam(lr), loss = MSE(target*mask, out*mask)
Parameters live in one flat vector with the engine's layout (per unit: W_bar, bias, gamma, beta).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def unit_dicts(units):
    return [u.as_dict() if hasattr(u, "as_dict") else dict(u) for u in units]


def param_offsets(units):
    """Flat offsets (w, b, gamma, beta) per unit, -1 when absent — the engine's layout."""
    offs, p = [], 0
    for u in unit_dicts(units):
        kc = u["cin"] * u["k"] * u["k"]
        w = p; p += u["cout"] * kc
        b = p; p += u["cout"]
        g = be = -1
        if u["bn"]:
            g = p; p += u["cout"]
            be = p; p += u["cout"]
        offs.append((w, b, g, be))
    return offs, p


def views(flat, units, i, offs):
    u = unit_dicts(units)[i]
    w, b, g, be = offs[i]
    kc = u["cin"] * u["k"] * u["k"]
    W = flat[w:w + u["cout"] * kc].view(u["cout"], u["cin"], u["k"], u["k"])
    return W, flat[b:b + u["cout"]], (flat[g:g + u["cout"]] if g >= 0 else None), \
        (flat[be:be + u["cout"]] if be >= 0 else None)


def sigma_scale(W):
    m = W.detach().reshape(W.shape[0], -1).double()
    s = torch.linalg.svdvals(m)[0].float()
    return s, torch.maximum(torch.ones_like(s), s)


def forward(flat, units, x, return_all=False):
    """x: (C, H, W) float32 -> (C_out, H, W)."""
    offs, _ = param_offsets(units)
    h = x.unsqueeze(0)
    acts = []
    for i, u in enumerate(unit_dicts(units)):
        W, b, g, be = views(flat, units, i, offs)
        _, sc = sigma_scale(W)
        Wn = W / sc
        if u["upsample"]:
            h = F.interpolate(h, scale_factor=2, mode="nearest")
        if u["pad"] > 0:
            p = u["pad"]
            h = F.pad(h, (p, p, p, p), mode="reflect" if u["pad_mode"] == 1 else "constant")
        z = F.conv2d(h, Wn, b, stride=u["stride"])
        if u["bn"]:
            c = max(float(g.detach().abs().max()), 1.0)
            z = F.batch_norm(z, None, None, g / c, be / c, training=True, momentum=0.1, eps=1e-5)
        if u["act"] == 1:
            z = F.leaky_relu(z, 0.2)
        elif u["act"] == 2:
            z = torch.sigmoid(z)
        h = z
        acts.append(h)
    return (h[0], acts) if return_all else h[0]


def loss_fn(out, target, mask):
    m = mask.view(1, *out.shape[1:]) if mask is not None else 1.0
    return F.mse_loss(target * m, out * m)


class RefTrainer:
    """get_DIP_out's inner loop (…1-LiP.py:229-237) on the flat parameter vector."""

    def __init__(self, units, flat0, lr=0.1):
        self.units = units
        self.p = flat0.detach().clone().requires_grad_(True)
        self.opt = torch.optim.Adam([self.p], lr)

    def step(self, x, target, mask):
        self.opt.zero_grad()
        out = forward(self.p, self.units, x)
        loss = loss_fn(out, target, mask)
        loss.backward()
        g = self.p.grad.detach().clone()
        self.opt.step()
        return out.detach(), float(loss.detach()), g


class EarlyStopRef:
    """EarlyStop + the variance test of get_DIP_out (…1-LiP.py:71-99, 244-264), numpy float32."""

    def __init__(self, size=30, patience=60):
        self.size, self.patience = size, patience
        self.wait, self.best, self.coll, self.stop, self.stop_epoch = 0, float("inf"), [], False, None
        self.vars = []

    def update(self, img, epoch):
        import numpy as np
        self.coll.append(np.asarray(img, np.float32).reshape(-1))
        if len(self.coll) > self.size:
            self.coll.pop(0)
        if len(self.coll) == self.size:
            ave = np.mean(np.stack(self.coll).astype(np.float64), axis=0)
            var = float(np.mean([((ave - t) ** 2).sum() / t.size for t in self.coll]))
            self.vars.append(var)
            if not self.stop:
                if var < self.best:
                    self.best, self.wait = var, 0
                else:
                    self.wait += 1
                    if self.wait >= self.patience:
                        self.stop, self.stop_epoch = True, epoch
        return self.stop
