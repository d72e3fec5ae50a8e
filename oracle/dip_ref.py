"""Plain-PyTorch fp32 restatement of the DIP networks and their training step (oracle).

TEST INFRASTRUCTURE ONLY (imported by tests/ and by bench.py's cpu_baseline leg): the numerics tests compare the HIP engine (lrs_dipnet_*) against this
module, and tests/test_dip_ref.py pins this module against outputs of the reference's own
my_Lipschitz_Unet and skip networks (tests/golden/dip_golden.npz, skip_golden.npz, made by
tests/golden/gen_dip_golden.py).

It follows, statement by statement:
  models/lipschitz_constraint_layer.py:36-44   sigma = svd(W.view(Co,-1))[0]; W = W_bar / max(1, sigma)
                                               (computed here in fp64, then rounded to float32)
  lipschitz_constraint_layer.py:65-78          ReflectionPad2d((k-1)//2) then Conv2d(pad 0)
  lipschitz_constraint_layer.py:88-101         c = max(max|gamma_orig|, 1); BN(gamma/c, beta/c), train mode
  lipschitz_constraint_layer.py:6-22           LeakyReLU(0.2)
  my_Lipschitz_Unet.py:71-94                   nn.Upsample(scale_factor=2, mode='nearest')
  models/common.py:11-42                       Concat: centre-crop to the smaller H, W, then cat
  models/skip.py:5-99                          the skip network (plain BatchNorm2d, Sigmoid)
  main_LRS_PnP_DIP_1-LiP.py:215-237            Adam(lr), loss = MSE(target*mask, out*mask)
The network is the engine's node list (lrspnp.dip.DipNode); parameters live in one flat vector
with the engine's layout (per CONV node: W, bias, [gamma, beta]; per BN node: gamma, beta).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

CONV, BN, CONCAT = 0, 1, 2


def node_dicts(nodes):
    return [n.as_dict() if hasattr(n, "as_dict") else dict(n) for n in nodes]


def shapes(nodes, c0, H, W):
    """Output (C, H, W) of every tensor: index 0 = input, i + 1 = node i."""
    sh = [(c0, H, W)]
    for d in node_dicts(nodes):
        c, h, w = sh[d["in0"]]
        if d["kind"] == CONV:
            hu, wu = (2 * h, 2 * w) if d["upsample"] else (h, w)
            ho = (hu + 2 * d["pad"] - d["k"]) // d["stride"] + 1
            wo = (wu + 2 * d["pad"] - d["k"]) // d["stride"] + 1
            sh.append((d["cout"], ho, wo))
        elif d["kind"] == BN:
            sh.append((c, h, w))
        else:
            cb, hb, wb = sh[d["in1"]]
            if d["upsample"]:
                hb, wb = 2 * hb, 2 * wb
            sh.append((c + cb, min(h, hb), min(w, wb)))
    return sh


def param_offsets(nodes, c0=None, H=36, W=36):
    """Flat offsets (w, b, gamma, beta) per node, -1 when absent — the engine's layout."""
    nd = node_dicts(nodes)
    if c0 is None:
        c0 = 128
    sh = shapes(nodes, c0, H, W)
    offs, p = [], 0
    for i, d in enumerate(nd):
        C = sh[i + 1][0]
        w = b = g = be = -1
        if d["kind"] == CONV:
            kc = sh[d["in0"]][0] * d["k"] * d["k"]
            w = p; p += C * kc
            b = p; p += C
        if d["kind"] != CONCAT and d["bn"]:
            g = p; p += C
            be = p; p += C
        offs.append((w, b, g, be))
    return offs, p


def views(flat, nodes, i, offs, c0=128, H=36, W=36):
    d = node_dicts(nodes)[i]
    sh = shapes(nodes, c0, H, W)
    w, b, g, be = offs[i]
    C = sh[i + 1][0]
    Wt = bt = None
    if d["kind"] == CONV:
        cin = sh[d["in0"]][0]
        Wt = flat[w:w + C * cin * d["k"] * d["k"]].view(C, cin, d["k"], d["k"])
        bt = flat[b:b + C]
    return Wt, bt, (flat[g:g + C] if g >= 0 else None), (flat[be:be + C] if be >= 0 else None)


def sigma_scale(W):
    m = W.detach().reshape(W.shape[0], -1).double()
    s = torch.linalg.svdvals(m)[0].to(W.dtype)
    return s, torch.maximum(torch.ones_like(s), s)


def _bn(z, g, be, lip):
    c = max(float(g.detach().abs().max()), 1.0) if lip else 1.0
    return F.batch_norm(z, None, None, g / c, be / c, training=True, momentum=0.1, eps=1e-5)


def _act(z, a):
    if a == 1:
        return F.leaky_relu(z, 0.2)
    if a == 2:
        return torch.sigmoid(z)
    return z


def forward(flat, nodes, x, return_all=False):
    """x: (C0, H, W) -> output of the last node (C, H', W')."""
    c0, H, W = x.shape
    offs, _ = param_offsets(nodes, c0, H, W)
    ts = [x.unsqueeze(0)]
    for i, d in enumerate(node_dicts(nodes)):
        Wt, bt, g, be = views(flat, nodes, i, offs, c0, H, W)
        h = ts[d["in0"]]
        if d["kind"] == CONV:
            if d["sn"]:
                _, sc = sigma_scale(Wt)
                Wt = Wt / sc
            if d["upsample"]:
                h = F.interpolate(h, scale_factor=2, mode="nearest")
            if d["pad"] > 0:
                p = d["pad"]
                h = F.pad(h, (p, p, p, p), mode="reflect" if d["pad_mode"] == 1 else "constant")
            z = F.conv2d(h, Wt, bt, stride=d["stride"])
            if d["bn"]:
                z = _bn(z, g, be, d["bn"] == 2)
            z = _act(z, d["act"])
        elif d["kind"] == BN:
            z = _act(_bn(h, g, be, d["bn"] == 2), d["act"])
        else:
            hb = ts[d["in1"]]
            if d["upsample"]:
                hb = F.interpolate(hb, scale_factor=2, mode="nearest")
            Ht, Wt2 = min(h.shape[2], hb.shape[2]), min(h.shape[3], hb.shape[3])
            parts = []
            for t in (h, hb):
                d2, d3 = (t.shape[2] - Ht) // 2, (t.shape[3] - Wt2) // 2
                parts.append(t[:, :, d2:d2 + Ht, d3:d3 + Wt2])
            z = torch.cat(parts, dim=1)
        ts.append(z)
    return (ts[-1][0], ts[1:]) if return_all else ts[-1][0]


def loss_fn(out, target, mask):
    m = mask.view(1, *out.shape[1:]) if mask is not None else 1.0
    return F.mse_loss(target * m, out * m)


class RefTrainer:
    """get_DIP_out's inner loop (…1-LiP.py:229-237) on the flat parameter vector."""

    def __init__(self, nodes, flat0, lr=0.1):
        self.units = nodes
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
