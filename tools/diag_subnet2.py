"""Full U-Net vs sub-nets, train_steps (loss head) vs backward(gout) (diagnostic)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
for p in ("../lrs-pnp-dip_amd", "../tests/golden", "../tests", ".."):
    sys.path.insert(0, os.path.join(HERE, p))
import torch  # noqa: E402
from gen_dip_golden import flat_params  # noqa: E402
from lrspnp.dip import DipNet, conv_node, lipschitz_unet_units, BN_NONE  # noqa: E402
import dip_ref  # noqa: E402


def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


def run(name, units, C, H, mode, Ho=None):
    Ho = Ho or H
    flat = torch.from_numpy(flat_params(units, 31, C, H, H))
    net = DipNet(units, C, H, H)
    net.params.copy_(flat.cuda())
    net.reset_optimizer()
    g = torch.Generator().manual_seed(8)
    x, t = torch.rand(C, H, H, generator=g), torch.rand(C, Ho, Ho, generator=g)
    m = (torch.rand(Ho * Ho, generator=g) > 0.1).float()
    res = {}
    for dt in (torch.float64, torch.float32):
        p = flat.to(dt).clone().requires_grad_(True)
        o = dip_ref.forward(p, units, x.to(dt))
        o.retain_grad()
        dip_ref.loss_fn(o, t.to(dt), m.to(dt)).backward()
        res[dt] = (o.detach(), p.grad.double(), o.grad.detach())
    if mode == "train":
        net.train_steps(x.cuda(), t.cuda(), m.cuda(), 1, use_graph=False)
    else:
        net.forward(x.cuda())
        net.backward(x.cuda(), res[torch.float64][2].float().cuda())
    torch.cuda.synchronize()
    gd = net.grads.cpu()
    offs, _ = dip_ref.param_offsets(units, C, H, H)
    s = f"{name} [{mode}]:"
    for i in range(len(units)):
        Wg, bg, gg, beg = dip_ref.views(gd, units, i, offs, C, H, H)
        Wr, br, gr, ber = dip_ref.views(res[torch.float64][1], units, i, offs, C, H, H)
        W32, *_ = dip_ref.views(res[torch.float32][1], units, i, offs, C, H, H)
        s += f" n{i} {rel(Wg, Wr):.1e}({rel(W32, Wr):.1e})"
    print(s, flush=True)


H = 36
u = lipschitz_unet_units(128, 128, 128)
for mode in ("train", "bwd"):
    run("unet", u, 128, H, mode)
    run("last2", [conv_node(0, 0, 128, 1), conv_node(1, 0, 128, 1, bn=BN_NONE)], 128, H, mode)
    run("up4+last2", [conv_node(0, 0, 128, 3, up=1)] + [conv_node(1, 0, 128, 1), conv_node(2, 0, 128, 1, bn=BN_NONE)],
        128, H // 2, mode, Ho=H)

# the [last1, last2] tail fed with the full net's own out11 (reference activations)
flat = torch.from_numpy(flat_params(u, 31, 128, H, H))
g = torch.Generator().manual_seed(8)
x = torch.rand(128, H, H, generator=g)
_, acts = dip_ref.forward(flat.double(), u, x.double(), return_all=True)
out11 = acts[10][0].float()       # output of node 10 = input of node 11 (up_4)? print shapes
print("act shapes", [tuple(a.shape) for a in acts])
for k in (10, 11):
    xin = acts[k][0].float()
    print(f"act {k}: mean {float(xin.mean()):.3f} std {float(xin.std()):.3f} min {float(xin.min()):.3f} max {float(xin.max()):.3f}")
tail = [conv_node(0, 0, 128, 1), conv_node(1, 0, 128, 1, bn=BN_NONE)]
xin = acts[11][0].float()
Ht = xin.shape[-1]
flat2 = torch.from_numpy(flat_params(tail, 31, 128, Ht, Ht))
net = DipNet(tail, 128, Ht, Ht)
net.params.copy_(flat2.cuda()); net.reset_optimizer()
res = {}
gg = torch.Generator().manual_seed(4)
gout = torch.randn(128, Ht, Ht, generator=gg)
for dt in (torch.float64, torch.float32):
    p = flat2.to(dt).clone().requires_grad_(True)
    dip_ref.forward(p, tail, xin.to(dt)).backward(gout.to(dt))
    res[dt] = p.grad.double()
net.forward(xin.cuda()); net.backward(xin.cuda(), gout.float().cuda()); torch.cuda.synchronize()
offs, _ = dip_ref.param_offsets(tail, 128, Ht, Ht)
for i in range(2):
    Wg, *_ = dip_ref.views(net.grads.cpu(), tail, i, offs, 128, Ht, Ht)
    Wr, *_ = dip_ref.views(res[torch.float64], tail, i, offs, 128, Ht, Ht)
    W32, *_ = dip_ref.views(res[torch.float32], tail, i, offs, 128, Ht, Ht)
    print(f"tail on out11: n{i} W {rel(Wg, Wr):.1e} ({rel(W32, Wr):.1e})")

# exact loss gradient of the full net, pushed through the tail with the reference's out11
print("---- tail with the full net's loss gradient")
p = flat.double().clone().requires_grad_(True)
gx = torch.Generator().manual_seed(8)
x = torch.rand(128, H, H, generator=gx); t = torch.rand(128, H, H, generator=gx)
m = (torch.rand(H * H, generator=gx) > 0.1).float()
o, acts = dip_ref.forward(p, u, x.double(), return_all=True)
o.retain_grad()
dip_ref.loss_fn(o, t.double(), m.double()).backward()
gout = o.grad.detach()
xin = acts[11][0].detach()
tail_flat = torch.cat([flat[int(a):int(b)] for a, b in []]) if False else None
offs_u, _ = dip_ref.param_offsets(u, 128, H, H)
# the tail's parameters = the full net's nodes 12, 13 (same flat layout order)
lo = offs_u[12][0]
flat_t = flat[lo:].clone()
net = DipNet(tail, 128, H, H)
assert net.n_params == flat_t.numel(), (net.n_params, flat_t.numel())
net.params.copy_(flat_t.cuda()); net.reset_optimizer()
for name, xi in (("ref out11", xin.float()),):
    res = {}
    for dt in (torch.float64, torch.float32):
        pp = flat_t.to(dt).clone().requires_grad_(True)
        dip_ref.forward(pp, tail, xi.to(dt)).backward(gout.to(dt))
        res[dt] = pp.grad.double()
    net.forward(xi.cuda()); net.backward(xi.cuda(), gout.float().cuda()); torch.cuda.synchronize()
    offs, _ = dip_ref.param_offsets(tail, 128, H, H)
    for i in range(2):
        Wg, bg, gg, beg = dip_ref.views(net.grads.cpu(), tail, i, offs, 128, H, H)
        Wr, br, gr, ber = dip_ref.views(res[torch.float64], tail, i, offs, 128, H, H)
        W32, *_ = dip_ref.views(res[torch.float32], tail, i, offs, 128, H, H)
        print(f"{name}: n{i} W {rel(Wg, Wr):.1e} ({rel(W32, Wr):.1e})", flush=True)
