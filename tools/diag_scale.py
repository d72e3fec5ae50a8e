"""Is the U-Net gradient drift a uniform scale?  Per node: best-fit scale of engine/ref W grads and the
residual after removing it (diagnostic)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
for p in ("../lrs-pnp-dip_amd", "../tests/golden", "../tests", ".."):
    sys.path.insert(0, os.path.join(HERE, p))
import torch  # noqa: E402
from gen_dip_golden import flat_params  # noqa: E402
from lrspnp.dip import DipNet, lipschitz_unet_units  # noqa: E402
import dip_ref  # noqa: E402

H = 36
u = lipschitz_unet_units(128, 128, 128)
flat = torch.from_numpy(flat_params(u, 31, 128, H, H))
g = torch.Generator().manual_seed(8)
x, t = torch.rand(128, H, H, generator=g), torch.rand(128, H, H, generator=g)
m = (torch.rand(H * H, generator=g) > 0.1).float()
p = flat.double().clone().requires_grad_(True)
o, acts = dip_ref.forward(p, u, x.double(), return_all=True)
for a in acts:
    a.retain_grad()
o.retain_grad()
dip_ref.loss_fn(o, t.double(), m.double()).backward()
net = DipNet(u, 128, H, H)
net.params.copy_(flat.cuda()); net.reset_optimizer()
net.forward(x.cuda())
net.backward(x.cuda(), o.grad.float().cuda())
torch.cuda.synchronize()
gd = net.grads.cpu().double()
offs, _ = dip_ref.param_offsets(u, 128, H, H)
for i in range(len(u)):
    Wg, bg, gg, beg = dip_ref.views(gd, u, i, offs, 128, H, H)
    Wr, br, gr, ber = dip_ref.views(p.grad, u, i, offs, 128, H, H)
    s = float((Wg * Wr).sum() / (Wr * Wr).sum())
    res = float((Wg - s * Wr).norm() / Wr.norm())
    line = f"node {i}: scale-1 {s - 1:+.2e} residual {res:.1e}"
    if gg is not None:
        sg = float((gg * gr).sum() / (gr * gr).sum())
        line += f"  gamma scale-1 {sg - 1:+.2e} res {float((gg - sg * gr).norm() / gr.norm()):.1e}"
    print(line, flush=True)
print("act grad norms", [f"{float(a.grad.norm()):.2e}" for a in acts])
print("---- per-node buffers vs fp64 reference (out_i, dL/dout_i)")
for i in range(len(u)):
    ob = net.node_buffer(i, 0)
    gb = net.node_buffer(i, 3)
    ra = acts[i][0].detach()
    rg = acts[i].grad[0] if acts[i].grad is not None else None
    print(f"node {i}: out {float((ob.double().cpu() - ra).norm() / ra.norm()):.1e}"
          + (f"  grad {float((gb.double().cpu() - rg).norm() / rg.norm()):.1e}" if rg is not None else ""), flush=True)
print("---- node 12 local: z, dL/dz")
import torch.nn.functional as F  # noqa: E402
W12, b12, g12, be12 = dip_ref.views(flat.double(), u, 12, offs, 128, H, H)
_, sc = dip_ref.sigma_scale(W12)
xin = acts[11].detach()
z = F.conv2d(xin, W12 / sc, b12).requires_grad_(True)
from oracle import dip_ref as odr  # noqa: E402
y = odr._act(odr._bn(z, g12, be12, True), 1)
y.backward(acts[12].grad)
zb = net.node_buffer(12, 1).double().cpu()
gzb = net.node_buffer(12, 2).double().cpu()
print(f"z12 {float((zb - z[0].detach()).norm() / z.norm()):.1e}  gz12 {float((gzb - z.grad[0]).norm() / z.grad.norm()):.1e}")
zc = z[0].detach() - z[0].detach().mean(dim=(1, 2), keepdim=True)
print(f"z12 centred err {float(((zb - zb.mean(dim=(1, 2), keepdim=True)) - zc).norm() / zc.norm()):.1e}",
      f"z12 mean/std ratio {float(z[0].detach().mean(dim=(1,2)).abs().mean() / z[0].detach().std(dim=(1,2)).mean()):.2e}")
gy = acts[12].grad[0]
gm = gy.mean(dim=(1, 2), keepdim=True)
print(f"gy12 mean/std ratio {float(gm.abs().mean() / gy.std(dim=(1,2)).mean()):.2e}; |dz|/|gy| {float(z.grad.norm()/gy.norm()):.2e}")
print("---- LeakyReLU branch flips (engine out > 0 vs reference out > 0)")
for i in range(len(u)):
    ob = net.node_buffer(i, 0).double().cpu()
    ra = acts[i][0].detach()
    flips = int(((ob > 0) != (ra > 0)).sum())
    near = float(ra.abs().min())
    print(f"node {i}: flips {flips}  min|out| {near:.2e}")
