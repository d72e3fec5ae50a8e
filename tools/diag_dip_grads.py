"""Per-layer gradient agreement of the engine vs tests/dip_ref.py (fp32 CPU and fp64 CPU)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("lrs-pnp-dip_amd", "tests", "tests/golden"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch
import dip_ref, gen_dip_golden as G
from lrspnp.dip import DipNet, lipschitz_unet_units
units = lipschitz_unet_units(128, 128, 128)
flat = torch.from_numpy(G.flat_params(units, 1234)); x, t, m = (torch.from_numpy(a) for a in G.problem(1234))
def grads(dtype):
    p = flat.to(dtype).clone().requires_grad_(True)
    out = dip_ref.forward(p, units, x.to(dtype)); loss = dip_ref.loss_fn(out, t.to(dtype), m.reshape(-1).to(dtype)); loss.backward()
    return p.grad.double(), [a.detach().double() for a in dip_ref.forward(p.detach(), units, x.to(dtype), True)[1]]
g32, a32 = grads(torch.float32); g64, a64 = grads(torch.float64)
net = DipNet(units, 36, 36); net.params.copy_(flat.cuda()); net.reset_optimizer()
net.train_steps(x.cuda(), t.cuda(), m.reshape(-1).cuda(), 1, use_graph=False); torch.cuda.synchronize()
gd = net.grads.cpu().double()
offs, _ = dip_ref.param_offsets(units)
r = lambda a, b: float((a - b).norm() / max(float(b.norm()), 1e-30))
for i in range(14):
    a, b, c = dip_ref.views(gd, units, i, offs), dip_ref.views(g32, units, i, offs), dip_ref.views(g64, units, i, offs)
    s = "%2d W gpu/64 %.2e cpu32/64 %.2e" % (i, r(a[0], c[0]), r(b[0], c[0]))
    if a[2] is not None:
        s += " | gamma %.2e %.2e beta %.2e %.2e" % (r(a[2], c[2]), r(b[2], c[2]), r(a[3], c[3]), r(b[3], c[3]))
    else:
        s += " | bias %.2e %.2e" % (r(a[1], c[1]), r(b[1], c[1]))
    print(s)
