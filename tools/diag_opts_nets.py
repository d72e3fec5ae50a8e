"""Per-node step-0 gradient errors of U-Nets created with different lrs_dip_opts (diagnostic)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lrs-pnp-dip_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from gen_dip_golden import flat_params  # noqa: E402
from lrspnp.dip import DipNet, lipschitz_unet_units  # noqa: E402
from oracle import dip_ref  # noqa: E402


def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


H = int(sys.argv[1]) if len(sys.argv) > 1 else 36
for pad, opts in [("reflection", dict(precision=1)), ("reflection", dict(precision=0)),
                  ("zero", dict(upsample_dgrad=1)), ("zero", dict(upsample_dgrad=0))]:
    units = lipschitz_unet_units(128, 128, 128, pad=pad)
    flat = torch.from_numpy(flat_params(units, 31, 128, H, H))
    net = DipNet(units, 128, H, H, **opts)
    net.params.copy_(flat.cuda())
    net.reset_optimizer()
    g = torch.Generator().manual_seed(8)
    x, t = torch.rand(128, H, H, generator=g), torch.rand(128, H, H, generator=g)
    m = (torch.rand(H * H, generator=g) > 0.1).float()
    net.train_steps(x.cuda(), t.cuda(), m.cuda(), 1, use_graph=False)
    torch.cuda.synchronize()
    gd = net.grads.cpu()
    grads = {}
    for dt in (torch.float64, torch.float32):
        p = flat.to(dt).clone().requires_grad_(True)
        dip_ref.loss_fn(dip_ref.forward(p, units, x.to(dt)), t.to(dt), m.to(dt)).backward()
        grads[dt] = p.grad.double()
    offs, _ = dip_ref.param_offsets(units, 128, H, H)
    print(pad, opts, "flat", rel(gd, grads[torch.float64]), "fp32-torch flat", rel(grads[torch.float32], grads[torch.float64]))
    for i in range(len(units)):
        Wg, bg, gg, beg = dip_ref.views(gd, units, i, offs, 128, H, H)
        Wr, br, gr, ber = dip_ref.views(grads[torch.float64], units, i, offs, 128, H, H)
        W32, b32, g32, be32 = dip_ref.views(grads[torch.float32], units, i, offs, 128, H, H)
        print(f"  node {i}: W {rel(Wg, Wr):.2e} (fp32 {rel(W32, Wr):.2e})  b {rel(bg, br):.2e} (fp32 {rel(b32, br):.2e})"
              + (f"  gamma {rel(gg, gr):.2e} (fp32 {rel(g32, gr):.2e}) beta {rel(beg, ber):.2e}" if gg is not None else ""))
