"""Bisect a step-0 gradient drift on small sub-networks (diagnostic): grads of the engine's
lrs_dipnet_backward against the fp64 / fp32 torch restatement for a given dL/dout."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
for p in ("../lrs-pnp-dip_amd", "../tests/golden", "../tests", ".."):
    sys.path.insert(0, os.path.join(HERE, p))
import torch  # noqa: E402
from gen_dip_golden import flat_params  # noqa: E402
from lrspnp.dip import DipNet, conv_node, BN_LIP, BN_NONE, ACT_LRELU, ACT_NONE  # noqa: E402
import dip_ref  # noqa: E402


def rel(a, b):
    a = torch.as_tensor(a).double().cpu(); b = torch.as_tensor(b).double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


def run(name, units, C, H, xs, gscale=1.0, gmean=0.0):
    flat = torch.from_numpy(flat_params(units, 31, C, H, H))
    net = DipNet(units, C, H, H)
    net.params.copy_(flat.cuda())
    net.reset_optimizer()
    g = torch.Generator().manual_seed(3)
    x = xs(g)
    out = net.forward(x.cuda())
    gout = (torch.randn(out.shape, generator=g) * gscale + gmean).float()
    net.backward(x.cuda(), gout.cuda())
    torch.cuda.synchronize()
    gd = net.grads.cpu()
    res = {}
    for dt in (torch.float64, torch.float32):
        p = flat.to(dt).clone().requires_grad_(True)
        o = dip_ref.forward(p, units, x.to(dt))
        o.backward(gout.to(dt))
        res[dt] = (o.detach(), p.grad.double())
    offs, _ = dip_ref.param_offsets(units, C, H, H)
    s = f"{name}: out {rel(out, res[torch.float64][0]):.1e}"
    for i in range(len(units)):
        Wg, bg, gg, beg = dip_ref.views(gd, units, i, offs, C, H, H)
        Wr, br, gr, ber = dip_ref.views(res[torch.float64][1], units, i, offs, C, H, H)
        W32, b32, g32, be32 = dip_ref.views(res[torch.float32][1], units, i, offs, C, H, H)
        s += f" | n{i} W {rel(Wg, Wr):.1e} ({rel(W32, Wr):.1e})"
        if gg is not None:
            s += f" g {rel(gg, gr):.1e} ({rel(g32, gr):.1e}) be {rel(beg, ber):.1e} ({rel(be32, ber):.1e})"
        else:
            s += f" b {rel(bg, br):.1e} ({rel(b32, br):.1e})"
    print(s, flush=True)


rnd = lambda C, H: (lambda g: torch.rand(C, H, H, generator=g))
for H in (36, 64):
    two = [conv_node(0, 0, 128, 1), conv_node(1, 0, 128, 1, bn=BN_NONE)]
    run(f"1x1bn+1x1 H{H}", two, 128, H, rnd(128, H))
    run(f"1x1bn+1x1 H{H} gmean", two, 128, H, rnd(128, H), gscale=0.1, gmean=1.0)
    one = [conv_node(0, 0, 128, 1)]
    run(f"1x1bn H{H}", one, 128, H, rnd(128, H))
    run(f"1x1bn H{H} gmean", one, 128, H, rnd(128, H), gscale=0.1, gmean=1.0)
    run(f"1x1bn H{H} gmean10", one, 128, H, rnd(128, H), gscale=0.01, gmean=1.0)
    three = [conv_node(0, 0, 128, 3), conv_node(1, 0, 128, 1)]
    run(f"3x3bn+1x1bn H{H} gmean", three, 128, H, rnd(128, H), gscale=0.1, gmean=1.0)
