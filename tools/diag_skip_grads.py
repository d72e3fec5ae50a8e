"""Per-node gradient agreement of the engine (skip net) vs fp64 / fp32 torch restatement."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("lrs-pnp-dip_amd", "tests", "tests/golden"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch
import dip_ref, gen_dip_golden as G
from lrspnp.dip import DipNet, skip_nodes
nodes = skip_nodes(128, 128)
flat = torch.from_numpy(G.flat_params(nodes, 1235)); x, t, m = (torch.from_numpy(a) for a in G.problem(1235))
gr = {}
for dt in (torch.float64, torch.float32):
    p = flat.to(dt).clone().requires_grad_(True)
    dip_ref.loss_fn(dip_ref.forward(p, nodes, x.to(dt)), t.to(dt), m.reshape(-1).to(dt)).backward()
    gr[dt] = p.grad.double()
net = DipNet(nodes, 128, 36, 36); net.params.copy_(flat.cuda()); net.reset_optimizer()
net.train_steps(x.cuda(), t.cuda(), m.reshape(-1).cuda(), 1, use_graph=False); torch.cuda.synchronize()
gd = net.grads.cpu().double()
offs, _ = dip_ref.param_offsets(nodes, 128)
r = lambda a, b: float((a - b).norm() / max(float(b.norm()), 1e-30))
for i, nd in enumerate(nodes):
    A, B, C = (dip_ref.views(g, nodes, i, offs) for g in (gd, gr[torch.float64], gr[torch.float32]))
    print(i, nd.kind, " ".join("%s gpu %.1e cpu32 %.1e" % (n, r(a, b), r(c, b)) for n, a, b, c in zip("Wbgt", A, B, C) if a is not None))
# structure of the node-34 weight-gradient error
i = 34
A, B = dip_ref.views(gd, nodes, i, offs)[0][:, :, 0, 0], dip_ref.views(gr[torch.float64], nodes, i, offs)[0][:, :, 0, 0]
E = (A - B).abs()
print("max err", float(E.max()), "max |ref|", float(B.abs().max()))
rows = E.max(1).values; cols = E.max(0).values
print("worst rows", rows.topk(5).indices.tolist(), rows.topk(5).values.tolist())
print("worst cols", cols.topk(5).indices.tolist(), cols.topk(5).values.tolist())
print("row err by 16-block", [round(float(rows[k:k+16].max() / B.abs().max()), 5) for k in range(0, 128, 16)])
print("col err by 16-block", [round(float(cols[k:k+16].max() / B.abs().max()), 5) for k in range(0, 128, 16)])
# determinism: the same step again from the same state
net2 = DipNet(nodes, 128, 36, 36); net2.params.copy_(flat.cuda()); net2.reset_optimizer()
net2.train_steps(x.cuda(), t.cuda(), m.reshape(-1).cuda(), 1, use_graph=False); torch.cuda.synchronize()
g2 = net2.grads.cpu().double()
d = (g2 - gd).abs()
print("run-to-run max diff", float(d.max()), "n differing", int((d > 0).sum()))
A2 = dip_ref.views(g2, nodes, 34, offs)[0][:, :, 0, 0]
print("row81 err run2", float((A2[81] - B[81]).abs().max()))
