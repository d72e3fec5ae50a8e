"""ISTA kernel time in the bench step (beside the SVT chain) vs alone on the same inputs."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]
import numpy as np, torch
import bench
from lrspnp import LrsPnP, LrsPnPConfig, ops
Y, M, D, clean = bench.make_problem(200, 200, 198, 8, 256, seed=0)
s = LrsPnP(Y, M, D, LrsPnPConfig(bb=8, sliding=8, Nit=80, variant="spec2"))
for _ in range(3):
    s.step()
torch.cuda.synchronize()
def t_alone():
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.ista(s.Yb, s.obs, s.D, s.n, s.alpha, s.thr, 80, s.prox, phi=s.phi)
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1)
print("alone", [round(t_alone(), 3) for _ in range(3)])
# with the SVT chain concurrently on the low-rank stream
lr = s.lowrank_stream
res = []
for _ in range(3):
    lr.wait_stream(torch.cuda.current_stream())
    ops.svt_gram(s.X, s.L2, s.c2, s.svt_ws, warm=True, stream=lr)
    ops.svt_finish(s.X, s.L2, s.c2, s.tau, s.svt_ws, s.U, warm=True, stream=lr)
    res.append(t_alone())
print("beside SVT", [round(v, 3) for v in res])
