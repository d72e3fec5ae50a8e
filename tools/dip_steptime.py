"""Median DIP training-step time (ms) of the bench's network (configs[2]: my_Lipschitz_Unet
198->128->198 on 196x196), for A/B of kernel builds (LRSPNP_LIB).  Several timed rounds of
`--steps` steps; prints each round and the median.

    python tools/dip_steptime.py [--hw 196] [--bands 198] [--steps 100] [--rounds 7] [--graph]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lrs-pnp-dip_amd"))
import torch  # noqa: E402
from lrspnp.dip import DipNet, lipschitz_unet_nodes, skip_nodes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--hw", type=int, default=196)
ap.add_argument("--bands", type=int, default=198)
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--graph", action="store_true")
ap.add_argument("--net", default="unet", choices=["unet", "skip"], help="the 1-Lip U-Net (configs[2]) or the skip "
                                                                          "net (configs[3])")
ap.add_argument("--priority", type=int, default=0, help="the net's stream priority (DipNet stream_priority; "
                                                         "its weight-gradient side stream follows it)")
ap.add_argument("--es", action="store_true", help="with the device early-stopping update every step (ring 30, "
                                                   "patience 60), as get_DIP_out runs with early stopping on")
ap.add_argument("--dump", default=None, help="also save the net output after the timed rounds (.npy): "
                                              "bit-for-bit A/B of output-preserving kernel changes")
a = ap.parse_args()
nodes = lipschitz_unet_nodes(a.bands, a.bands, 128) if a.net == "unet" else skip_nodes(a.bands, a.bands)
net = DipNet(nodes, a.bands, a.hw, a.hw, stream_priority=a.priority)
net.init_params(0)
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.rand(a.bands, a.hw, a.hw, device="cuda", generator=g)
t = torch.rand(a.bands, a.hw, a.hw, device="cuda", generator=g)
m = (torch.rand(a.hw, a.hw, device="cuda", generator=g) > 0.2).float()
es = None
if a.es:
    from lrspnp.dip import EarlyStopper
    es = EarlyStopper(a.bands * a.hw * a.hw, 30, 10 ** 6)   # never stops: every step runs the full test
net.train_steps(x, t, m, 10, use_graph=a.graph, es=es)
torch.cuda.synchronize()
res = []
for r in range(a.rounds):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    net.train_steps(x, t, m, a.steps, use_graph=a.graph, es=es)
    e1.record()
    torch.cuda.synchronize()
    res.append(e0.elapsed_time(e1) / a.steps)
print("dip step ms:", " ".join(f"{v:.4f}" for v in res), "median", f"{statistics.median(res):.4f}")
if a.dump:
    import numpy as np
    np.save(a.dump, net.output().detach().cpu().numpy())
