"""Host enqueue time vs GPU time of DIP training steps (is the step host-launch-bound?).

    python tools/host_enqueue.py [--hw 196] [--bands 198] [--steps 100] [--graph]
Prints, per round: host seconds to enqueue `steps` steps (train_steps returns without a sync) and
the wall time until the GPU finished them."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lrs-pnp-dip_amd"))
import torch  # noqa: E402
from lrspnp.dip import DipNet, lipschitz_unet_nodes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--hw", type=int, default=196)
ap.add_argument("--bands", type=int, default=198)
ap.add_argument("--steps", type=int, default=100)
ap.add_argument("--graph", action="store_true")
a = ap.parse_args()
net = DipNet(lipschitz_unet_nodes(a.bands, a.bands, 128), a.bands, a.hw, a.hw)
net.init_params(0)
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.rand(a.bands, a.hw, a.hw, device="cuda", generator=g)
t = torch.rand(a.bands, a.hw, a.hw, device="cuda", generator=g)
m = (torch.rand(a.hw, a.hw, device="cuda", generator=g) > 0.2).float()
net.train_steps(x, t, m, 10, use_graph=a.graph)
torch.cuda.synchronize()
for r in range(3):
    t0 = time.perf_counter()
    net.train_steps(x, t, m, a.steps, use_graph=a.graph)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0) / a.steps:.3f} ms/step, wall {1e3 * (t2 - t0) / a.steps:.3f} ms/step")
