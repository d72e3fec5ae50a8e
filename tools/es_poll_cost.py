"""Cost of the early-stopping polls (DipProx.run: train_steps in batches of poll_every steps, a 4-byte
state read after each) against the same steps in one call, wall clock, ES on and never stopping.

    python tools/es_poll_cost.py [--hw 196] [--bands 198] [--steps 200] [--poll 10]"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lrs-pnp-dip_amd"))
import torch  # noqa: E402
from lrspnp.dip import DipNet, EarlyStopper, lipschitz_unet_nodes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--hw", type=int, default=196)
ap.add_argument("--bands", type=int, default=198)
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--poll", type=int, default=10)
ap.add_argument("--rounds", type=int, default=5)
a = ap.parse_args()
net = DipNet(lipschitz_unet_nodes(a.bands, a.bands, 128), a.bands, a.hw, a.hw)
net.init_params(0)
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.rand(a.bands, a.hw, a.hw, device="cuda", generator=g)
t = torch.rand(a.bands, a.hw, a.hw, device="cuda", generator=g)
m = (torch.rand(a.hw, a.hw, device="cuda", generator=g) > 0.2).float()
es = EarlyStopper(a.bands * a.hw * a.hw, 30, 10 ** 6)
net.train_steps(x, t, m, 10, es=es)
torch.cuda.synchronize()
one, polled = [], []
for r in range(a.rounds):
    t0 = time.perf_counter()
    net.train_steps(x, t, m, a.steps, es=es)
    es.read(net.stream)
    one.append((time.perf_counter() - t0) * 1e3 / a.steps)
    t0 = time.perf_counter()
    done = 0
    while done < a.steps:
        k = min(a.poll, a.steps - done)
        net.train_steps(x, t, m, k, es=es)
        done += k
        es.read(net.stream)
    polled.append((time.perf_counter() - t0) * 1e3 / a.steps)
print(f"{a.hw}^2 ms per step: one call {statistics.median(one):.4f}, polled every {a.poll}: {statistics.median(polled):.4f}"
      f" -> {1e3 * (statistics.median(polled) - statistics.median(one)) * a.poll:.1f} us per poll")
