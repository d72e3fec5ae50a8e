"""Time DIP training steps (lrs_dipnet_train_steps) at the native 36x36x128 and the generalised
196x196x198 sizes, eager vs hipGraph replay.  Prints one JSON line per configuration."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lrs-pnp-dip_amd"))

import torch  # noqa: E402

from lrspnp.dip import DipNet, lipschitz_unet_units  # noqa: E402


def run(bands, H, steps, graph):
    net = DipNet(lipschitz_unet_units(bands, bands, 128), bands, H, H)
    net.init_params(1)
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.rand(bands, H, H, device="cuda", generator=g)
    t = torch.rand(bands, H, H, device="cuda", generator=g)
    m = (torch.rand(H * H, device="cuda", generator=g) > 0.2).float()
    net.train_steps(x, t, m, 3, use_graph=graph)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    net.train_steps(x, t, m, steps, use_graph=graph)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"bands": bands, "H": H, "graph": graph, "steps": steps, "ms_per_step": dt / steps * 1e3,
            "steps_per_s": steps / dt, "loss": net.last_loss()}


if __name__ == "__main__":
    if len(sys.argv) > 1:      # bands H steps graph
        b, h, n, gr = (int(v) for v in sys.argv[1:5])
        print(json.dumps(run(b, h, n, bool(gr))), flush=True)
    else:
        for bands, H, steps in ((128, 36, 200), (198, 196, 20)):
            for graph in (False, True):
                print(json.dumps(run(bands, H, steps, graph)), flush=True)
