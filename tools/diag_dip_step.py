"""Time DIP training steps (lrs_dipnet_train_steps, graph replay) per net / size / GEMM precision.

GPU diagnostic: python tools/diag_dip_step.py  -> one line per case (ms per Adam step)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lrs-pnp-dip_amd"))
from lrspnp import _lib  # noqa: E402
from lrspnp.dip import DipNet, lipschitz_unet_nodes, skip_nodes  # noqa: E402

L = _lib.device_lib()
CASES = [("unet1lip", 128, 36, 36), ("unet1lip", 198, 196, 196), ("skip", 128, 36, 36), ("skip", 224, 512, 512)]


def nodes_for(net, C):
    return lipschitz_unet_nodes(C, C) if net == "unet1lip" else skip_nodes(C, C)


for net, C, H, W in CASES:
    for prec in ((1,) if os.environ.get('DIAG_B3_ONLY') else (0, 1)):
        L.lrs_dip_set_precision(prec)
        n = DipNet(nodes_for(net, C), C, H, W)
        n.init_params(1)
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.rand(C, H, W, device="cuda", generator=g)
        t = torch.rand(n.out_shape, device="cuda", generator=g)
        m = (torch.rand(n.out_shape[1:], device="cuda", generator=g) > 0.2).float()
        steps = 20 if H <= 200 else 5
        for graph in (False, True):
            n.train_steps(x, t, m, 2, use_graph=graph)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            n.train_steps(x, t, m, steps, use_graph=graph)
            e1.record()
            torch.cuda.synchronize()
            print(f"{net:9s} {C}x{H}x{W} precision {'split-bf16 implicit' if prec else 'f32 explicit    '} "
                  f"{'graph' if graph else 'eager'}: {e0.elapsed_time(e1) / steps:8.3f} ms/step  "
                  f"loss {n.last_loss():.6e}", flush=True)
        del n
L.lrs_dip_set_precision(1)
