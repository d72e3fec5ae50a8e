"""Phase timing of k_sn_sigma on the real U-Net weights after a few Adam steps.

    python tools/diag_sigma_net.py [C=198] [H=196] [steps=0,5,30]

Prints per conv: the Lanczos step count at exit, and the load / Lanczos / final-multisection time."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lrs-pnp-dip_amd"))
import torch  # noqa: E402

from lrspnp import _lib  # noqa: E402
from lrspnp.dip import DipNet, lipschitz_unet_nodes  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 198
H = int(sys.argv[2]) if len(sys.argv) > 2 else 196
marks = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0,5,30").split(",")]
L = _lib.device_lib()
net = DipNet(lipschitz_unet_nodes(C, C), C, H, H)
net.init_params(1)
g = torch.Generator(device="cuda").manual_seed(0)
x = torch.rand(C, H, H, device="cuda", generator=g)
t = torch.rand(net.out_shape, device="cuda", generator=g)
m = (torch.rand(net.out_shape[1:], device="cuda", generator=g) > 0.2).float()
done = 0
for mk in marks:
    if mk > done:
        net.train_steps(x, t, m, mk - done, use_graph=False)
        done = mk
    torch.cuda.synchronize()
    mats = []
    for i in range(len(net.nodes)):
        w = net.param_views(i)[0]
        if w is not None and net.nodes[i].sn:
            mats.append(w.reshape(w.shape[0], -1).contiguous())
    n = len(mats)
    W = (ctypes.c_void_p * n)(*[a.data_ptr() for a in mats])
    rows = (ctypes.c_int * n)(*[a.shape[0] for a in mats])
    cols = (ctypes.c_int * n)(*[a.shape[1] for a in mats])
    nb = L.lrs_sigma_max_workspace(n) + 8 * n
    ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
    prof = torch.zeros(8 * n, dtype=torch.int64, device="cuda")
    for _ in range(3):
        assert L.lrs_diag_sigma_phases(W, rows, cols, n, ctypes.c_void_p(ws.data_ptr()), nb,
                                       ctypes.c_void_p(prof.data_ptr()), None) == 0
        torch.cuda.synchronize()
    p = prof.view(n, 8).cpu()
    sv = [float(torch.linalg.matrix_norm(a.double(), 2)) for a in mats]
    print(f"after {mk} steps")
    for i in range(n):
        t0 = p[i, 0]
        print(f"  conv {i:2d} {tuple(mats[i].shape)} sigma {sv[i]:.4f}: load {(p[i, 1] - t0) / 100:6.1f} us  "
              f"lanczos {(p[i, 2] - p[i, 1]) / 100:6.1f} us (k={int(p[i, 4])}, checks {p[i, 5] / 100:6.1f} us = {int(p[i, 6])} clk)  final {(p[i, 3] - p[i, 2]) / 100:5.1f} us")
