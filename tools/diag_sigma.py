"""Phase timing of the sigma_max kernel (k_sn_sigma) on 14 U-Net-shaped weights."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lrs-pnp-dip_amd"))
import torch
from lrspnp import _lib
L = _lib.device_lib()
shapes = [(128, 1152)] * 10 + [(128, 512)] * 2 + [(128, 128)] * 2
g = torch.Generator(device="cuda").manual_seed(0)
mats = [(torch.rand(s, device="cuda", generator=g) * 2 - 1) * (6 / s[1]) ** 0.5 for s in shapes]
n = len(mats)
W = (ctypes.c_void_p * n)(*[m.data_ptr() for m in mats])
rows = (ctypes.c_int * n)(*[s[0] for s in shapes]); cols = (ctypes.c_int * n)(*[s[1] for s in shapes])
nb = L.lrs_sigma_max_workspace(n) + 8 * n
ws = torch.empty(nb, dtype=torch.uint8, device="cuda")
prof = torch.zeros(8 * n, dtype=torch.int64, device="cuda")
for it in range(3):
    assert L.lrs_diag_sigma_phases(W, rows, cols, n, ctypes.c_void_p(ws.data_ptr()), nb, ctypes.c_void_p(prof.data_ptr()), None) == 0
    torch.cuda.synchronize()
p = prof.view(n, 8).cpu()
for i in range(n):
    t0 = p[i, 0]
    print(i, "load %.1f us  lanczos %.1f us (k=%d)  final %.1f us" % ((p[i, 1] - t0) / 100, (p[i, 2] - p[i, 1]) / 100, p[i, 4], (p[i, 3] - p[i, 2]) / 100))
