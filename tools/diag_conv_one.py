"""Run one conv shape's implicit forward + backward N times (for rocprofv3 --pmc passes).

python tools/diag_conv_one.py cin cout H W k stride pad up [reps]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lrs-pnp-dip_amd"))
from lrspnp import _lib  # noqa: E402

L = _lib.device_lib()
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
cin, cout, H, W, k, s, p, up = (int(v) for v in sys.argv[1:9])
reps = int(sys.argv[9]) if len(sys.argv) > 9 else 5
torch.manual_seed(0)
x = torch.randn(cin, H, W, device="cuda")
w = torch.randn(cout, cin, k, k, device="cuda") * 0.05
b = torch.zeros(cout, device="cuda")
Ho, Wo = ctypes.c_int(), ctypes.c_int()
L.lrs_conv2d_out_size(H, W, k, s, p, up, ctypes.byref(Ho), ctypes.byref(Wo))
nws = L.lrs_conv2d_workspace(cin, H, W, cout, k, s, p, up, None)
ws = torch.empty(nws // 4 + 1, device="cuda")
y = torch.empty(cout, Ho.value, Wo.value, device="cuda")
gy = torch.randn_like(y)
gx, gw = torch.empty_like(x), torch.empty_like(w)
div = torch.ones(1, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(reps):
    assert L.lrs_conv2d_fwd_f32(P(x), cin, H, W, P(w), P(b), cout, k, s, p, 1, up, None, P(y), None, P(ws), nws, st) == 0
    assert L.lrs_conv2d_bwd_x_f32(P(gy), P(x), P(w), P(div), cin, H, W, cout, k, s, p, 1, up,
                                  P(gx), P(gw), None, P(ws), nws, st) == 0
torch.cuda.synchronize()
print("ok")
