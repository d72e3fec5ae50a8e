"""Time one conv layer (forward, or backward with --bwd) through the C ABI, HIP events.

    python tools/micro_conv.py Cin Cout H W k stride pad up [--bwd] [--explicit] [--reps N]

col == NULL (the implicit / pointwise kernels) unless --explicit."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lrs-pnp-dip_amd"))
import torch  # noqa: E402

from lrspnp import _lib  # noqa: E402

a = [int(v) for v in sys.argv[1:9]]
cin, cout, H, W, k, stride, pad, up = a
bwd = "--bwd" in sys.argv
explicit = "--explicit" in sys.argv
reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 50
L = _lib.device_lib()
P = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else None
Ho, Wo = ctypes.c_int(), ctypes.c_int()
L.lrs_conv2d_out_size(H, W, k, stride, pad, up, ctypes.byref(Ho), ctypes.byref(Wo))
x = torch.randn(cin, H, W, device="cuda")
w = torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5
b = torch.randn(cout, device="cuda")
y = torch.empty(cout, Ho.value, Wo.value, device="cuda")
gy = torch.randn_like(y)
gx, gw = torch.empty_like(x), torch.empty_like(w)
div = torch.ones(1, device="cuda")
ncol = L.lrs_conv2d_col_size(cin, H, W, k, stride, pad, up)
col = torch.empty(max(ncol, 1), device="cuda") if explicit else None
nws = L.lrs_conv2d_workspace(cin, H, W, cout, k, stride, pad, up, None)
ws = torch.empty(nws // 4 + 1, device="cuda")
s = torch.cuda.current_stream()


def run():
    if not bwd:
        rc = L.lrs_conv2d_fwd_f32(P(x), cin, H, W, P(w), P(b), cout, k, stride, pad, 1, up, P(col) if explicit and ncol else None,
                                  P(y), None, P(ws), nws, ctypes.c_void_p(s.cuda_stream))
    elif explicit:
        rc = L.lrs_conv2d_bwd_f32(P(gy), P(col) if ncol else P(x), P(w), P(div), cin, H, W, cout, k, stride, pad, 1, up,
                                  P(gx), P(gw), None, P(ws), nws, ctypes.c_void_p(s.cuda_stream))
    else:
        rc = L.lrs_conv2d_bwd_x_f32(P(gy), P(x), P(w), P(div), cin, H, W, cout, k, stride, pad, 1, up, P(gx), P(gw),
                                    None, P(ws), nws, ctypes.c_void_p(s.cuda_stream))
    assert rc == 0, rc


for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    run()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / reps
fl = 2.0 * cout * cin * k * k * Ho.value * Wo.value * (2 if bwd else 1)
print(f"conv {tuple(a)} {'bwd' if bwd else 'fwd'}{' explicit' if explicit else ''}: {ms * 1e3:.1f} us/call, "
      f"{fl / ms / 1e9:.1f} TFLOP/s")
