"""Time the DIP conv layers (lrs_conv2d_fwd_f32 + lrs_conv2d_bwd_f32) at both GEMM precisions.

GPU diagnostic: python tools/diag_gemm.py  (prints one line per layer shape)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lrs-pnp-dip_amd"))
from lrspnp import _lib  # noqa: E402

L = _lib.device_lib()
P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

SHAPES = [  # cin, cout, H, W, k, stride, pad, up  (196x196 U-Net, 512x512 skip net)
    (198, 128, 196, 196, 3, 2, 1, 0),
    (128, 128, 98, 98, 3, 1, 1, 0),
    (128, 128, 98, 98, 2, 1, 0, 1),
    (128, 198, 196, 196, 1, 1, 0, 0),
    (224, 128, 512, 512, 3, 2, 1, 0),
    (128, 128, 256, 256, 3, 1, 1, 0),
    (132, 128, 512, 512, 3, 1, 1, 0),
    (128, 128, 512, 512, 1, 1, 0, 0),
    (256, 128, 512, 512, 1, 1, 0, 0),
    (128, 4, 512, 512, 1, 1, 0, 0),
]


def run(shape, reps=10, implicit=False):
    cin, cout, H, W, k, s, p, up = shape
    torch.manual_seed(0)
    x = torch.randn(cin, H, W, device="cuda")
    w = torch.randn(cout, cin, k, k, device="cuda") * 0.05
    b = torch.zeros(cout, device="cuda")
    Ho, Wo = ctypes.c_int(), ctypes.c_int()
    L.lrs_conv2d_out_size(H, W, k, s, p, up, ctypes.byref(Ho), ctypes.byref(Wo))
    ncol = L.lrs_conv2d_col_size(cin, H, W, k, s, p, up)
    col = torch.empty(max(ncol, 1), device="cuda")
    nws = L.lrs_conv2d_workspace(cin, H, W, cout, k, s, p, up)
    ws = torch.empty(nws // 4 + 1, device="cuda")
    y = torch.empty(cout, Ho.value, Wo.value, device="cuda")
    gy = torch.randn_like(y)
    gx, gw = torch.empty_like(x), torch.empty_like(w)
    div = torch.ones(1, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cp = P(col) if ncol and not implicit else None

    def fwd():
        assert L.lrs_conv2d_fwd_f32(P(x), cin, H, W, P(w), P(b), cout, k, s, p, 1, up, cp, P(y), P(ws), nws, st) == 0

    def bwd():
        fn = L.lrs_conv2d_bwd_x_f32 if implicit else L.lrs_conv2d_bwd_f32
        assert fn(P(gy), cp if cp is not None else P(x), P(w), P(div), cin, H, W, cout, k, s, p, 1, up,
                  P(gx), P(gw), P(ws), nws, st) == 0
    out = []
    for f in (fwd, bwd):
        f(); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            f()
        e1.record(); torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps * 1e3)
    fl = 2 * cout * cin * k * k * Ho.value * Wo.value
    return out, fl, (y.clone(), gx.clone(), gw.clone())


for sh in SHAPES[int(os.environ.get('DIAG_FIRST', 0)):]:
    res = {}
    for prec, name in ((0, "f32"), (1, "b3")):
        L.lrs_dip_set_precision(prec)
        res[name] = run(sh)
    res["imp"] = run(sh, implicit=True)
    (tf, tb), fl, o32 = res["f32"]
    (bf, bb), _, ob3 = res["b3"]
    err = [float((a - c).norm() / c.norm()) for a, c in zip(ob3, o32)]
    print(f"{sh}: fwd f32 {tf:8.1f} us b3 {bf:8.1f} us ({fl / bf / 1e6:6.1f} TF/s) | bwd f32 {tb:8.1f} b3 {bb:8.1f} us "
          f"({2 * fl / bb / 1e6:6.1f} TF/s) | rel diff y/gx/gw {err[0]:.1e} {err[1]:.1e} {err[2]:.1e}", flush=True)
    (tf, tb), _, oim = res["imp"]
    err = [float((a - c).norm() / c.norm()) for a, c in zip(oim, o32)]
    print(f"    implicit: fwd {tf:8.1f} us ({fl / tf / 1e6:6.1f} TF/s) bwd {tb:8.1f} us ({2 * fl / tb / 1e6:6.1f} TF/s)"
          f" | rel diff {err[0]:.1e} {err[1]:.1e} {err[2]:.1e}", flush=True)
