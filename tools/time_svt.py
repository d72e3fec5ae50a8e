"""Time the SVT prox (lrs_svt_gram_f32 + lrs_svt_finish_f32) with the one-workgroup eigensolver and
with LRS_SVT_MULTI_WG, alone on the GPU (HIP events), on a P x B slab.

    python tools/time_svt.py [--P 5000] [--B 198] [--reps 10]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lrspnp import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--P", type=int, default=5000)
ap.add_argument("--B", type=int, default=198)
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
rng = np.random.default_rng(0)
X = torch.from_numpy((rng.random((a.P, 8)) @ rng.random((8, a.B)) * 0.3 +
                      0.05 * rng.standard_normal((a.P, a.B))).astype(np.float32)).cuda()
U = torch.empty_like(X)
ws = ops.svt_workspace(a.P, a.B, "cuda")
st = torch.cuda.current_stream()
res = {}
for mw in (False, True, False, True):
    ops.svt(X, None, 1.0, 1.0, ws, U=U, multi_wg=mw)
    torch.cuda.synchronize()
    ts = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        ops.svt(X, None, 1.0, 1.0, ws, U=U, multi_wg=mw)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    res.setdefault("multi_wg" if mw else "one_wg", []).append(float(np.median(ts)))
print(json.dumps({"P": a.P, "B": a.B, "ms_median": res, "path": ops.svt_state(ws, a.P, a.B)[4]}))
