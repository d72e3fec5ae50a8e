"""Time the fused ISTA kernel (lrs_ista_f32) on the benchmark workloads (HIP events on its stream).

    python tools/time_ista.py [--reps 5]

Workloads: configs[2] sparse coding (196x196x198 cube, 36x36 blocks, Nit 100, fro4: 6,408 blocks),
the native 36x36x128 image (144 blocks), configs[3] (512x512x224, 50,974 blocks), and the bb = 8
headline (200x200x198, 125,000 blocks, Nit 80, spec2).  Prints one JSON line per workload.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "lrs-pnp-dip_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from lrspnp import LrsPnP, LrsPnPConfig, _lib  # noqa: E402
from lrspnp.data import load_fixture, mask_matrix, synthetic_cube, synthetic_dictionary, unfold  # noqa: E402


def run(name, H, W, B, bb, nit, variant, reps, K=256, patterns="auto"):
    base = load_fixture("data_img5.npz")["lrs_mask"]
    obs, clean, mask = synthetic_cube(H, W, B, seed=0, base_mask=base)
    Y, M = unfold(obs), mask_matrix(mask, B)
    D = synthetic_dictionary(bb * bb, K, 0)
    s = LrsPnP(Y, M, D, LrsPnPConfig(bb=bb, sliding=bb, Nit=nit, variant=variant, ista_patterns=patterns))
    st = torch.cuda.current_stream()
    s.sparse_coding(stream=st)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        s.sparse_coding(stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    n = bb * bb
    pat = s.pat_plan is not None
    flops = (s.nb * (4 * n * K + nit * 2 * K * K) if pat else nit * s.nb * 4 * n * K + s.nb * 2 * n * K)
    ms = float(np.median(ts))
    print(json.dumps({"workload": name, "blocks": s.nb, "path": "pattern-gram" if pat else "row-split",
                      "npat": s.npat, "ms": ms, "ms_all": ts, "gflop": flops / 1e9,
                      "tflops": flops / ms / 1e9, "frac_f32_peak": flops / ms / 1e9 / 157.3}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--patterns", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--variant", default=None, help="override the ISTA variant (e.g. soft: prox ablation)")
    a = ap.parse_args()
    jobs = [("cfg2_196x196x198_bb36_fro4", 196, 196, 198, 36, 100, "fro4"),
            ("native_36x36x128_bb36_fro4", 36, 36, 128, 36, 100, "fro4"),
            ("cfg1_200x200x198_bb8_spec2", 200, 200, 198, 8, 80, "spec2"),
            ("cfg3_512x512x224_bb36_fro4", 512, 512, 224, 36, 100, "fro4")]
    for j in jobs:
        if a.only and a.only not in j[0]:
            continue
        j = list(j)
        if a.variant:
            j[6] = a.variant
        run(*j, reps=a.reps, patterns=a.patterns)


if __name__ == "__main__":
    main()
