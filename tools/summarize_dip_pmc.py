"""Summarise tools/dip_conv_pmc.sh into profiles/<tag>/dip_conv_pmc.json.

Per implicit-GEMM conv kernel of one 512x512 128->128 3x3 layer: mean duration (kernel trace),
algorithmic fp32 GEMM FLOPs and TFLOP/s, matrix-core busy fraction (SQ_VALU_MFMA_BUSY_CYCLES
over duration x 1024 SIMDs x 2.4 GHz), VALU and MFMA instruction counts, HBM bytes (FETCH_SIZE
KiB x 1024, also x2 as the gfx950 upper bound for wide streaming reads; WRITE_SIZE KiB x 1024)
against the algorithmic bytes."""
import csv
import json
import os
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C, H, W, K = 128, 512, 512, 3
P, Kc, Qp = H * W, C * K * K, (H + 2) * (W + 2)
ALG = {   # flops, algorithmic HBM bytes (operands read once, output written once)
    "LdFwdTM": (2 * C * Kc * P, 4 * (C * P + C * P)),
    "LdWgradTM": (2 * C * Kc * P, 4 * (C * P + C * P)),
    "LdDgradTM": (2 * C * Qp * C * K * K, 4 * (C * P + C * Qp)),
}


def key(name):
    for k in ALG:
        if k in name:
            return k
    return None


dur = defaultdict(list)
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
    k = key(r["Kernel_Name"])
    if k:
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
ctr = defaultdict(lambda: defaultdict(list))
for sub in ("sq", "fetch", "write"):
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(os.path.join(src, sub, "run_counter_collection.csv"))):
        k = key(r["Kernel_Name"])
        if k:
            per[(k, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for (k, _), cs in per.items():
        for c, v in cs.items():
            ctr[k][c].append(v)
out = {"layer": f"{C}->{C} ch, {K}x{K}, reflection pad 1, {H}x{W} (tools/diag_conv_one.py)", "kernels": {}}
for k, (fl, ab) in ALG.items():
    t = sorted(dur[k])[len(dur[k]) // 2]
    m = {c: sum(v) / len(v) for c, v in ctr[k].items()}
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    out["kernels"][k] = {
        "median_us": t * 1e6,
        "flops": fl,
        "tflops": fl / t / 1e12,
        "frac_of_f32_mfma_peak": fl / t / 157.3e12,
        "mfma_busy_frac_at_2p4GHz": busy / (t * 2.4e9 * 1024),
        "insts_valu_per_mfma": m.get("SQ_INSTS_VALU", 0.0) / max(m.get("SQ_INSTS_MFMA", 1.0), 1.0),
        "hbm_read_bytes": m.get("FETCH_SIZE", 0.0) * 1024,
        "hbm_read_bytes_x2_bound": 2 * m.get("FETCH_SIZE", 0.0) * 1024,
        "hbm_write_bytes": m.get("WRITE_SIZE", 0.0) * 1024,
        "algorithmic_bytes": ab,
        "achieved_alg_GBps": ab / t / 1e9,
    }
dst = os.path.join(repo, "profiles", tag)
os.makedirs(dst, exist_ok=True)
json.dump(out, open(os.path.join(dst, "dip_conv_pmc.json"), "w"), indent=1)
print(json.dumps(out, indent=1))
