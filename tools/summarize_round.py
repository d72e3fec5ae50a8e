"""Summarise tools/profile_r02.sh output into committed evidence (profiles/r02/).

    python tools/summarize_round.py gpurun_out/<run>/profile profiles/<round>  (tools/gpu.sh profile)

Per workload <wl> in {dip, pnp} (whatever was profiled):
  <wl>_kernel_stats.csv   rocprofv3 --stats of the bench command (copied)
  <wl>_bench.json         the bench line of the same round
  <wl>_summary.json       per-kernel mean duration (trace), HBM bytes (PMC), SQ counters
and traffic.json (read by bench.py for roofline.traffic):
  dip_hbm_bytes_per_outer_iter       sum over the DIP prox's kernels / outer iterations profiled
  dip_ista_hbm_bytes_per_launch      the sparse-coding kernel (k_ista_pat, or k_ista_rs), mean per launch
  pnp_ista_hbm_bytes_per_launch      k_ista_ln2, mean per launch

HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE for every kernel (MI355X_MICROARCH.md §HBM: on gfx950
FETCH_SIZE tallies 64 B per 128-B read request of a wide coalesced stream, so it reads 1/2 of
those bytes; WRITE_SIZE is exact for 16-B-per-lane stores).  The same x2 is applied to every
kernel, so for kernels whose reads are narrower than 16 B per lane the figure is an upper bound.
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
NOT_DIP = ("k_ista", "k_pat_gram", "k_admm_update", "k_alpha", "k_psnr", "at::native", "__amd_rocclr", "k_ssim")


def kname(r):
    return r["Kernel_Name"]


def short(n):
    return n.split("(")[0] if not n.startswith("k_im2col(") else "k_im2col[admm]"


def is_dip(n):
    if n.startswith("k_im2col("):          # the ADMM im2col (global namespace), not the DIP's lrs::k_im2col
        return False
    return not any(t in n for t in NOT_DIP)


def pmc(path, counter):
    vals = defaultdict(list)
    if not os.path.exists(path):
        return vals
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[kname(r)].append(float(r["Counter_Value"]))
    return vals


traffic = {}
for wl in ("dip", "pnp"):
    tr = os.path.join(src, f"{wl}_trace", "run_kernel_trace.csv")
    if not os.path.exists(tr):
        continue
    shutil.copy(os.path.join(src, f"{wl}_trace", "run_kernel_stats.csv"), os.path.join(dst, f"{wl}_kernel_stats.csv"))
    bj = os.path.join(src, f"{wl}_bench.json")
    lines = [l for l in open(bj) if l.startswith("{")]
    bench = json.loads(lines[-1])
    json.dump(bench, open(os.path.join(dst, f"{wl}_bench.json"), "w"), indent=1)
    outer = bench["warmup"] + bench["steps"]
    dur = defaultdict(list)
    for r in csv.DictReader(open(tr)):
        dur[kname(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    fetch = pmc(os.path.join(src, f"{wl}_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(src, f"{wl}_write", "run_counter_collection.csv"), "WRITE_SIZE")
    sq = defaultdict(lambda: defaultdict(list))
    sqp = os.path.join(src, f"{wl}_sq", "run_counter_collection.csv")
    if os.path.exists(sqp):
        for r in csv.DictReader(open(sqp)):
            sq[kname(r)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kern = {}
    dip_bytes = dip_ms = 0.0
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        f = sum(fetch.get(k, [])) * 1024.0
        w = sum(write.get(k, [])) * 1024.0
        e = {"calls": len(v), "mean_ms": statistics.mean(v), "total_ms": sum(v),
             "fetch_size_bytes_raw_total": f, "write_size_bytes_total": w, "hbm_bytes_total": 2 * f + w,
             "sq_mean": {c: statistics.mean(x) for c, x in sq.get(k, {}).items()}}
        kern[short(k)] = e
        if wl == "dip" and is_dip(k):
            dip_bytes += 2 * f + w
            dip_ms += sum(v)
    ista = [k for k in dur if "k_ista_pat<" in k or "k_ista_rs<" in k or "k_ista_ln2<" in k]
    summ = {"workload": wl, "outer_iterations_profiled": outer, "kernels": kern}
    if ista:
        k = ista[0]
        n = len(fetch.get(k, [])) or 1
        per = (2 * sum(fetch.get(k, [])) * 1024.0 + sum(write.get(k, [])) * 1024.0) / n
        summ["ista_kernel"] = short(k)
        summ["ista_hbm_bytes_per_launch"] = per
        summ["ista_mean_ms_trace"] = statistics.mean(dur[k])
        traffic[f"{wl}_ista_hbm_bytes_per_launch"] = per
    if wl == "dip":
        summ["dip_hbm_bytes_per_outer_iter"] = dip_bytes / outer
        summ["dip_kernel_ms_per_outer_iter"] = dip_ms / outer
        summ["dip_launches_per_outer_iter"] = sum(len(v) for k, v in dur.items() if is_dip(k)) / outer
        traffic["dip_hbm_bytes_per_outer_iter"] = dip_bytes / outer
    json.dump(summ, open(os.path.join(dst, f"{wl}_summary.json"), "w"), indent=1)
    print(wl, json.dumps({k: v for k, v in summ.items() if k != "kernels"}, indent=1))

old = {}
tp = os.path.join(dst, "traffic.json")
if os.path.exists(tp):
    old = json.load(open(tp))
old.update(traffic)
old["correction"] = "2 x FETCH_SIZE + WRITE_SIZE per kernel (gfx950: FETCH_SIZE counts 64 B per 128-B read request)"
old["source"] = f"{dst}/<workload>_summary.json (rocprofv3 --pmc passes of the bench command, tools/gpu.sh profile)"
json.dump(old, open(tp, "w"), indent=1)
