"""Summarise a tools/profile_round.sh run into profiles/<tag>/ (committed evidence).

Writes kernel_stats.csv (rocprofv3 --stats), summary.json (per-kernel mean duration from the
trace, per-launch HBM bytes of the ISTA kernel from the PMC passes) and profiles/ista_pmc_traffic.json
(read by bench.py for roofline.traffic).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 64 B per TCC_EA0_RDREQ while wide
streaming reads issue 128-B requests, so it reads 1/2 of the fetched bytes for such streams;
WRITE_SIZE is exact for 16-B-per-lane stores.  hbm_read = 2 * FETCH_SIZE KiB * 1024 (upper bound
for mixed-width traffic: the ISTA kernel's loads are 16-B-per-lane).
"""
import csv
import json
import os
import shutil
import statistics
import sys
from collections import defaultdict

src = sys.argv[1]              # gpurun_out/profile_<tag>
tag = sys.argv[2]
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
dst = os.path.join(repo, "profiles", tag)
os.makedirs(dst, exist_ok=True)
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
shutil.copy(os.path.join(src, "bench.json"), os.path.join(dst, "bench.json"))

dur = defaultdict(list)
for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
    dur[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)


def pmc(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    return vals


fetch = pmc(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
write = pmc(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
sq = defaultdict(dict)
for r in csv.DictReader(open(os.path.join(src, "sq", "run_counter_collection.csv"))):
    sq[r["Kernel_Name"].split("(")[0]].setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))

ista = [k for k in dur if "k_ista" in k][0]
fk = statistics.mean(fetch[ista]) * 1024.0
wk = statistics.mean(write[ista]) * 1024.0
summary = {
    "tag": tag,
    "kernel_mean_ms": {k: statistics.mean(v) for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1]))},
    "kernel_calls": {k: len(v) for k, v in dur.items()},
    "ista_kernel": ista,
    "ista_fetch_size_bytes_raw": fk,
    "ista_write_size_bytes": wk,
    "ista_hbm_bytes_per_launch_corrected": 2 * fk + wk,
    "ista_sq_counters_mean": {k: statistics.mean(v) for k, v in sq[ista].items()},
}
json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1)
json.dump({"kernel": ista, "hbm_bytes_per_launch": 2 * fk + wk, "fetch_size_raw_bytes": fk, "write_size_bytes": wk,
           "correction": "2 x FETCH_SIZE (gfx950 counts 64 B per 128-B read request) + WRITE_SIZE",
           "source": f"profiles/{tag}/summary.json"},
          open(os.path.join(repo, "profiles", "ista_pmc_traffic.json"), "w"), indent=1)
print(json.dumps(summary, indent=1))
