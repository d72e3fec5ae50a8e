#!/bin/bash
# Where the DIP step's kernels spend their wave cycles (196^2 bench net, 10 eager steps, no ISTA):
# one rocprofv3 SQ pass (8 SQ counters, no tracing), summarised per kernel on the box.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf /tmp/pmcw
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES -d /tmp/pmcw -o run --output-format csv -- python3 tools/prof_dip_step.py unet1lip ${1:-198} ${2:-196} ${2:-196} 10 > gpurun_out/pmcw.log 2>&1 || { tail gpurun_out/pmcw.log; exit 1; }
f=$(find /tmp/pmcw -name "*counter_collection.csv" | head -1)
python3 - "$f" > gpurun_out/pmc_step_waits_${2:-196}.txt <<'PY'
import csv, sys
from collections import defaultdict
per = defaultdict(lambda: defaultdict(float))
names = {}
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Dispatch_Id"]
    per[k][r["Counter_Name"]] += float(r["Counter_Value"])
    names[k] = r["Kernel_Name"].replace("lrs::", "").split("(")[0][:60]
agg = defaultdict(lambda: defaultdict(float))
cnt = defaultdict(int)
for k, cs in per.items():
    n = names[k]
    cnt[n] += 1
    for c, v in cs.items():
        agg[n][c] += v
rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))
print(f"{'kernel':60s} {'n':>4s} {'wave_cyc':>10s} {'wait%':>6s} {'instst%':>7s} {'active%':>7s} {'valu':>9s} {'mfma':>9s} {'lds':>8s}")
for n, c in rows:
    m = cnt[n]; w = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{n:60s} {m:4d} {w / m:10.0f} {100 * c.get('SQ_WAIT_ANY', 0) / w:6.1f} {100 * c.get('SQ_WAIT_INST_ANY', 0) / w:7.1f} "
          f"{100 * c.get('SQ_ACTIVE_INST_ANY', 0) / w:7.1f} {c.get('SQ_INSTS_VALU', 0) / m:9.0f} {c.get('SQ_INSTS_MFMA', 0) / m:9.0f} {c.get('SQ_INSTS_LDS', 0) / m:8.0f}")
PY
cat gpurun_out/pmc_step_waits_${2:-196}.txt | head -40
