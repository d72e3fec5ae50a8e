#!/bin/bash
# configs[1] (LRS-PnP, SVT, bb 8) A/B on one box: the round-1 end tree (ab_r01/, built from commit
# 1c05b02 by tools/build_ab_r01.sh) against HEAD, interleaved 3 times; k_ista_ln2 from a kernel trace of each.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r04d/ab_pnp
mkdir -p $o
for rnd in 1 2 3; do
  (cd ab_r01 && timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline) > $o/r01_$rnd.json 2> $o/r01.err || { tail $o/r01.err; exit 1; }
  timeout -k 10 200 python bench.py --workload pnp --steps 20 --warmup 3 --no-cpu-baseline > $o/head_$rnd.json 2> $o/head.err || { tail $o/head.err; exit 1; }
  python - <<PY
import json
for t in ("r01", "head"):
    d = json.loads(open(f"$o/{t}_$rnd.json").read().strip().splitlines()[-1])
    print("$rnd", t, round(d["value"], 2), "outer it/s")
PY
done
for t in r01 head; do
  if [ $t = r01 ]; then cmd="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"; dir=ab_r01; else cmd="python3 bench.py --workload pnp --steps 10 --warmup 2 --no-cpu-baseline"; dir=.; fi
  (cd $dir && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/abtr_$t -o run --output-format csv -- $cmd > /tmp/abtr_$t.log 2>&1) || { tail /tmp/abtr_$t.log; exit 1; }
  f=$(find /tmp/abtr_$t -name "*kernel_stats.csv" | head -1)
  cp $f $o/${t}_kernel_stats.csv
  grep -i "ista_ln2\|k_ista<\|k_ista_" $f | cut -c1-200
done
