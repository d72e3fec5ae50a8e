#!/bin/bash
# Round 4: the sparse coding beside the DIP training (default) vs before it (the DIP's stream waits),
# configs[2], 2 alternating rounds; then the kernel trace of the "before" order.
set -o pipefail
o=gpurun_out/r04g
mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for m in beside before; do
    timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ista-dip-order $m > $o/order_${m}_$r.json 2> $o/order_${m}_$r.err || { tail $o/order_${m}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$o/order_${m}_$r.json').read().strip().splitlines()[-1]); print('$m run $r', round(d['value'],3), d['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ordb -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --ista-dip-order before > $o/trace_before.log 2>&1 || { tail $o/trace_before.log; exit 1; }
f=$(find /tmp/ordb -name "*kernel_trace.csv" | head -1); cp $f $o/trace_before.csv
f=$(find /tmp/ordb -name "*kernel_stats.csv" | head -1); cp $f $o/stats_before.csv
grep k_ista_rs $o/stats_before.csv | cut -d, -f1-4
