#!/bin/bash
# Kernel trace + stats of the default bench command at HEAD (no CPU baseline).
set -o pipefail
o=gpurun_out/trace_head
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/t -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > $o/bench.json 2> $o/trace.log || { tail $o/trace.log; exit 1; }
cp "$(find $o/t -name '*kernel_stats.csv' | head -n 1)" $o/dip_kernel_stats_head.csv
cat $o/bench.json
