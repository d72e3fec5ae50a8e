#!/bin/bash
# Round 4: kernel trace of the configs[3] (dip-pro) bench at the current build.
set -o pipefail
o=gpurun_out/r04t
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/trpro -o run --output-format csv -- python3 bench.py --workload dip-pro --steps 1 --warmup 1 --no-cpu-baseline > $o/dip_pro_trace.log 2>&1 || { tail $o/dip_pro_trace.log; exit 1; }
cp $(find /tmp/trpro -name "*kernel_stats.csv" | head -1) $o/dip_pro_kernel_stats.csv
python3 tools/step_timeline.py $(find /tmp/trpro -name "*kernel_trace.csv" | head -1) 3 > $o/timeline_512.txt 2>&1 || true
tail -2 $o/timeline_512.txt
