#!/bin/bash
# Round-4 profile at HEAD (tools/profile_r02.sh: kernel trace + separate FETCH_SIZE / WRITE_SIZE / SQ
# passes of the default and pnp bench commands, summarised on the box into gpurun_out/r04sum), then a
# kernel trace of the configs[3] (dip-pro) bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04sum
SUMDIR=gpurun_out/r04sum bash tools/profile_r02.sh || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/trpro -o run --output-format csv -- python3 bench.py --workload dip-pro --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r04sum/dip_pro_trace.log 2>&1 || { tail gpurun_out/r04sum/dip_pro_trace.log; exit 1; }
cp $(find /tmp/trpro -name "*kernel_stats.csv" | head -1) gpurun_out/r04sum/dip_pro_kernel_stats.csv
head -25 gpurun_out/r04sum/dip_pro_kernel_stats.csv | cut -d, -f1-4 | cut -c1-150
