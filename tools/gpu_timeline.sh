#!/bin/bash
# DIP step timeline on the box: rocprofv3 kernel trace of N training steps (no ISTA beside),
# summarised there (tools/step_timeline.py) -> gpurun_out/timeline_<net>_<H>.txt
set -o pipefail
export TMPDIR=/tmp
net=${1:-unet1lip}; C=${2:-198}; H=${3:-196}; steps=${4:-12}
d=gpurun_out/tl_$net_$H
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 tools/prof_dip_step.py $net $C $H $H $steps > gpurun_out/tl.log 2>&1 || { tail gpurun_out/tl.log; exit 1; }
f=$(find $d -name "*kernel_trace.csv" | head -1)
python tools/step_timeline.py $f 2 > gpurun_out/timeline_${net}_${H}.txt
rm -rf $d
tail -1 gpurun_out/timeline_${net}_${H}.txt
