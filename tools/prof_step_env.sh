#!/bin/bash
# Kernel timeline of one 196^2 U-Net training step per environment setting:
#   prof_step_env.sh "VAR=a" "VAR=b" ...   -> gpurun_out/steptl_<i>.txt
set -o pipefail
export TMPDIR=/tmp
i=0
for v in "$@"; do
  rm -rf /tmp/pse
  env $v timeout -k 10 120 rocprofv3 --kernel-trace -d /tmp/pse -o run --output-format csv -- python3 tools/prof_dip_step.py unet1lip 198 196 196 30 > /tmp/pse.log 2>&1 || { tail /tmp/pse.log; exit 1; }
  f=$(find /tmp/pse -name "*kernel_trace.csv" | head -1)
  { echo "== $v"; python3 tools/step_timeline.py $f 3; } > gpurun_out/steptl_$i.txt || exit 1
  tail -1 gpurun_out/steptl_$i.txt
  i=$((i+1))
done
