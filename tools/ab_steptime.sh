#!/bin/bash
# A/B of the DIP step time between environment settings of the tuning build:
#   bash tools/ab_steptime.sh "LRS_DIP_DEFER_SN=0" "LRS_DIP_DEFER_SN=1"   (then the product build)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    env $v LRSPNP_LIB=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so timeout -k 10 120 python tools/dip_steptime.py --rounds 5 ${STEP_ARGS:-} > gpurun_out/ab.txt 2>&1 || { tail gpurun_out/ab.txt; exit 1; }
    echo "$v: $(tail -1 gpurun_out/ab.txt)"
  done
  timeout -k 10 120 python tools/dip_steptime.py --rounds 5 ${STEP_ARGS:-} > gpurun_out/ab.txt 2>&1 || { tail gpurun_out/ab.txt; exit 1; }
  echo "product: $(tail -1 gpurun_out/ab.txt)"
done
