#!/bin/bash
# A/B of library builds tools/ab/lib_<v>.so on the DIP step (196^2 bench net, or STEP_ARGS), interleaved twice:
#   bash tools/ab_libs_step.sh base fold
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in "$@"; do
    LRSPNP_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 120 python tools/dip_steptime.py --rounds 5 ${STEP_ARGS:-} > gpurun_out/ab.txt 2>&1 || { tail gpurun_out/ab.txt; exit 1; }
    echo "$v: $(tail -1 gpurun_out/ab.txt)"
  done
done
