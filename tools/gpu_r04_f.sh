#!/bin/bash
# Round 4: the persistent, pipelined k_pw (tuning build, LRS_DIP_PW_PIPE = workgroups per CU of the
# persistent grid; 0 = the one-tile grid): the 1x1 convs alone, then the 196^2 step; correctness via the
# 1x1 conv / whole-net GPU tests on the tuning build.
set -o pipefail
o=gpurun_out/r04f
mkdir -p $o
export TMPDIR=/tmp
TL=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
LRS_DIP_PW_PIPE=1 LRSPNP_LIB=$TL timeout -k 10 300 python -u -m pytest tests/test_gpu_dip.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread -k "pw or unet or conv" > $o/pytest_pipe.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $o/pytest_pipe.log | head -20; tail -3 $o/pytest_pipe.log; exit 1; }
tail -1 $o/pytest_pipe.log
for v in 0 1 2; do
  for cfg in "128 128 196 196 1 1 0 0" "198 128 196 196 1 1 0 0"; do
    for d in "" "--bwd"; do
      LRS_DIP_PW_PIPE=$v LRSPNP_LIB=$TL timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/pw$v$d -o run --output-format csv -- python3 tools/micro_conv.py $cfg $d --reps 30 > $o/pw.log 2>&1 || { tail $o/pw.log; exit 1; }
      f=$(find /tmp/pw$v$d -name "*kernel_stats.csv" | head -1); echo "pipe=$v $cfg $d: $(grep k_pw $f | cut -d, -f1,4 | tr '\n' ' ')"
      rm -rf /tmp/pw$v$d
    done
  done
done
for r in 1 2; do
  for v in 0 1 2; do
    LRS_DIP_PW_PIPE=$v LRSPNP_LIB=$TL timeout -k 10 120 python tools/dip_steptime.py --rounds 5 > $o/st_$v.txt 2>&1 || { tail $o/st_$v.txt; exit 1; }
    echo "196 pipe=$v: $(tail -1 $o/st_$v.txt)"
  done
done
