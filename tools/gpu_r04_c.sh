#!/bin/bash
# Round 4: deferred BN stage 1 (producer finish + statistics in the conv GEMM, y by k_bn_coef_apply):
# the DIP tests, then the step time A/B (tuning build, LRS_DIP_DEFER 0/1/2) at 196^2 and 36^2.
set -o pipefail
o=gpurun_out/r04c
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dip.py tests/test_gpu_nn.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $o/pytest_dip.log 2>&1; rc=$?
tail -25 $o/pytest_dip.log
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for v in 0 1 2; do
    LRS_DIP_DEFER=$v LRSPNP_LIB=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so timeout -k 10 120 python tools/dip_steptime.py --rounds 5 > $o/st196_$v.txt 2>&1 || { tail $o/st196_$v.txt; exit 1; }
    echo "196 defer=$v: $(tail -1 $o/st196_$v.txt)"
    LRS_DIP_DEFER=$v LRSPNP_LIB=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so timeout -k 10 120 python tools/dip_steptime.py --hw 36 --bands 128 --rounds 5 > $o/st36_$v.txt 2>&1 || { tail $o/st36_$v.txt; exit 1; }
    echo "36 defer=$v: $(tail -1 $o/st36_$v.txt)"
  done
done
for v in 512 256 128; do
  LRS_DIP_WGRAD_SPLIT_WG=$v LRSPNP_LIB=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so timeout -k 10 120 python tools/dip_steptime.py --rounds 5 > $o/stw_$v.txt 2>&1 || { tail $o/stw_$v.txt; exit 1; }
  echo "196 wgrad split $v: $(tail -1 $o/stw_$v.txt)"
done
