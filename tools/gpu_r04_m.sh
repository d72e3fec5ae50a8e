#!/bin/bash
# Round 4: k_fold_pad over 4 channels per thread vs the one-channel fold (tools/ab/lib_fold_v1.so):
# bit-for-bit DIP outputs, interleaved step times; the side-stream priority test; DIP conv/net tests.
set -o pipefail
o=gpurun_out/r04m
mkdir -p $o
export TMPDIR=/tmp
V1=$PWD/tools/ab/lib_fold_v1.so
V2=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip.so
for hw in 196 132; do
  LRSPNP_LIB=$V1 timeout -k 10 120 python tools/dip_steptime.py --hw $hw --rounds 2 --steps 30 --dump /tmp/v1_$hw.npy > $o/d1.txt 2>&1 || { tail $o/d1.txt; exit 1; }
  LRSPNP_LIB=$V2 timeout -k 10 120 python tools/dip_steptime.py --hw $hw --rounds 2 --steps 30 --dump /tmp/v2_$hw.npy > $o/d2.txt 2>&1 || { tail $o/d2.txt; exit 1; }
  python -c "import numpy as np; a=np.load('/tmp/v1_$hw.npy'); b=np.load('/tmp/v2_$hw.npy'); print('hw $hw bitwise', np.array_equal(a.view(np.uint32), b.view(np.uint32)))"
done
for r in 1 2 3; do
  for L in v1 v2; do
    lib=$V1; [ $L = v2 ] && lib=$V2
    LRSPNP_LIB=$lib timeout -k 10 120 python tools/dip_steptime.py --rounds 5 > $o/st_${L}_$r.txt 2>&1 || { tail $o/st_${L}_$r.txt; exit 1; }
    echo "$L round $r: $(tail -1 $o/st_${L}_$r.txt)"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_dip.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "priority or conv or unet or dgrad or skip" > $o/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $o/pytest.log | head -20; tail -5 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
