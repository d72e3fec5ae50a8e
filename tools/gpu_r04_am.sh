#!/bin/bash
# Round 4: k_sn_gram with its whole inner slab staged at once (one barrier; bit-identical) vs the
# previous build (tools/ab/lib_gram_v1.so): bit-for-bit outputs, 196^2 / 36^2 / 512^2 step times, DIP tests.
set -o pipefail
o=gpurun_out/r04am
mkdir -p $o
export TMPDIR=/tmp
V1=$PWD/tools/ab/lib_gram_v1.so
V2=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip.so
for cfg in "--net unet --hw 196" "--net unet --hw 36 --bands 128" "--net skip --hw 200 --bands 198" "--net skip --hw 256 --bands 64"; do
  tag=$(echo $cfg | tr -d ' -')
  LRSPNP_LIB=$V1 timeout -k 10 200 python tools/dip_steptime.py $cfg --rounds 1 --steps 10 --dump /tmp/a_$tag.npy > $o/d.txt 2>&1 || { tail $o/d.txt; exit 1; }
  LRSPNP_LIB=$V2 timeout -k 10 200 python tools/dip_steptime.py $cfg --rounds 1 --steps 10 --dump /tmp/b_$tag.npy > $o/d.txt 2>&1 || { tail $o/d.txt; exit 1; }
  python -c "import numpy as np; a=np.load('/tmp/a_$tag.npy'); b=np.load('/tmp/b_$tag.npy'); print('$cfg bitwise', np.array_equal(a.view(np.uint32), b.view(np.uint32)))"
done
for r in 1 2 3; do
  for L in v1 v2; do
    lib=$V1; [ $L = v2 ] && lib=$V2
    LRSPNP_LIB=$lib timeout -k 10 200 python tools/dip_steptime.py --rounds 5 > $o/st_${L}_$r.txt 2>&1 || { tail $o/st_${L}_$r.txt; exit 1; }
    echo "$L round $r unet 196: $(tail -1 $o/st_${L}_$r.txt)"
  done
done
for r in 1 2; do
  for L in v1 v2; do
    lib=$V1; [ $L = v2 ] && lib=$V2
    LRSPNP_LIB=$lib timeout -k 10 200 python tools/dip_steptime.py --net unet --hw 36 --bands 128 --rounds 3 > $o/n36_${L}_$r.txt 2>&1 || { tail $o/n36_${L}_$r.txt; exit 1; }
    echo "$L round $r unet 36: $(tail -1 $o/n36_${L}_$r.txt)"
  done
done
for r in 1; do
  for L in v1 v2; do
    lib=$V1; [ $L = v2 ] && lib=$V2
    LRSPNP_LIB=$lib timeout -k 10 200 python tools/dip_steptime.py --net skip --hw 512 --bands 224 --rounds 3 --steps 10 > $o/sk_${L}_$r.txt 2>&1 || { tail $o/sk_${L}_$r.txt; exit 1; }
    echo "$L round $r skip 512: $(tail -1 $o/sk_${L}_$r.txt)"
  done
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_dip.py tests/test_gpu_nn.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $o/pytest.log | head -20; tail -5 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
