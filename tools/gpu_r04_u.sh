#!/bin/bash
# Round 4: the row-quad single-partial fold vs k_fold_pad (tools/ab/lib_fold1_v1.so):
# bit-for-bit skip-net outputs (512^2, 256^2, the literal 200^2 with its odd-size crops, 100^2),
# configs[3]-size step times, skip-net tests, dip-pro bench.
set -o pipefail
o=gpurun_out/r04u
mkdir -p $o
export TMPDIR=/tmp
V1=$PWD/tools/ab/lib_fold1_v1.so
V2=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip.so
for cfg in "--net skip --hw 512 --bands 224" "--net skip --hw 256 --bands 64" "--net skip --hw 200 --bands 198" "--net skip --hw 100 --bands 31" "--net unet --hw 196"; do
  tag=$(echo $cfg | tr -d ' -')
  LRSPNP_LIB=$V1 timeout -k 10 200 python tools/dip_steptime.py $cfg --rounds 1 --steps 10 --dump /tmp/a_$tag.npy > $o/d.txt 2>&1 || { tail $o/d.txt; exit 1; }
  LRSPNP_LIB=$V2 timeout -k 10 200 python tools/dip_steptime.py $cfg --rounds 1 --steps 10 --dump /tmp/b_$tag.npy > $o/d.txt 2>&1 || { tail $o/d.txt; exit 1; }
  python -c "import numpy as np; a=np.load('/tmp/a_$tag.npy'); b=np.load('/tmp/b_$tag.npy'); print('$cfg bitwise', np.array_equal(a.view(np.uint32), b.view(np.uint32)))"
done
for r in 1 2; do
  for L in v1 v2; do
    lib=$V1; [ $L = v2 ] && lib=$V2
    LRSPNP_LIB=$lib timeout -k 10 200 python tools/dip_steptime.py --net skip --hw 512 --bands 224 --rounds 3 --steps 10 > $o/st_${L}_$r.txt 2>&1 || { tail $o/st_${L}_$r.txt; exit 1; }
    echo "$L round $r skip 512: $(tail -1 $o/st_${L}_$r.txt)"
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_dip.py tests/test_gpu_nn.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "skip or bn or batch" > $o/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $o/pytest.log | head -20; tail -5 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 400 python bench.py --workload dip-pro --steps 3 --warmup 1 --no-cpu-baseline > $o/dip_pro.json 2> $o/dip_pro.err || { tail $o/dip_pro.err; exit 1; }
python -c "import json; d=json.loads(open('$o/dip_pro.json').read().strip().splitlines()[-1]); print('configs[3]', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['kernels'][0]['ms_per_launch'])"
