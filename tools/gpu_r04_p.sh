#!/bin/bash
# Round 4: k_ista_pat bounded to 128 registers (two 512-thread workgroups per CU; LRS_ISTA_PAT_WPE=4,
# tuning build) vs the 183-register form: bit-for-bit sparse coding, kernel time, configs[2] bench.
set -o pipefail
o=gpurun_out/r04p
mkdir -p $o
export TMPDIR=/tmp
TL=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
LRSPNP_LIB=$TL timeout -k 10 200 python tools/pat_dump.py /tmp/w2.npz cfg2 > $o/dump.log 2>&1 || { tail $o/dump.log; exit 1; }
LRS_ISTA_PAT_WPE=4 LRSPNP_LIB=$TL timeout -k 10 200 python tools/pat_dump.py /tmp/w4.npz cfg2 >> $o/dump.log 2>&1 || { tail $o/dump.log; exit 1; }
python -c "
import numpy as np
a=np.load('/tmp/w2.npz'); b=np.load('/tmp/w4.npz')
print('bitwise phi', np.array_equal(a['phi'].view(np.uint32), b['phi'].view(np.uint32)), 'coefs', np.array_equal(a['coefs'].view(np.uint32), b['coefs'].view(np.uint32)))"
for r in 1 2; do
  for w in 0 4; do
    LRS_ISTA_PAT_WPE=$w LRSPNP_LIB=$TL timeout -k 10 200 python tools/time_ista.py --only cfg2 --reps 5 > $o/t_${w}_$r.json 2> $o/t.err || { tail $o/t.err; exit 1; }
    LRS_ISTA_PAT_WPE=$w LRSPNP_LIB=$TL timeout -k 10 300 python tools/time_ista.py --only cfg3 --reps 3 > $o/t3_${w}_$r.json 2> $o/t.err || { tail $o/t.err; exit 1; }
    echo "wpe $w round $r: cfg2 $(python -c "import json; print(round(json.loads(open('$o/t_${w}_$r.json').read().strip().splitlines()[-1])['ms'],3))") ms, cfg3 $(python -c "import json; print(round(json.loads(open('$o/t3_${w}_$r.json').read().strip().splitlines()[-1])['ms'],3))") ms"
  done
done
for r in 1 2; do
  for w in 0 4; do
    LRS_ISTA_PAT_WPE=$w LRSPNP_LIB=$TL timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $o/b_${w}_$r.json 2> $o/b.err || { tail $o/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$o/b_${w}_$r.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels'][0]; print('bench wpe $w run $r', round(d['value'],3), round(d['ms_per_step'],2), 'ista ms', round(k['ms_per_launch'],3))"
  done
done
