#!/bin/bash
# Round 4: k_ista_pat with the XCD-aware tile order and 16-byte prox window loads vs the first
# version (tools/ab/lib_pat_v1.so): bit-for-bit outputs, kernel time (interleaved), bench.
set -o pipefail
o=gpurun_out/r04j
mkdir -p $o
export TMPDIR=/tmp
V1=$PWD/tools/ab/lib_pat_v1.so
for c in cfg2 cfg3; do
  LRSPNP_LIB=$V1 timeout -k 10 200 python tools/pat_dump.py /tmp/v1_$c.npz $c > $o/dump.log 2>&1 || { tail $o/dump.log; exit 1; }
  timeout -k 10 200 python tools/pat_dump.py /tmp/v2_$c.npz $c >> $o/dump.log 2>&1 || { tail $o/dump.log; exit 1; }
  python -c "
import numpy as np
a=np.load('/tmp/v1_$c.npz'); b=np.load('/tmp/v2_$c.npz')
print('$c bitwise phi', np.array_equal(a['phi'].view(np.uint32), b['phi'].view(np.uint32)), 'coefs', np.array_equal(a['coefs'].view(np.uint32), b['coefs'].view(np.uint32)))"
done
for r in 1 2; do
  for L in v1 v2; do
    lib=$V1; [ $L = v2 ] && lib=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip.so
    LRSPNP_LIB=$lib timeout -k 10 200 python tools/time_ista.py --only cfg2 --reps 5 > $o/t_$L_$r.json 2> $o/t.err || { tail $o/t.err; exit 1; }
    echo "$L run $r cfg2: $(python -c "import json; d=json.loads(open('$o/t_$L_$r.json').read().strip().splitlines()[-1]); print(round(d['ms'],3), 'ms')")"
  done
done
LRS_ISTA_PAT_WAVES=8 LRSPNP_LIB=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so timeout -k 10 200 python tools/time_ista.py --only cfg2 --variant soft --reps 5 > $o/t_soft.json 2> $o/t.err || { tail $o/t.err; exit 1; }
echo "v2 soft prox: $(python -c "import json; d=json.loads(open('$o/t_soft.json').read().strip().splitlines()[-1]); print(round(d['ms'],3), 'ms')")"
timeout -k 10 300 python tools/time_ista.py --only cfg3 --reps 3 > $o/t3.json 2> $o/t.err || { tail $o/t.err; exit 1; }
echo "v2 cfg3: $(python -c "import json; d=json.loads(open('$o/t3.json').read().strip().splitlines()[-1]); print(round(d['ms'],3), 'ms')")"
timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $o/b.json 2> $o/b.err || { tail $o/b.err; exit 1; }
python -c "import json; d=json.loads(open('$o/b.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels'][0]; print('bench', round(d['value'],3), round(d['ms_per_step'],2), 'ista ms', round(k['ms_per_launch'],3))"
