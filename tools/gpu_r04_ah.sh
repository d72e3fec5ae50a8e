#!/bin/bash
# Round 4: the sparse coding beside the DIP with 4-wave workgroups (LRS_ISTA_PAT_WAVES=4, tuning build:
# one wave per SIMD at 192 registers leaves 320, room for a DIP GEMM wave) with and without a
# one-per-CU grid (--ista-max-wg 256), vs the default 8-wave form; configs[2] bench, 3 rounds.
set -o pipefail
o=gpurun_out/r04ah
mkdir -p $o
export TMPDIR=/tmp
T=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
for r in 1 2 3; do
  for v in "8 0" "4 0" "4 256"; do
    set -- $v
    LRSPNP_LIB=$T LRS_ISTA_PAT_WAVES=$1 timeout -k 10 200 python bench.py --steps 8 --warmup 1 --no-cpu-baseline --ista-max-wg $2 > $o/b.json 2> $o/b.err || { tail $o/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$o/b.json').read().strip().splitlines()[-1]); print('round $r waves $1 max_wg $2', d['value'], d['ms_per_step'], d['roofline']['kernels'][0]['ms_per_launch'])"
  done
done
