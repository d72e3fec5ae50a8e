#!/bin/bash
# A/B on the full configs[2] outer iteration (tuning build): the 98^2 maps' register BN forward on
# 1024- (default) vs 256-thread workgroups (LRS_DIP_BNR_SMALL_WG), interleaved twice.
set -o pipefail
o=gpurun_out/bnr
mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for v in 0 1; do
    LRS_DIP_BNR_SMALL_WG=$v LRSPNP_LIB=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so timeout -k 10 240 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $o/b_${v}_$r.json 2> $o/b_${v}_$r.err || { tail $o/b_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('$o/b_${v}_$r.json')); print('small_wg $v run $r', d['value'], d['ms_per_step'], d.get('mpsnr', d.get('config', {}).get('mpsnr')))"
  done
done
