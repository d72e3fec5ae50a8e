#!/bin/bash
# Round 4, first box: GPU suite at HEAD, then two A/Bs interleaved twice:
#  - configs[1] (`--workload pnp`): k_ista_ln2's quotient variant DIV=1 (round-3 product) vs DIV=2
#    (tools/ab/lib_div{1,2}.so, LRSPNP_LIB);
#  - configs[2] (default): the 98^2 register BN forward on 1024- vs 256-thread workgroups
#    (tuning build, LRS_DIP_BNR_SMALL_WG).
set -o pipefail
o=gpurun_out/r04a
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
for r in 1 2; do
  for v in div1 div2; do
    LRSPNP_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 200 python bench.py --workload pnp --no-cpu-baseline --steps 20 > $o/pnp_${v}_$r.json 2> $o/pnp_${v}_$r.err || { tail $o/pnp_${v}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$o/pnp_${v}_$r.json').read().strip().splitlines()[-1]); print('pnp $v run $r', round(d['value'],2), d['roofline'].get('kernels', d['roofline']))"
  done
done
for r in 1 2; do
  for v in 0 1; do
    LRS_DIP_BNR_SMALL_WG=$v LRSPNP_LIB=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so timeout -k 10 240 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $o/bnr_${v}_$r.json 2> $o/bnr_${v}_$r.err || { tail $o/bnr_${v}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$o/bnr_${v}_$r.json').read().strip().splitlines()[-1]); print('bnr small_wg $v run $r', round(d['value'],3), d['ms_per_step'])"
  done
done
