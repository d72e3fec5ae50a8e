#!/bin/bash
# Round 4: per-pattern Gram sparse coding after the prepare / execute split: parity, the kernel alone
# (4 vs 8 waves, NLM vs soft prox), configs[2] bench.
set -o pipefail
o=gpurun_out/r04i
mkdir -p $o
export TMPDIR=/tmp
TL=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solver.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "pattern or sparse_coding or ista" > $o/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $o/pytest.log | head -20; tail -5 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for wv in 4 8; do
  for v in fro4 soft; do
    LRS_ISTA_PAT_WAVES=$wv LRSPNP_LIB=$TL timeout -k 10 200 python tools/time_ista.py --only cfg2 --variant $v --reps 5 > $o/t_${wv}_$v.json 2> $o/t_${wv}_$v.err || { tail $o/t_${wv}_$v.err; exit 1; }
    echo "waves $wv prox $v: $(python -c "import json; d=json.loads(open('$o/t_${wv}_$v.json').read().strip().splitlines()[-1]); print(d['path'], round(d['ms'],3), 'ms', round(d['tflops'],1), 'TF')")"
  done
done
LRS_ISTA_PAT_WAVES=8 LRSPNP_LIB=$TL timeout -k 10 300 python tools/time_ista.py --only cfg3 --reps 3 > $o/t3_8.json 2> $o/t3_8.err || { tail $o/t3_8.err; exit 1; }
LRS_ISTA_PAT_WAVES=4 LRSPNP_LIB=$TL timeout -k 10 300 python tools/time_ista.py --only cfg3 --reps 3 > $o/t3_4.json 2> $o/t3_4.err || { tail $o/t3_4.err; exit 1; }
timeout -k 10 300 python tools/time_ista.py --only cfg3 --reps 3 --patterns off > $o/t3_off.json 2> $o/t3_off.err || { tail $o/t3_off.err; exit 1; }
tail -qn1 $o/t3_8.json $o/t3_4.json $o/t3_off.json | cut -c1-200
for r in 1 2; do
  for wv in 4 8; do
    LRS_ISTA_PAT_WAVES=$wv LRSPNP_LIB=$TL timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $o/b_${wv}_$r.json 2> $o/b_${wv}_$r.err || { tail $o/b_${wv}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$o/b_${wv}_$r.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels'][0]; print('bench waves $wv run $r', round(d['value'],3), round(d['ms_per_step'],2), 'ista ms', round(k['ms_per_launch'],3))"
  done
done
