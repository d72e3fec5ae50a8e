set -o pipefail
# A/B of library builds under tools/ab/lib_*.so (LRSPNP_LIB): one conv micro + the default bench each,
# interleaved twice to see the noise
for rnd in 1 2; do
for v in "$@"; do
  export LRSPNP_LIB=$PWD/tools/ab/lib_$v.so
  echo "== $v"
  timeout -k 10 60 python tools/micro_conv.py 128 128 98 98 3 1 1 1 --reps 20 || exit 1
  timeout -k 10 60 python tools/micro_conv.py 128 128 98 98 3 1 1 1 --bwd --reps 20 || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 > gpurun_out/ab_$v.json 2> gpurun_out/ab.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('bench', round(d['value'],4), round(d['roofline']['ms_per_outer_iter'],2))"
done
done
