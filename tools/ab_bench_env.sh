set -o pipefail
# bench.py (default workload) A/B of environment settings, interleaved twice: ab_bench_env.sh "VAR=a" ...
for rnd in 1 2; do
for v in "$@"; do
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 > gpurun_out/abb.json 2> gpurun_out/abb.err || { tail gpurun_out/abb.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/abb.json').read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], 'value', round(d['value'],4), 'dip ms', round(r['ms_per_outer_iter'],2), 'ista ms', round(r['kernels'][0]['ms_per_launch'],2))" "$v"
done
done
