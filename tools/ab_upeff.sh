set -o pipefail
for v in 1 0 1 0; do
  LRS_DIP_UPEFF=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 > gpurun_out/ab_$v.json 2> gpurun_out/ab.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); print('upeff=$v', round(d['value'],4), round(d['roofline']['ms_per_outer_iter'],2))"
done
