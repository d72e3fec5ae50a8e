set -o pipefail
mkdir -p gpurun_out/r03
o=gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -p no:cacheprovider -k "warm_start or bounded_grid or ista_kernel_vs_oracle" --timeout 120 --timeout-method thread > $o/pt_warm.log 2>&1 || { tail -30 $o/pt_warm.log; exit 1; }
tail -1 $o/pt_warm.log
for r in 1 2; do
for sl in 1 4 10 25; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --ista-slices $sl > $o/sl_$sl.json 2> $o/sl.err || { tail $o/sl.err; exit 1; }
  python -c "import json; d=json.loads(open('$o/sl_$sl.json').read().strip().splitlines()[-1]); print('slices $sl', round(d['value'],4), 'dip ms', round(d['roofline']['ms_per_outer_iter'],2), 'ista ms', round(d['roofline']['kernels'][0]['ms_per_launch'],2))"
done
done
