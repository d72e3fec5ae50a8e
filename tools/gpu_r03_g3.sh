set -o pipefail
mkdir -p gpurun_out/r03
o=gpurun_out/r03
timeout -k 10 500 python -u -m pytest tests -m gpu -q -p no:cacheprovider -x --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { tail -40 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
timeout -k 10 300 python tools/time_ista.py --reps 3 > $o/time_ista.log 2>&1 || { tail $o/time_ista.log; exit 1; }
grep -v amdgpu.ids $o/time_ista.log
timeout -k 10 200 python tools/dip_steptime.py --rounds 5 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > $o/bench_g3.json 2> $o/bench_g3.err || { tail $o/bench_g3.err; exit 1; }
python -c "import json; d=json.loads(open('$o/bench_g3.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['roofline']['frac'], d['roofline']['kernels'][0]['ms_per_launch'], d['roofline']['kernels'][0]['frac'])"
timeout -k 10 300 python tools/e2e_dip_gpu.py > $o/e2e_g3.log 2>&1 || { tail $o/e2e_g3.log; exit 1; }
tail -5 $o/e2e_g3.log
