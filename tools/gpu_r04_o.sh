#!/bin/bash
# Round 4: the weight-gradient side stream at every size: the whole GPU suite, smoke, the native
# 36^2 x 128 line and the default bench.
set -o pipefail
o=gpurun_out/r04o
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 150 --timeout-method thread -rA > $o/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $o/pytest_gpu.log | head -30; tail -5 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 300 python bench.py --cube 36x36x128 --steps 20 --warmup 3 --no-cpu-baseline > $o/native36_bench.json 2> $o/native36.err || { tail $o/native36.err; exit 1; }
python -c "import json; d=json.loads(open('$o/native36_bench.json').read().strip().splitlines()[-1]); print('native36', d['value'], d['ms_per_step'], d['roofline']['ms_per_outer_iter'])"
timeout -k 10 120 python tools/dip_steptime.py --hw 36 --bands 128 --rounds 5 > $o/st36.txt 2>&1 || { tail $o/st36.txt; exit 1; }
echo "36: $(tail -1 $o/st36.txt)"
timeout -k 10 120 python tools/dip_steptime.py --rounds 5 > $o/st196.txt 2>&1 || { tail $o/st196.txt; exit 1; }
echo "196: $(tail -1 $o/st196.txt)"
timeout -k 10 300 python bench.py > $o/bench_default.json 2> $o/bench_default.err || { tail $o/bench_default.err; exit 1; }
python -c "import json; d=json.loads(open('$o/bench_default.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernels'][0]['ms_per_launch'], d.get('cpu_baseline',{}).get('value'))"
