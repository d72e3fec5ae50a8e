#!/bin/bash
# Round 4 evidence at HEAD: the whole GPU suite (incl. the new headline-path parity tests), the
# configs[1] A/B against the round-1 tree, the literal 200^2x198 configs[2] line (skip net), and a
# kernel trace of the default bench (co-scheduling stall).
set -o pipefail
o=gpurun_out/r04d
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 150 --timeout-method thread -rA > $o/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $o/pytest_gpu.log | head -30; tail -5 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
grep -E "GPU \[|worst" $o/pytest_gpu.log | head
timeout -k 10 300 python bench.py --workload dip-pro --cube 200x200x198 --steps 3 --warmup 1 --no-cpu-baseline > $o/dip_pro_200.json 2> $o/dip_pro_200.err || { tail $o/dip_pro_200.err; exit 1; }
python -c "import json; d=json.loads(open('$o/dip_pro_200.json').read().strip().splitlines()[-1]); print('literal 200^2x198 skip:', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['mpsnr'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/trdip -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $o/trace_dip.log 2>&1 || { tail $o/trace_dip.log; exit 1; }
cp $(find /tmp/trdip -name "*kernel_stats.csv" | head -1) $o/dip_kernel_stats.csv
head -14 $o/dip_kernel_stats.csv | cut -c1-160
bash tools/ab_pnp_r01.sh > $o/ab_pnp.log 2>&1 || { tail $o/ab_pnp.log; exit 1; }
cat $o/ab_pnp.log | cut -c1-200
