#!/bin/bash
# Round 4: the per-pattern Gram sparse coding (lrs_ista_pat_f32): parity tests, then configs[2]
# with the pattern path (auto) vs the row-split kernel (off), the kernel trace, 8-wave variant.
set -o pipefail
o=gpurun_out/r04h
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solver.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "pattern or sparse_coding or ista" > $o/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $o/pytest.log | head -20; tail -5 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for r in 1 2; do
  for m in auto off; do
    timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --ista-patterns $m > $o/pat_${m}_$r.json 2> $o/pat_${m}_$r.err || { tail $o/pat_${m}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$o/pat_${m}_$r.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels'][0]; print('$m run $r', round(d['value'],3), round(d['ms_per_step'],2), 'ista ms', round(k['ms_per_launch'],3), k['kernel'][:40], 'mpsnr', d['mpsnr'])"
  done
done
LRS_ISTA_PAT_WAVES=8 LRSPNP_LIB=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $o/pat_w8.json 2> $o/pat_w8.err || { tail $o/pat_w8.err; exit 1; }
python -c "import json; d=json.loads(open('$o/pat_w8.json').read().strip().splitlines()[-1]); k=d['roofline']['kernels'][0]; print('waves 8', round(d['value'],3), 'ista ms', round(k['ms_per_launch'],3))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/patp -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $o/trace.log 2>&1 || { tail $o/trace.log; exit 1; }
f=$(find /tmp/patp -name "*kernel_stats.csv" | head -1); cp $f $o/stats.csv
f=$(find /tmp/patp -name "*kernel_trace.csv" | head -1); cp $f $o/trace.csv
grep -E "k_ista_pat|k_pat_gram|k_ista_rs" $o/stats.csv | cut -d, -f1-4
