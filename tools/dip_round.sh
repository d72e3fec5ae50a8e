#!/bin/bash
# GPU box: DIP tests, both DIP workload benches, kernel-trace stats of the configs[2] bench.
set -o pipefail
mkdir -p gpurun_out/dip_$1
export TMPDIR=/tmp
o=gpurun_out/dip_$1
timeout -k 10 600 python -u -m pytest tests/test_gpu_dip.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest.log 2>&1 || { tail -40 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
timeout -k 10 400 python bench.py --workload dip --steps 3 --warmup 1 --no-cpu-baseline > $o/dip_bench.json 2> $o/dip_bench.err || { tail $o/dip_bench.err; exit 1; }
cat $o/dip_bench.json
timeout -k 10 400 python bench.py --workload dip-pro --steps 2 --warmup 1 --no-cpu-baseline > $o/dip_pro_bench.json 2> $o/dip_pro_bench.err || { tail $o/dip_pro_bench.err; exit 1; }
cat $o/dip_pro_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $o/trace -o dip --output-format csv -- python bench.py --workload dip --steps 2 --warmup 1 --no-cpu-baseline > $o/trace.log 2>&1 || { tail $o/trace.log; exit 1; }
echo dip-ok
