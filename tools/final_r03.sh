#!/bin/bash
# Round-3 evidence on the GPU box: full GPU suite, smoke, default bench line (+ configs[3] and
# configs[1] lines), then the profile (tools/profile_r02.sh: kernel trace + separate FETCH_SIZE /
# WRITE_SIZE / SQ passes, summarised on the box into gpurun_out/r03sum).
set -o pipefail
mkdir -p gpurun_out/r03
o=gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo smoke failed; cat $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err || { echo bench failed; tail $o/bench.err; exit 1; }
cat $o/bench.json
timeout -k 10 300 python bench.py --workload pnp > $o/pnp_bench.json 2> $o/pnp_bench.err || { echo pnp failed; tail $o/pnp_bench.err; exit 1; }
timeout -k 10 400 python bench.py --workload dip-pro --steps 2 --warmup 1 > $o/dip_pro_bench.json 2> $o/dip_pro_bench.err || { echo dip-pro failed; tail $o/dip_pro_bench.err; exit 1; }
timeout -k 10 200 python tools/dip_steptime.py --rounds 5 > $o/step196.log 2>&1 || exit 1
timeout -k 10 200 python tools/dip_steptime.py --hw 36 --bands 128 --rounds 5 > $o/step36.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --cube 36x36x128 --no-cpu-baseline --steps 5 --warmup 1 > $o/native36_bench.json 2> $o/native36.err || { tail $o/native36.err; exit 1; }
tail -1 $o/step196.log $o/step36.log
SUMDIR=gpurun_out/r03sum bash tools/profile_r02.sh
