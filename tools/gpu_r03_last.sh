#!/bin/bash
# Round-3 closing check at HEAD: full GPU suite, smoke, default bench line (configs[2]).
set -o pipefail
o=gpurun_out/r03last
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $o/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { echo smoke failed; cat $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
timeout -k 10 300 python bench.py > $o/bench.json 2> $o/bench.err || { echo bench failed; tail $o/bench.err; exit 1; }
cat $o/bench.json
