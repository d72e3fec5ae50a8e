#!/bin/bash
# One GPU-box check: selected GPU tests (default: all), the default bench line, the DIP step time.
#   TESTS="tests/test_gpu_dip.py" BENCH=1 STEP=1 bash tools/gpu_step.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TESTS:-tests}
if [ "${PYTEST:-1}" = 1 ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-500} python -u -m pytest $T -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 300 python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
if [ "${STEP:-0}" = 1 ]; then
  timeout -k 10 200 python tools/dip_steptime.py --rounds 5 ${STEP_ARGS:-} > gpurun_out/steptime.txt 2>&1 || { echo steptime failed; tail gpurun_out/steptime.txt; exit 1; }
  cat gpurun_out/steptime.txt
fi
