#!/bin/bash
# Round 4: the per-pattern sparse coding back on its unspilled 192-register form: its tests, then the
# HEAD profile (tools/final_r04.sh: kernel trace + PMC passes -> gpurun_out/r04sum).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04z
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solver.py -m gpu -q -x -p no:cacheprovider --timeout 150 --timeout-method thread -k "pattern or config2 or config3" > gpurun_out/r04z/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" gpurun_out/r04z/pytest.log | head -20; tail -5 gpurun_out/r04z/pytest.log; exit 1; }
tail -1 gpurun_out/r04z/pytest.log
bash tools/final_r04.sh
