#!/bin/bash
# Round 4: the new headline-path parity tests (196^2 U-Net / 512^2 skip gradients vs fp64, skip net on
# the literal 200^2 cube, ADVICE cases) and the configs[2] MPSNR trajectory of LrsPnP.
set -o pipefail
o=gpurun_out/r04b
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dip.py tests/test_gpu_kernels.py -m gpu -v -s -p no:cacheprovider --timeout 150 --timeout-method thread -k "bench_size_196 or config3_size or literal_config2 or warm_start or top_of_k" > $o/pytest_new.log 2>&1; rc=$?
grep -E "PASS|FAIL|worst|Error|assert" $o/pytest_new.log | head -40
[ $rc -le 1 ] || exit 1
timeout -k 10 200 python tools/traj196_gpu.py 4 4 > $o/traj.log 2>&1 || { tail $o/traj.log; exit 1; }
cat $o/traj.log
