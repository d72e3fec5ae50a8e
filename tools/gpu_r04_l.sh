#!/bin/bash
# Round 4: the multi-workgroup eigensolver chain (LRS_SVT_MULTI_WG): bit-identity with the
# one-workgroup chain, every SVT test, the row-slab sharding tests (sharded ranks use it), timing.
set -o pipefail
o=gpurun_out/r04l
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_solver.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "svt or slab or config1 or pnp" > $o/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $o/pytest.log | head -20; tail -5 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
for P in 5000 40000; do
  timeout -k 10 120 python tools/time_svt.py --P $P --B 198 > $o/svt_$P.json 2> $o/svt.err || { tail $o/svt.err; exit 1; }
  cat $o/svt_$P.json
done
