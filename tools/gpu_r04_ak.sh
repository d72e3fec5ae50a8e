#!/bin/bash
# Round 4: implicit-GEMM threshold 1024 (product default now): the DIP / nn / e2e / solver GPU tests,
# then 196^2 U-Net step at 1024 vs 512 (its 25^2 maps are 625 pixels; tuning build), 2 rounds.
set -o pipefail
o=gpurun_out/r04ak
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dip.py tests/test_gpu_nn.py tests/test_gpu_e2e_dip.py tests/test_gpu_solver.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $o/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $o/pytest.log | head -20; tail -5 $o/pytest.log; exit 1; }
tail -1 $o/pytest.log
T=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
for r in 1 2; do
  for v in 1024 512; do
    LRSPNP_LIB=$T LRS_DIP_IMPLICIT_MIN_P=$v timeout -k 10 200 python tools/dip_steptime.py --rounds 3 > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
    echo "min_p=$v round $r unet 196: $(tail -1 $o/st.txt)"
  done
done
