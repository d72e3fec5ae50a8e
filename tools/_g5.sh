set -o pipefail
export OUT=gpurun_out/g5 TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_dip.py -m gpu -q -x -p no:cacheprovider --timeout 150 --timeout-method thread -k "196 or graph or priority or golden" > $OUT/pytest_dip.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $OUT/pytest_dip.log | head -30; tail -5 $OUT/pytest_dip.log; exit 1; }
tail -1 $OUT/pytest_dip.log
ROUNDS=3 tools/gpu.sh steptime "u196@--rounds 3" "u196_ov0:LRSPNP_LIB=tune,LRS_DIP_SN_OVERLAP=0@--rounds 3" "u196_r04:LRSPNP_LIB=r04@--rounds 3" "u36@--hw 36 --bands 128 --rounds 3" "u36_r04:LRSPNP_LIB=r04@--hw 36 --bands 128 --rounds 3" &&
tools/gpu.sh trace e196 python tools/dip_steptime.py --rounds 1 --steps 20
