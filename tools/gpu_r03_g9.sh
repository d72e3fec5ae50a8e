set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dip.py tests/test_gpu_nn.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_dip.log 2>&1 || { tail -30 gpurun_out/pt_dip.log; exit 1; }
tail -1 gpurun_out/pt_dip.log
bash tools/ab_libs_step.sh wg adam || exit 1
STEP_ARGS="--hw 36 --bands 128" bash tools/ab_libs_step.sh wg adam || exit 1
