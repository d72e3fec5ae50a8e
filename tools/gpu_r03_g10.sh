set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_all.log 2>&1 || { tail -30 gpurun_out/pt_all.log; exit 1; }
tail -1 gpurun_out/pt_all.log
bash tools/ab_libs_step.sh adam adam2 || exit 1
bash tools/gpu_r03_g11.sh || exit 1
