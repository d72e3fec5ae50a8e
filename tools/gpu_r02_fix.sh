set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dip.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread -k "early_stop" > gpurun_out/pytest_fix.log 2>&1 || { tail -40 gpurun_out/pytest_fix.log; exit 1; }
tail -4 gpurun_out/pytest_fix.log
bash tools/profile_r02.sh
