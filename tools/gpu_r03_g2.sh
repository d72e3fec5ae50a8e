set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/micro/event_cost.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_dip.py tests/test_gpu_nn.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_dip.log 2>&1 || { tail -30 gpurun_out/pt_dip.log; exit 1; }
tail -1 gpurun_out/pt_dip.log
bash tools/ab_steptime.sh "LRS_DIP_X=0" "LRS_DIP_FORK_SET=13,12,11,10,7,4,1,0" "LRS_DIP_FORK_SET=13,12,11,10,8,6,4,2,1,0" "LRS_DIP_FORK_SET=13,12,11,10,9,6,3,1,0"
