set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dip.py tests/test_gpu_nn.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pt_dip.log 2>&1 || { tail -30 gpurun_out/pt_dip.log; exit 1; }
tail -1 gpurun_out/pt_dip.log
bash tools/ab_libs_step.sh head new pf2 cheap || exit 1
LRSPNP_LIB=$PWD/tools/ab/lib_cheap.so bash tools/gpu_timeline.sh unet1lip 198 196 12 || exit 1
cp gpurun_out/timeline_unet1lip_196.txt gpurun_out/timeline_cheap_196.txt
LRSPNP_LIB=$PWD/tools/ab/lib_pf2.so bash tools/gpu_timeline.sh unet1lip 198 196 12 || exit 1
