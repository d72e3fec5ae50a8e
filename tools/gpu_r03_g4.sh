set -o pipefail
mkdir -p gpurun_out/r03
o=gpurun_out/r03
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $o/bench_g4.json 2> $o/bench_g4.err || { tail $o/bench_g4.err; exit 1; }
python -c "import json; d=json.loads(open('$o/bench_g4.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['roofline']['frac'], d['roofline']['alg_bytes'], d['roofline']['kernels'][0]['ms_per_launch'])"
bash tools/gpu_timeline.sh unet1lip 198 196 12 || exit 1
bash tools/pmc_step_waits.sh 198 196 || exit 1
