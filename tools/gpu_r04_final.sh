#!/bin/bash
# Round-4 end-of-round evidence at HEAD: the whole GPU suite, smoke, the default bench (configs[2],
# with the CPU baseline), configs[3] (dip-pro 512^2x224), the literal 200^2x198 skip-net line,
# configs[1] (pnp), the native 36^2x128 line, and the driver's torchrun launch form at N = 1 (RCCL).
set -o pipefail
o=gpurun_out/r04final
mkdir -p $o
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 150 --timeout-method thread -rA > $o/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $o/pytest_gpu.log | head -30; tail -5 $o/pytest_gpu.log; exit 1; }
tail -1 $o/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail $o/smoke.log; exit 1; }
tail -2 $o/smoke.log
timeout -k 10 300 python bench.py > $o/bench_default.json 2> $o/bench_default.err || { tail $o/bench_default.err; exit 1; }
python -c "import json; d=json.loads(open('$o/bench_default.json').read().strip().splitlines()[-1]); print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernels'][0]['ms_per_launch'], d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 400 python bench.py --workload dip-pro --steps 3 --warmup 1 --no-cpu-baseline > $o/dip_pro.json 2> $o/dip_pro.err || { tail $o/dip_pro.err; exit 1; }
python -c "import json; d=json.loads(open('$o/dip_pro.json').read().strip().splitlines()[-1]); print('configs[3]', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['kernels'][0]['ms_per_launch'])"
timeout -k 10 300 python bench.py --workload dip-pro --cube 200x200x198 --steps 3 --warmup 1 --no-cpu-baseline > $o/dip_pro_200.json 2> $o/dip_pro_200.err || { tail $o/dip_pro_200.err; exit 1; }
python -c "import json; d=json.loads(open('$o/dip_pro_200.json').read().strip().splitlines()[-1]); print('literal 200^2x198 skip:', d['value'], d['ms_per_step'], d['roofline']['kernels'][0]['ms_per_launch'])"
timeout -k 10 200 python bench.py --workload pnp --steps 20 --warmup 3 --no-cpu-baseline > $o/pnp.json 2> $o/pnp.err || { tail $o/pnp.err; exit 1; }
python -c "import json; d=json.loads(open('$o/pnp.json').read().strip().splitlines()[-1]); print('configs[1]', d['value'], d['ms_per_step'])"
timeout -k 10 300 python bench.py --cube 36x36x128 --steps 20 --warmup 3 --no-cpu-baseline > $o/native36_bench.json 2> $o/native36.err || { tail $o/native36.err; exit 1; }
python -c "import json; d=json.loads(open('$o/native36_bench.json').read().strip().splitlines()[-1]); print('native36', d['value'], d['ms_per_step'], d['roofline']['ms_per_outer_iter'])"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $o/torchrun_n1.json 2> $o/torchrun_n1.err || { tail -20 $o/torchrun_n1.err; exit 1; }
python -c "import json; d=json.loads(open('$o/torchrun_n1.json').read().strip().splitlines()[-1]); print('torchrun N=1', d['value'], d['ms_per_step'])"
