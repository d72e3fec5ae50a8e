#!/bin/bash
# GPU box rehearsal of bench.py's multi-rank paths with 2 gloo ranks sharing the one GPU
# (the driver runs the real N>1 RCCL benches on an 8-GPU node).
set -o pipefail
mkdir -p gpurun_out/dist
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
timeout -k 10 300 $R --master-port 29511 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dist/weak.json 2> gpurun_out/dist/weak.err || { tail -20 gpurun_out/dist/weak.err; exit 1; }
cat gpurun_out/dist/weak.json
timeout -k 10 300 $R --master-port 29512 bench.py --gpus 2 --backend gloo --split-cube --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/dist/split.json 2> gpurun_out/dist/split.err || { tail -20 gpurun_out/dist/split.err; exit 1; }
cat gpurun_out/dist/split.json
