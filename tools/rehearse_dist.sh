#!/bin/bash
# GPU box rehearsal of bench.py's multi-rank paths with 2 gloo ranks sharing the one GPU
# (the driver runs the real N>1 RCCL benches on an 8-GPU node): per workload (dip = the default,
# configs[2]; pnp = configs[1]) one cube per rank (weak) and one cube over both ranks (--split-cube:
# dip task-parallel, pnp pixel-row slabs).  Output: gpurun_out/dist/<workload>_{weak,split}.json
set -o pipefail
mkdir -p gpurun_out/dist
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
port=29511
for wl in dip pnp; do
  for mode in weak split; do
    extra=""; [ $mode = split ] && extra="--split-cube"
    timeout -k 10 300 $R --master-port $port bench.py --workload $wl --gpus 2 --backend gloo $extra --steps 3 --warmup 1 \
      --no-cpu-baseline > gpurun_out/dist/${wl}_${mode}.json 2> gpurun_out/dist/${wl}_${mode}.err \
      || { tail -20 gpurun_out/dist/${wl}_${mode}.err; exit 1; }
    grep -h '"metric"' gpurun_out/dist/${wl}_${mode}.json | cut -c1-200
    port=$((port + 1))
  done
done
