# The driver's multi-GPU launch form at N = 1 on the one-GPU box (nccl = RCCL backend): torchrun,
# barrier + MAX-over-ranks timing, one JSON line from rank 0.
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03/torchrun_n1.json 2> gpurun_out/r03/torchrun_n1.err || { tail -20 gpurun_out/r03/torchrun_n1.err; exit 1; }
tail -1 gpurun_out/r03/torchrun_n1.json
