#!/bin/bash
# Round profile on the GPU box: bench JSON, kernel-trace --stats of the same bench command, and
# separate PMC passes for HBM traffic (FETCH_SIZE, WRITE_SIZE) — never combined with tracing.
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r01}
out=gpurun_out/profile_$tag
mkdir -p $out
B="python bench.py --steps 5 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 python bench.py --steps 10 --warmup 2 > $out/bench.json 2> $out/bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/trace -o run --output-format csv -- $B > $out/trace.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $out/fetch -o run --output-format csv -- $B > $out/fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $out/write -o run --output-format csv -- $B > $out/write.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $out/sq -o run --output-format csv -- $B > $out/sq.log 2>&1 || exit 1
echo profile-ok
