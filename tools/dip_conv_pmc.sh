#!/bin/bash
# GPU box: MFMA utilisation and HBM bytes of the implicit-GEMM conv kernels on one 512x512
# 128->128 3x3 layer (tools/diag_conv_one.py), one rocprofv3 pass per counter group.
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/dip_conv_pmc
mkdir -p $out
cmd="python tools/diag_conv_one.py 128 128 512 512 3 1 1 0 3"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o run -- $cmd > $out/trace.log 2>&1 || { echo trace failed; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_ANY --output-format csv -d $out/sq -o run -- $cmd > $out/sq.log 2>&1 || { echo sq failed; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- $cmd > $out/fetch.log 2>&1 || { echo fetch failed; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o run -- $cmd > $out/write.log 2>&1 || { echo write failed; exit 1; }
echo all-ok
