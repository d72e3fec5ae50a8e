#!/bin/bash
# PMC passes over the ISTA ablation diagnostic (separate --pmc passes, kernel-trace only).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/pmc_ista
mkdir -p $out
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES -d $out/p1 -o run --output-format csv -- python tools/diag_ista.py 125000 20 > $out/p1.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $out/p2 -o run --output-format csv -- python tools/diag_ista.py 125000 20 > $out/p2.log 2>&1 || exit 1
echo pmc-ok
