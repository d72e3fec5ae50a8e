#!/bin/bash
# Round 4: k_sn_sigma phase timing (load / Lanczos / checks / final multisection) on the U-Net weights
# after 0, 30 and 90 Adam steps, 196^2 x 198 and 36^2 x 128.
set -o pipefail
mkdir -p gpurun_out/r04af
export TMPDIR=/tmp
timeout -k 10 200 python tools/diag_sigma_net.py 198 196 0,30,90 > gpurun_out/r04af/sigma_196.txt 2>&1 || { tail gpurun_out/r04af/sigma_196.txt; exit 1; }
timeout -k 10 200 python tools/diag_sigma_net.py 128 36 0,30,90 > gpurun_out/r04af/sigma_36.txt 2>&1 || { tail gpurun_out/r04af/sigma_36.txt; exit 1; }
cat gpurun_out/r04af/sigma_196.txt
