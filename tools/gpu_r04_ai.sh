#!/bin/bash
# Round 4: the implicit-GEMM threshold at the native 36^2 size (LRS_DIP_IMPLICIT_MIN_P on the tuning
# build: 2048 = default keeps the 36^2 maps on k_conv_sm / k_gemm64; 1024 moves them to k_gemm_s3 /
# k_pw), 36^2 U-Net step, 3 interleaved rounds.
set -o pipefail
o=gpurun_out/r04ai
mkdir -p $o
export TMPDIR=/tmp
T=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
for r in 1 2 3; do
  for v in 2048 1024; do
    LRSPNP_LIB=$T LRS_DIP_IMPLICIT_MIN_P=$v timeout -k 10 200 python tools/dip_steptime.py --net unet --hw 36 --bands 128 --rounds 3 > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
    echo "min_p=$v round $r unet 36: $(tail -1 $o/st.txt)"
  done
done
