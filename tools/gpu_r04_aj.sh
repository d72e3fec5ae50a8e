#!/bin/bash
# Round 4: the implicit-GEMM threshold on the other nets: 512^2 skip net (its 32^2 maps are 1024
# pixels) at 2048 / 1024, and 36^2 U-Net at 1100; 2 interleaved rounds.
set -o pipefail
o=gpurun_out/r04aj
mkdir -p $o
export TMPDIR=/tmp
T=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
for r in 1 2; do
  for v in 2048 1024; do
    LRSPNP_LIB=$T LRS_DIP_IMPLICIT_MIN_P=$v timeout -k 10 200 python tools/dip_steptime.py --net skip --hw 512 --bands 224 --rounds 3 --steps 10 > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
    echo "min_p=$v round $r skip 512: $(tail -1 $o/st.txt)"
  done
  for v in 2048 1100; do
    LRSPNP_LIB=$T LRS_DIP_IMPLICIT_MIN_P=$v timeout -k 10 200 python tools/dip_steptime.py --net unet --hw 36 --bands 128 --rounds 3 > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
    echo "min_p=$v round $r unet 36: $(tail -1 $o/st.txt)"
  done
done
