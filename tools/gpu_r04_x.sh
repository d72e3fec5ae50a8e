#!/bin/bash
# Round 4: size threshold of the row-quad split-K reduce (LRS_DIP_RED4 on the tuning build: 0 = scalar
# everywhere, else the minimum M N for k_gemm_reduce4), 196^2 U-Net and 512^2 skip-net step times.
set -o pipefail
o=gpurun_out/r04x
mkdir -p $o
export TMPDIR=/tmp
T=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
for r in 1 2; do
  for q in 0 1048576 4194304 16777216; do
    LRSPNP_LIB=$T LRS_DIP_RED4=$q timeout -k 10 200 python tools/dip_steptime.py --rounds 3 > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
    echo "red4=$q round $r unet 196: $(tail -1 $o/st.txt)"
    LRSPNP_LIB=$T LRS_DIP_RED4=$q timeout -k 10 200 python tools/dip_steptime.py --net skip --hw 512 --bands 224 --rounds 3 --steps 10 > $o/sk.txt 2>&1 || { tail $o/sk.txt; exit 1; }
    echo "red4=$q round $r skip 512: $(tail -1 $o/sk.txt)"
  done
done
