#!/bin/bash
# Round 4: first convergence check of the sigma_max Lanczos (LRS_SN_FIRST_CHECK on the tuning build:
# 24 = the default), 196^2 and 36^2 U-Net step times, 2 interleaved rounds; sigma phases at 12 / 24.
set -o pipefail
o=gpurun_out/r04ag
mkdir -p $o
export TMPDIR=/tmp
T=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
for r in 1 2; do
  for f in 24 20 16 12; do
    LRSPNP_LIB=$T LRS_SN_FIRST_CHECK=$f timeout -k 10 200 python tools/dip_steptime.py --rounds 3 > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
    echo "first=$f round $r unet 196: $(tail -1 $o/st.txt)"
    LRSPNP_LIB=$T LRS_SN_FIRST_CHECK=$f timeout -k 10 200 python tools/dip_steptime.py --net unet --hw 36 --bands 128 --rounds 3 > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
    echo "first=$f round $r unet 36: $(tail -1 $o/st.txt)"
  done
done
for f in 12 16; do
  LRSPNP_LIB=$T LRS_SN_FIRST_CHECK=$f timeout -k 10 200 python tools/diag_sigma_net.py 198 196 0,90 > $o/sigma_$f.txt 2>&1 || { tail $o/sigma_$f.txt; exit 1; }
done
grep -h "conv  0\|conv  1 \|conv 10" $o/sigma_12.txt $o/sigma_16.txt
