#!/bin/bash
# Round 4: split-K cap of the small-tile GEMMs (the 1x1 convs' weight gradients over 196^2 pixels:
# 2 tiles, 64 splits) -- LRS_DIP_SPLIT_CAP on the tuning build, 196^2 and 36^2 U-Net step times.
set -o pipefail
o=gpurun_out/r04aa
mkdir -p $o
export TMPDIR=/tmp
T=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
for r in 1 2; do
  for c in 64 128 256 32; do
    LRSPNP_LIB=$T LRS_DIP_SPLIT_CAP=$c timeout -k 10 200 python tools/dip_steptime.py --rounds 3 > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
    echo "cap=$c round $r unet 196: $(tail -1 $o/st.txt)"
  done
done
for c in 64 128; do
  LRSPNP_LIB=$T LRS_DIP_SPLIT_CAP=$c timeout -k 10 200 python tools/dip_steptime.py --net unet --hw 36 --bands 128 --rounds 3 > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
  echo "cap=$c unet 36: $(tail -1 $o/st.txt)"
done
