#!/bin/bash
# Round 4: the DIP engine's launch knobs at the configs[3] size (512^2 x 224 skip net; tuning build),
# 2 interleaved rounds against the default.
set -o pipefail
o=gpurun_out/r04ao
mkdir -p $o
export TMPDIR=/tmp
T=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
run() {
  env LRSPNP_LIB=$T "$@" timeout -k 10 200 python tools/dip_steptime.py --net skip --hw 512 --bands 224 --rounds 3 --steps 10 > $o/st.txt 2>&1 || { tail $o/st.txt; return 1; }
  echo "$* : $(tail -1 $o/st.txt)"
}
for r in 1 2; do
  run X=default || exit 1
  run LRS_DIP_FWD_SPLIT_WG=256 || exit 1
  run LRS_DIP_FWD_SPLIT_WG=512 || exit 1
  run LRS_DIP_DGRAD_SPLIT_WG=256 || exit 1
  run LRS_DIP_SPLIT_CAP=128 || exit 1
  run LRS_DIP_PREP_WG=256 || exit 1
  run LRS_DIP_UPC=0 || exit 1
done
