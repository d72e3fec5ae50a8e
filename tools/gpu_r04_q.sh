#!/bin/bash
# Round 4: re-sweep of the DIP engine's tuning knobs at 196^2 now that the sparse coding beside it is
# short (tuning build, tools/dip_steptime.py, baseline interleaved).
set -o pipefail
o=gpurun_out/r04q
mkdir -p $o
export TMPDIR=/tmp
TL=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
run() {   # name, env assignments...
  local name=$1; shift
  env "$@" LRSPNP_LIB=$TL timeout -k 10 120 python tools/dip_steptime.py --rounds 5 > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
  echo "$name: $(tail -1 $o/st.txt)"
}
run base X=1
run fwd256 LRS_DIP_FWD_SPLIT_WG=256
run fwd512 LRS_DIP_FWD_SPLIT_WG=512
run base X=1
run sm480 LRS_DIP_SM_WG=480
run sm800 LRS_DIP_SM_WG=800
run base X=1
run prep256 LRS_DIP_PREP_WG=256
run prep1024 LRS_DIP_PREP_WG=1024
run base X=1
run dgrad384 LRS_DIP_DGRAD_SPLIT_WG=384
run implicit4096 LRS_DIP_IMPLICIT_MIN_P=4096
run base X=1
