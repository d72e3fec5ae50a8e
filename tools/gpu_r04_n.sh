#!/bin/bash
# Round 4: native 36^2 x 128 DIP step (item 7): the weight-gradient side stream (LRS_DIP_FORK, tuning
# build) and graph replay, interleaved.
set -o pipefail
o=gpurun_out/r04n
mkdir -p $o
export TMPDIR=/tmp
TL=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || { tail $o/smoke.log; exit 1; }
tail -1 $o/smoke.log
for r in 1 2; do
  for f in 0 1; do
    for gr in "" "--graph"; do
      LRS_DIP_FORK=$f LRSPNP_LIB=$TL timeout -k 10 120 python tools/dip_steptime.py --hw 36 --bands 128 --rounds 5 --steps 100 $gr > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
      echo "fork $f graph '$gr' round $r: $(tail -1 $o/st.txt)"
    done
  done
done
for fs in "13,11,9,7,5,3,1" "13,12,11,10,9,8,7,6,5,4,3,2,1,0" "13,10,7,4,1"; do
  LRS_DIP_FORK=1 LRS_DIP_FORK_SET=$fs LRSPNP_LIB=$TL timeout -k 10 120 python tools/dip_steptime.py --hw 36 --bands 128 --rounds 5 --steps 100 > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
  echo "fork set $fs: $(tail -1 $o/st.txt)"
done
