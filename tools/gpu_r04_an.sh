#!/bin/bash
# Round 4: graph replay vs eager for the DIP training step at HEAD (36^2 x 128 and 196^2 x 198),
# 2 interleaved rounds.
set -o pipefail
o=gpurun_out/r04an
mkdir -p $o
export TMPDIR=/tmp
for r in 1 2; do
  for g in "" "--graph"; do
    timeout -k 10 200 python tools/dip_steptime.py --net unet --hw 36 --bands 128 --rounds 3 $g > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
    echo "36 eager/graph[$g] round $r: $(tail -1 $o/st.txt)"
    timeout -k 10 200 python tools/dip_steptime.py --rounds 3 $g > $o/st.txt 2>&1 || { tail $o/st.txt; exit 1; }
    echo "196 eager/graph[$g] round $r: $(tail -1 $o/st.txt)"
  done
done
