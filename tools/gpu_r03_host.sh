#!/bin/bash
# Is the DIP step host-launch-bound?  Host enqueue vs GPU time, eager and graph, 196^2 and 36^2;
# then the configs[1] A/B against the round-1 tree.
set -o pipefail
mkdir -p gpurun_out/r03
o=gpurun_out/r03
export TMPDIR=/tmp
for hw in 196 36; do
  b=198; [ $hw = 36 ] && b=128
  timeout -k 10 120 python tools/host_enqueue.py --hw $hw --bands $b > $o/host_${hw}.log 2>&1 || { cat $o/host_${hw}.log; exit 1; }
  timeout -k 10 120 python tools/host_enqueue.py --hw $hw --bands $b --graph > $o/host_${hw}_graph.log 2>&1 || { cat $o/host_${hw}_graph.log; exit 1; }
  timeout -k 10 120 python tools/dip_steptime.py --hw $hw --bands $b --rounds 3 --graph > $o/step${hw}_graph.log 2>&1 || exit 1
  echo "== $hw"; cat $o/host_${hw}.log $o/host_${hw}_graph.log $o/step${hw}_graph.log | grep -v amdgpu.ids
done
bash tools/ab_pnp_r01.sh
