#!/bin/bash
# The round-1 end tree (commit 1c05b02: library, package, bench, oracle) under ab_r01/ for the
# configs[1] A/B of tools/ab_pnp_r01.sh.  Built here (hipcc cross-compiles), shipped by gpurun.
set -e
rm -rf ab_r01 && mkdir ab_r01
git archive 1c05b02 lrs-pnp-dip_amd bench.py oracle include __graft_entry__.py BASELINE.json | tar -x -C ab_r01
make -s -j8 -C ab_r01/lrs-pnp-dip_amd/csrc && make -s -C ab_r01/oracle
mkdir -p ab_r01/tests/golden && git show 1c05b02:tests/golden/data_img5.npz > ab_r01/tests/golden/data_img5.npz
