#!/bin/bash
# Round 4: workgroups of the per-pattern sparse coding beside the DIP (bench.py --ista-max-wg,
# lrs_ista_opts.max_workgroups; 0 = one per tile, 405 at configs[2]) re-measured on k_ista_pat,
# 3 interleaved rounds of the default configs[2] bench.
set -o pipefail
o=gpurun_out/r04y
mkdir -p $o
export TMPDIR=/tmp
for r in 1 2 3; do
  for wg in 0 256 128; do
    timeout -k 10 200 python bench.py --steps 8 --warmup 1 --no-cpu-baseline --ista-max-wg $wg > $o/b.json 2> $o/b.err || { tail $o/b.err; exit 1; }
    python -c "import json; d=json.loads(open('$o/b.json').read().strip().splitlines()[-1]); print('round $r max_wg $wg', d['value'], d['ms_per_step'])"
  done
done
