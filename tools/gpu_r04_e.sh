#!/bin/bash
# Round 4: (1) configs[2] A/B of the sparse coding's occupancy beside the DIP (tuning build,
# LRS_ISTA_RS_LDS: 98304 B of LDS per workgroup = one per CU); (2) k_pw alone at 196^2 (trace + SQ
# counters) for the 1x1 convs of the U-Net head.
set -o pipefail
o=gpurun_out/r04e
mkdir -p $o
export TMPDIR=/tmp
TL=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
for r in 1 2; do
  for v in 0 98304; do
    LRS_ISTA_RS_LDS=$v LRSPNP_LIB=$TL timeout -k 10 240 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > $o/occ_${v}_$r.json 2> $o/occ_${v}_$r.err || { tail $o/occ_${v}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$o/occ_${v}_$r.json').read().strip().splitlines()[-1]); print('ista lds $v run $r', round(d['value'],3), round(d['ms_per_step'],2), 'dip ms', round(d['roofline']['ms_per_outer_iter'],2), 'ista ms', round(d['roofline']['kernels'][0]['ms_per_launch'],2))"
  done
done
for cfg in "128 128 196 196 1 1 0 0" "128 198 196 196 1 1 0 0"; do
  for d in "" "--bwd"; do
    tag=$(echo "$cfg $d" | tr ' -' '__')
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/pw$tag -o run --output-format csv -- python3 tools/micro_conv.py $cfg $d --reps 30 > $o/pw$tag.log 2>&1 || { tail $o/pw$tag.log; exit 1; }
    f=$(find /tmp/pw$tag -name "*kernel_stats.csv" | head -1); echo "== $cfg $d"; cut -c1-150 $f | head -6
    timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d /tmp/pwc$tag -o run --output-format csv -- python3 tools/micro_conv.py $cfg $d --reps 5 > $o/pwc$tag.log 2>&1 || { tail $o/pwc$tag.log; exit 1; }
    f=$(find /tmp/pwc$tag -name "*counter_collection.csv" | head -1); python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:40]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    if "k_pw" not in k: continue
    c = max(n[(k, x)] for x in d)
    print(k, {x: round(v / c) for x, v in d.items()})
PY
  done
done
for r in 1 2; do
  timeout -k 10 200 python bench.py --workload pnp --steps 20 --warmup 3 --no-cpu-baseline > $o/pnp_$r.json 2> $o/pnp_$r.err || { tail $o/pnp_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$o/pnp_$r.json').read().strip().splitlines()[-1]); print('pnp run $r', round(d['value'],2), d['roofline']['ms_per_launch'])"
done
