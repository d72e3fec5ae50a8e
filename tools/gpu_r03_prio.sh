set -o pipefail
# A/B of the low-rank (DIP) stream priority at configs[2] (bench.py --lowrank-priority), alternating
# runs on one box, then the kernel stats of the high-priority run (max vs mean of the DIP kernels).
mkdir -p gpurun_out/prio
o=gpurun_out/prio
export TMPDIR=/tmp
for r in 1 2; do
  for p in 0 -1; do
    timeout -k 10 240 python bench.py --no-cpu-baseline --steps 5 --warmup 1 --lowrank-priority $p > $o/b_${p}_$r.json 2> $o/b_${p}_$r.err || { tail $o/b_${p}_$r.err; exit 1; }
    python -c "import json,sys; d=json.load(open('$o/b_${p}_$r.json')); print('prio $p run $r', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --lowrank-priority -1 > $o/prof.log 2>&1 || { tail $o/prof.log; exit 1; }
f=$(find $o/prof -name '*kernel_stats.csv' | head -n 1)
cp "$f" $o/dip_kernel_stats_prio.csv
python - <<'EOF'
import csv
for x in csv.DictReader(open('gpurun_out/prio/dip_kernel_stats_prio.csv')):
    mx, av = float(x['MaxNs']), float(x['AverageNs'])
    if mx > 5 * av:
        print('max/mean %.1f' % (mx / av), x['Name'][:70], av, mx)
EOF
