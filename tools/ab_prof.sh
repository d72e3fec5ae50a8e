set -o pipefail
# per-kernel totals of the default bench for library builds tools/ab/lib_*.so, side by side
export TMPDIR=/tmp
for v in "$@"; do
  LRSPNP_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abp_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 4 > gpurun_out/abp_$v.log 2>&1 || { tail -5 gpurun_out/abp_$v.log; exit 1; }
done
python - "$@" <<'PY'
import csv, glob, sys
vs = sys.argv[1:]
tab = {}
for v in vs:
    f = glob.glob(f'gpurun_out/abp_{v}/**/run_kernel_stats.csv', recursive=True)[0]
    for r in csv.DictReader(open(f)):
        tab.setdefault(r['Name'][:90], {})[v] = (float(r['TotalDurationNs']) / 1e3, int(r['Calls']))
rows = sorted(tab.items(), key=lambda kv: -max(t for t, _ in kv[1].values()))
for k, d in rows[:40]:
    print(f"{k[:90]:90s}", "  ".join(f"{v}:{d.get(v, (0, 0))[0]:10.0f}us/{d.get(v, (0, 0))[1]:5d}" for v in vs))
PY
rm -rf gpurun_out/abp_*/
