set -o pipefail
# PMC passes for one conv layer's kernels (micro_conv.py args in $@), summarised per kernel name
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcc
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM" "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $pass -d gpurun_out/pmcc/p$i -o run --output-format csv -- python3 tools/micro_conv.py "$@" --reps 3 > gpurun_out/pmcc/p$i.log 2>&1 || { tail -5 gpurun_out/pmcc/p$i.log; exit 1; }
done
python - <<'PY'
import csv,glob,collections
acc=collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pmcc/*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        k=r['Kernel_Name'].split('(')[0][-60:]
        acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k,d in acc.items():
    print(k)
    for c,v in sorted(d.items()): print('   ', c, sum(v)/len(v))
PY
rm -rf gpurun_out/pmcc
