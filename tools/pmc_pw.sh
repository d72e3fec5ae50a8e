set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcpw
timeout -k 10 60 python tools/micro_conv.py 128 198 196 196 1 1 0 0 --reps 20
timeout -k 10 60 python tools/micro_conv.py 128 198 196 196 1 1 0 0 --reps 20 --explicit
timeout -k 10 60 python tools/micro_conv.py 128 128 196 196 1 1 0 0 --reps 20
timeout -k 10 60 python tools/micro_conv.py 128 128 98 98 3 1 1 1 --reps 20
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE"; do
  n=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 60 rocprofv3 --pmc $pass -d gpurun_out/pmcpw/$n -o run --output-format csv -- python3 tools/micro_conv.py 128 198 196 196 1 1 0 0 --reps 5 > /dev/null 2>&1 || exit 1
done
python - <<'PY'
import csv,glob,collections
acc=collections.defaultdict(list)
for f in glob.glob('gpurun_out/pmcpw/*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        if 'k_pw' in r['Kernel_Name']:
            acc[r['Counter_Name']].append(float(r['Counter_Value']))
for k,v in sorted(acc.items()): print(k, sum(v)/len(v))
PY
rm -rf gpurun_out/pmcpw
