#!/bin/bash
# Round-2 profile on the GPU box, per workload (dip = bench default / configs[2], pnp = configs[1]):
#   bench JSON; rocprofv3 --kernel-trace --stats of the same bench command (no CPU baseline);
#   separate PMC passes FETCH_SIZE, WRITE_SIZE, and an SQ pass — never combined with tracing.
# Then: python tools/summarize_r02.py gpurun_out/profile_r02 profiles/r02  (in the build container)
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/profile_r02
mkdir -p $out
for wl in ${WORKLOADS:-dip pnp}; do
  if [ $wl = dip ]; then S="--steps 3 --warmup 1"; else S="--steps 10 --warmup 2"; fi
  B="bench.py --workload $wl $S --no-cpu-baseline"
  echo "== $wl bench"
  timeout -k 10 400 python bench.py --workload $wl $S > $out/${wl}_bench.json 2> $out/${wl}_bench.err || exit 1
  echo "== $wl trace"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/${wl}_trace -o run --output-format csv -- python3 $B > $out/${wl}_trace.log 2>&1 || exit 1
  echo "== $wl fetch"
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $out/${wl}_fetch -o run --output-format csv -- python3 $B > $out/${wl}_fetch.log 2>&1 || exit 1
  echo "== $wl write"
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $out/${wl}_write -o run --output-format csv -- python3 $B > $out/${wl}_write.log 2>&1 || exit 1
  echo "== $wl sq"
  timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $out/${wl}_sq -o run --output-format csv -- python3 $B > $out/${wl}_sq.log 2>&1 || exit 1
done
# summarise on the box (the raw per-dispatch CSVs exceed what gpurun copies back), keep only the summary
python tools/summarize_r02.py $out ${SUMDIR:-gpurun_out/r02sum} > $out/summary.log 2>&1 || { cat $out/summary.log; exit 1; }
rm -rf $out/*_trace $out/*_fetch $out/*_write $out/*_sq
echo profile-ok
