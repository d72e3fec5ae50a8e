#!/bin/bash
# The one GPU launcher (run on the box through gpurun from the repo root):
#   tools/gpu.sh suite                 pytest -m gpu, then smoke()
#   tools/gpu.sh bench [tag]           every bench line (configs[2] default + random mask, configs[3],
#                                      literal 200^2 skip net, configs[1], native 36^2 (synthetic and the
#                                      reference's image), ES-on lines, torchrun N = 1)
#   tools/gpu.sh steptime SPEC...      DIP step-time A/B: SPEC = label[:ENV=V[,ENV=V...]][@args],
#                                      interleaved over $ROUNDS rounds (default 2); ENV LRSPNP_LIB=tune
#                                      selects the tuning build; args go to tools/dip_steptime.py
#   tools/gpu.sh host SPEC...          host enqueue vs GPU time per step (tools/host_enqueue.py)
#   tools/gpu.sh trace NAME CMD...     rocprofv3 kernel trace + stats of CMD into profiles-ready files
#   tools/gpu.sh pmc NAME CMD...       the HBM counter passes (FETCH_SIZE, WRITE_SIZE) of CMD
#   tools/gpu.sh profile               the round profile of the default (dip) and pnp bench commands:
#                                      kernel trace + stats, then separate FETCH_SIZE, WRITE_SIZE and SQ
#                                      passes, summarised on the box by tools/summarize_round.py into
#                                      $O/sum (copy to profiles/<round>/); WORKLOADS="dip pnp" default
# Every GPU step runs under its own timeout and the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=${OUT:-gpurun_out/run}
mkdir -p $O
T=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_tune.so
what=$1
shift

run_spec() {   # $1 = tool, $2 = spec
  local tool=$1 spec=$2 label envs args
  label=${spec%%[:@]*}
  envs=""
  args=""
  [[ $spec == *:* ]] && { envs=${spec#*:}; envs=${envs%%@*}; }
  [[ $spec == *@* ]] && args=${spec#*@}
  local -a ev=()
  IFS=',' read -ra kv <<< "$envs"
  for e in "${kv[@]}"; do
    [[ -z $e ]] && continue
    # LRSPNP_LIB=<v>: the build lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_<v>.so (tune = the tuning build)
    [[ $e == LRSPNP_LIB=* && $e != LRSPNP_LIB=/* ]] && e="LRSPNP_LIB=$PWD/lrs-pnp-dip_amd/lrspnp/liblrspnp_hip_${e#LRSPNP_LIB=}.so"
    ev+=("$e")
  done
  env "${ev[@]}" timeout -k 10 ${STEP_TIMEOUT:-200} python $tool $args > $O/spec.txt 2>&1 || { tail $O/spec.txt; return 1; }
  echo "$label: $(tail -${TAIL:-1} $O/spec.txt)"
}

case $what in
suite)
  timeout -k 10 ${SUITE_TIMEOUT:-560} python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 150 \
    --timeout-method thread -rA "$@" > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|assert" $O/pytest_gpu.log | head -30; tail -5 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
  tail -2 $O/smoke.log
  ;;
bench)
  line() {   # name, timeout, args...
    local n=$1 t=$2
    shift 2
    timeout -k 10 $t python bench.py "$@" > $O/$n.json 2> $O/$n.err || { tail $O/$n.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))"
  }
  line default 300
  line random_mask 300 --mask random --no-cpu-baseline
  line dip_pro 400 --workload dip-pro --steps 3 --warmup 1 --no-cpu-baseline
  line dip_pro_200 300 --workload dip-pro --cube 200x200x198 --steps 3 --warmup 1 --no-cpu-baseline
  line pnp 200 --workload pnp --steps 20 --warmup 3 --no-cpu-baseline
  line native36 300 --cube 36x36x128 --steps 20 --warmup 3 --no-cpu-baseline
  line native36_img 300 --data native --steps 20 --warmup 3 --no-cpu-baseline
  # early stopping on (the reference's real configuration): DIP steps to the stop per outer iteration
  line es_native 300 --data native --early-stop --steps 8 --warmup 1 --no-cpu-baseline
  line es196 600 --early-stop --steps 3 --warmup 1 --no-cpu-baseline
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > $O/torchrun_n1.json 2> $O/torchrun_n1.err || { tail -20 $O/torchrun_n1.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/torchrun_n1.json').read().strip().splitlines()[-1]); print('torchrun N=1', d['value'], d['ms_per_step'])"
  ;;
steptime|host)
  tool=tools/dip_steptime.py
  [[ $what == host ]] && { tool=tools/host_enqueue.py; TAIL=3; }
  for r in $(seq 1 ${ROUNDS:-2}); do
    for s in "$@"; do run_spec $tool "$s" || exit 1; done
  done
  ;;
trace)
  name=$1
  shift
  timeout -k 10 ${STEP_TIMEOUT:-300} rocprofv3 --kernel-trace --stats -d $O/trace_$name -o run --output-format csv -- "$@" > $O/trace_$name.log 2>&1 || { tail $O/trace_$name.log; exit 1; }
  find $O/trace_$name -name '*kernel_stats.csv' -exec cp {} $O/${name}_kernel_stats.csv \;
  find $O/trace_$name -name '*kernel_trace.csv' -exec cp {} $O/${name}_kernel_trace.csv \;
  ;;
pmc)
  name=$1
  shift
  timeout -s KILL ${STEP_TIMEOUT:-200} rocprofv3 --pmc FETCH_SIZE -d $O/pmc_${name}_f -o run --output-format csv -- "$@" > $O/pmc_${name}_f.log 2>&1 || { tail $O/pmc_${name}_f.log; exit 1; }
  timeout -s KILL ${STEP_TIMEOUT:-200} rocprofv3 --pmc WRITE_SIZE -d $O/pmc_${name}_w -o run --output-format csv -- "$@" > $O/pmc_${name}_w.log 2>&1 || { tail $O/pmc_${name}_w.log; exit 1; }
  find $O/pmc_${name}_f -name '*counter_collection.csv' -exec cp {} $O/${name}_fetch.csv \;
  find $O/pmc_${name}_w -name '*counter_collection.csv' -exec cp {} $O/${name}_write.csv \;
  ;;
profile)
  P=$O/profile
  mkdir -p $P
  for wl in ${WORKLOADS:-dip pnp}; do
    if [ $wl = pnp ]; then S="--steps 10 --warmup 2"; else S="--steps 3 --warmup 1"; fi
    B="bench.py --workload $wl $S --no-cpu-baseline"
    timeout -k 10 400 python bench.py --workload $wl $S > $P/${wl}_bench.json 2> $P/${wl}_bench.err || { tail $P/${wl}_bench.err; exit 1; }
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/${wl}_trace -o run --output-format csv -- python3 $B > $P/${wl}_trace.log 2>&1 || { tail $P/${wl}_trace.log; exit 1; }
    timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $P/${wl}_fetch -o run --output-format csv -- python3 $B > $P/${wl}_fetch.log 2>&1 || { tail $P/${wl}_fetch.log; exit 1; }
    timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $P/${wl}_write -o run --output-format csv -- python3 $B > $P/${wl}_write.log 2>&1 || { tail $P/${wl}_write.log; exit 1; }
    timeout -s KILL 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d $P/${wl}_sq -o run --output-format csv -- python3 $B > $P/${wl}_sq.log 2>&1 || { tail $P/${wl}_sq.log; exit 1; }
  done
  # summarised on the box (the raw per-dispatch CSVs exceed what gpurun copies back)
  python tools/summarize_round.py $P $O/sum > $P/summary.log 2>&1 || { cat $P/summary.log; exit 1; }
  rm -rf $P/*_trace $P/*_fetch $P/*_write $P/*_sq
  echo profile-ok
  ;;
*)
  echo "unknown purpose: $what" >&2
  exit 2
  ;;
esac
