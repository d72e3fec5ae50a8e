#!/bin/bash
# GPU box: DIP workload benches (configs[2], configs[3]) and their kernel-trace profiles.
# Output: gpurun_out/profile_dip/{dip,dip_pro}.json and {dip,dip_pro}_trace/ (copied into
# profiles/<tag>/ by the caller).
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/profile_dip
mkdir -p $out
timeout -k 10 300 python bench.py --workload dip --steps 3 --warmup 1 > $out/dip.json 2> $out/dip.err || { echo dip bench failed; tail $out/dip.err; exit 1; }
timeout -k 10 400 python bench.py --workload dip-pro --steps 2 --warmup 1 --no-cpu-baseline > $out/dip_pro.json 2> $out/dip_pro.err || { echo dip-pro bench failed; tail $out/dip_pro.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/dip_trace -o run --output-format csv -- python bench.py --workload dip --steps 2 --warmup 1 --no-cpu-baseline > $out/dip_prof.json 2> $out/dip_prof.err || { echo dip prof failed; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/dip_pro_trace -o run --output-format csv -- python bench.py --workload dip-pro --steps 1 --warmup 1 --no-cpu-baseline > $out/dip_pro_prof.json 2> $out/dip_pro_prof.err || { echo dip-pro prof failed; exit 1; }
echo all-ok
