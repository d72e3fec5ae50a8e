#!/bin/bash
# rocprofv3 kernel stats of DIP training steps (196x196x198, graph off) -> gpurun_out/prof_dip
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dip -o dip --output-format csv -- python3 tools/diag_dip.py ${1:-198} ${2:-196} ${3:-20} 0
find gpurun_out/prof_dip -name "*kernel_stats.csv" | head -3
