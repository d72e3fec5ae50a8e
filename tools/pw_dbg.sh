set -o pipefail
for d in 0 1 2 4 3 7; do echo "dbg $d"; LRS_PW_DBG=$d timeout -k 10 60 python tools/micro_conv.py 128 198 196 196 1 1 0 0 --reps 20 || exit 1; done
