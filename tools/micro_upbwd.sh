set -o pipefail
# up_4 / up_3 data gradient (+ weight gradient) alone: the effective-kernel path
timeout -k 10 60 python tools/micro_conv.py 128 128 98 98 3 1 1 1 --bwd --reps 20 || exit 1
timeout -k 10 60 python tools/micro_conv.py 128 128 49 49 3 1 1 1 --bwd --reps 20 || exit 1
