set -o pipefail
# DIP step-time A/B of environment settings (tuning knobs), interleaved: ab_env.sh "VAR=a" "VAR=b" ...
for rnd in 1 2 3; do
for v in "$@"; do
  echo -n "$v: "
  env $v timeout -k 10 120 python tools/dip_steptime.py --rounds 5 || exit 1
done
done
