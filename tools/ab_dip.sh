set -o pipefail
# DIP step-time A/B of library builds tools/ab/lib_*.so, interleaved
for rnd in 1 2 3; do
for v in "$@"; do
  echo -n "$v: "
  LRSPNP_LIB=$PWD/tools/ab/lib_$v.so timeout -k 10 120 python tools/dip_steptime.py --rounds 5 || exit 1
done
done
