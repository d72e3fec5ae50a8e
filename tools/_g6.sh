set -o pipefail
export OUT=gpurun_out/g6 TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 120 tools/micro/fork_cost 200 > $OUT/fork_cost.txt 2>&1 || echo "fork_cost failed"
cat $OUT/fork_cost.txt
ROUNDS=2 tools/gpu.sh steptime "u196_r04:LRSPNP_LIB=r04@--rounds 3" "u196@--rounds 3" "u196_t:LRSPNP_LIB=tune@--rounds 3" "u196_t_off:LRSPNP_LIB=tune,LRS_DIP_BN1_SMALL=0,LRS_DIP_SN_OVERLAP=0@--rounds 3" "u196_A_off:LRSPNP_LIB=tuneA,LRS_DIP_BN1_SMALL=0,LRS_DIP_SN_OVERLAP=0@--rounds 3" "u196_A:LRSPNP_LIB=tuneA@--rounds 3" "u36_r04:LRSPNP_LIB=r04@--hw 36 --bands 128 --rounds 3" "u36@--hw 36 --bands 128 --rounds 3" "u36_t_off:LRSPNP_LIB=tune,LRS_DIP_BN1_SMALL=0@--hw 36 --bands 128 --rounds 3" "u36_A_off:LRSPNP_LIB=tuneA,LRS_DIP_BN1_SMALL=0@--hw 36 --bands 128 --rounds 3" "u36_A:LRSPNP_LIB=tuneA@--hw 36 --bands 128 --rounds 3"
