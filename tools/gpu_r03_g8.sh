set -o pipefail
mkdir -p gpurun_out
bash tools/ab_steptime.sh "LRS_DIP_X=0" "LRS_DIP_FWD_SPLIT_WG=256" "LRS_DIP_FWD_SPLIT_WG=512" "LRS_DIP_SM_WG=448" "LRS_DIP_SM_WG=896" "LRS_DIP_PREP_WG=256" || exit 1
STEP_ARGS="--hw 36 --bands 128" bash tools/ab_steptime.sh "LRS_DIP_X=0" "LRS_DIP_SM_WG=448" "LRS_DIP_SM_WG=896" "LRS_DIP_SM_WG=320" || exit 1
