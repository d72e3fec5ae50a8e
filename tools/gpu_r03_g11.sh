set -o pipefail
mkdir -p gpurun_out/r03
# SVT eigensolver phase times on the configs[1] cube (one workgroup, isolated and synchronised)
timeout -k 10 300 python -u tools/diag_svt.py 200x200x198 3 > gpurun_out/r03/svt_phases.txt 2>&1 || { tail -20 gpurun_out/r03/svt_phases.txt; exit 1; }
cat gpurun_out/r03/svt_phases.txt
