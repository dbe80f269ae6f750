set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_sweep.sh r2sw head base alive rpl3 tb2048_f384 tb2048_f352 alive_tb2048_f384 || exit $?
bash tools/gpu_r2f3.sh iws
