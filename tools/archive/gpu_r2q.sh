# round-2: TM_PRELOOK=10 default — same-process sweep vs HEAD, all GPU tests, smoke, bench
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_sweep.sh r2q head base base2 nopre || exit $?
bash tools/gpu_run.sh r2q
