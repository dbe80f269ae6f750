# round-2: new occupancy defaults — sweep vs HEAD, then all GPU tests, smoke, bench, trace + PMC
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_sweep.sh r2sw3 head base w20 f416 s96 noalive || exit $?
bash tools/gpu_run.sh r2i || exit $?
bash tools/prof_pmc.sh gpurun_out/prof_r2i
