# round-2 gate: all GPU tests, smoke, default bench line, then kernel trace + PMC passes
set -o pipefail
bash tools/gpu_run.sh r2g || exit $?
bash tools/prof_pmc.sh gpurun_out/prof_r2g
