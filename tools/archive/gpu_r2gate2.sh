# round-2 gate after the DPP scans: all GPU tests, smoke, default bench line, trace + PMC passes
set -o pipefail
bash tools/gpu_run.sh r2h || exit $?
bash tools/prof_pmc.sh gpurun_out/prof_r2h
