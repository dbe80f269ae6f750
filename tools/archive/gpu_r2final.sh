# round-2 final tree: all GPU tests, smoke, default bench line, trace + PMC passes, churn line
set -o pipefail
bash tools/gpu_run.sh r2z || exit $?
bash tools/prof_pmc.sh gpurun_out/prof_r2z || exit $?
timeout -k 10 400 python -u bench.py --churn 15 > gpurun_out/churn_r2z.json 2> gpurun_out/churn_r2z.err && head -c 700 gpurun_out/churn_r2z.json
