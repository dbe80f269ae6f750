# round 2: batcher/NIF/filter tests, default bench, then a k_match_fast variant sweep
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_r2d.sh r2e || exit $?
timeout -k 10 500 python -u tools/sweep.py run --variants base nt rpl3 nt16 > gpurun_out/sweep_r2e.jsonl 2> gpurun_out/sweep_r2e.err
rc=$?; cat gpurun_out/sweep_r2e.jsonl; tail -n 3 gpurun_out/sweep_r2e.err; exit $rc
