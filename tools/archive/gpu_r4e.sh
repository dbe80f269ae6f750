# Round-4 GPU pass e: probes (runs pinned/pageable on config B; batcher delivery prefetch;
# topic grouping for k_match_fast), the churn leg (commit phases), the 2-rank sharded rehearsal.
set -o pipefail
T=${1:-e}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_concurrency.py -m gpu \
    > gpurun_out/pytest_conc_$T.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_conc_$T.log; grep -E "FAILED|form:" gpurun_out/pytest_conc_$T.log | head -5
timeout -k 10 300 python -u tools/probe_runs_pinned.py --config B > gpurun_out/probe_runs_B_$T.jsonl 2> gpurun_out/probe_runs_B_$T.err
rc=$?; cat gpurun_out/probe_runs_B_$T.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_sorted.py > gpurun_out/probe_sorted_$T.jsonl 2> gpurun_out/probe_sorted_$T.err
rc=$?; cat gpurun_out/probe_sorted_$T.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/probe_sorted_$T.err; exit $rc; }
PIN=1 timeout -k 10 300 python -u tools/batcher_gpu.py 65536:13:200:0:0 65536:13:200:0:1 65536:13:200:0:2 \
    65536:13:200:0:1:6:65536:2:6:16 65536:13:200:0:1:6:65536:2:12:32 65536:13:200:0:0:6:65536:2:6:16 \
    65536:13:200:0:0:6:65536:2:12:32 65536:14:200:0:0 65536:15:200:0:0 65536:14:200:0:1 > gpurun_out/batcher_pf_$T.jsonl 2> gpurun_out/batcher_pf_$T.err
rc=$?; cat gpurun_out/batcher_pf_$T.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --churn 5 --warmup 1 > gpurun_out/churn_E_$T.json 2> gpurun_out/churn_E_$T.err
rc=$?; head -c 900 gpurun_out/churn_E_$T.json; echo; [ $rc -eq 0 ] || exit $rc
EMQX_BENCH_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --mode sharded --config D --scale 0.25 \
    --steps 20 --warmup 3 > gpurun_out/bench_D_gloo2_$T.json 2> gpurun_out/bench_D_gloo2_$T.err
rc=$?; tail -n 5 gpurun_out/bench_D_gloo2_$T.err; head -c 1500 gpurun_out/bench_D_gloo2_$T.json; echo
exit $rc
