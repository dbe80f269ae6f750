# Round-4 GPU pass f: native vs Python-thread host calls, commit sub-phases (churn trace),
# the default bench line (distinct batches per step).
set -o pipefail
T=${1:-f}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_batcher.py -m gpu > gpurun_out/pytest_batcher_$T.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_batcher_$T.log; grep -E "FAILED" gpurun_out/pytest_batcher_$T.log | head -5; [ $rc -eq 0 ] || exit $rc
PIN=1 timeout -k 10 300 python -u tools/batcher_gpu.py 65536:14:200:0:0:6:65536:2:6:0:8 65536:14:200:0:0:6:65536:2:6:0:4 \
    65536:14:200:0:1:6:65536:2:6:0:8 65536:14:200:0:1:6:65536:2:6:0:4 65536:14:200:0:3:6:65536:2:6:0:4 \
    65536:14:200:0:4:6:65536:2:6:0:4 > gpurun_out/batcher_idw_$T.jsonl 2> gpurun_out/batcher_idw_$T.err
rc=$?; cat gpurun_out/batcher_idw_$T.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/probe_host_concurrency.py --form runs --threads 1,4 --native > gpurun_out/probe_conc_$T.jsonl 2> gpurun_out/probe_conc_$T.err
rc=$?; cat gpurun_out/probe_conc_$T.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/probe_conc_$T.err; exit $rc; }
timeout -k 10 200 python -u tools/probe_host_concurrency.py --form keys --threads 1,4 --native >> gpurun_out/probe_conc_$T.jsonl 2>> gpurun_out/probe_conc_$T.err
rc=$?; tail -4 gpurun_out/probe_conc_$T.jsonl; [ $rc -eq 0 ] || exit $rc
EMQX_TM_COMMIT_TRACE=1 timeout -k 10 300 python -u bench.py --churn 5 --warmup 1 > gpurun_out/churn_E_$T.json 2> gpurun_out/churn_E_$T.err
rc=$?; grep "tm commit" gpurun_out/churn_E_$T.err | tail -8; head -c 600 gpurun_out/churn_E_$T.json; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; tail -n 3 gpurun_out/bench_$T.err; head -c 700 gpurun_out/bench_$T.json; echo
exit $rc
