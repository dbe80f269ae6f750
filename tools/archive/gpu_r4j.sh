# Round-4 GPU pass j: churn trace (commit work pool, radix dirty lists, parallel list
# placement), the GPU suite, and config B's runs legs under a kernel + memory-copy trace.
set -o pipefail
T=${1:-j}
mkdir -p gpurun_out
EMQX_TM_COMMIT_TRACE=1 timeout -k 10 300 python -u bench.py --churn 5 --warmup 1 > gpurun_out/churn_E_$T.json 2> gpurun_out/churn_E_$T.err
rc=$?; grep "tm commit" gpurun_out/churn_E_$T.err | tail -4; head -c 700 gpurun_out/churn_E_$T.json; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -v --timeout 420 --timeout-method thread tests -m gpu -x > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$T.log | head -20
[ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/prof_B_$T -o b -- \
    python -u tools/probe_runs_order.py --skip-c > gpurun_out/probe_runs_order_$T.jsonl 2> gpurun_out/probe_runs_order_$T.err
rc=$?; cat gpurun_out/probe_runs_order_$T.jsonl; exit $rc
