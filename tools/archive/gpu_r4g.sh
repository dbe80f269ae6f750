# Round-4 GPU pass g: churn trace (huge pages, staged scatters), the GPU suite, the B-order
# probe, and the PMC passes of the final kernel source (tools/prof_pmc.sh).
set -o pipefail
T=${1:-g}
mkdir -p gpurun_out
EMQX_TM_COMMIT_TRACE=1 timeout -k 10 300 python -u bench.py --churn 5 --warmup 1 > gpurun_out/churn_E_$T.json 2> gpurun_out/churn_E_$T.err
rc=$?; grep "tm commit" gpurun_out/churn_E_$T.err | tail -6; head -c 500 gpurun_out/churn_E_$T.json; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -v --timeout 420 --timeout-method thread tests -m gpu -x > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error|form:" gpurun_out/pytest_gpu_$T.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_runs_order.py > gpurun_out/probe_runs_order_$T.jsonl 2> gpurun_out/probe_runs_order_$T.err
rc=$?; cat gpurun_out/probe_runs_order_$T.jsonl; [ $rc -eq 0 ] || { tail -3 gpurun_out/probe_runs_order_$T.err; exit $rc; }
bash tools/prof_pmc.sh gpurun_out/prof_$T > gpurun_out/prof_$T.log 2>&1
rc=$?; tail -3 gpurun_out/prof_$T.log
exit $rc
