# Round-4 GPU pass k: churn trace (pre-interned new words, contiguous parallel ranges, radix
# delta sort) and the GPU suite.
set -o pipefail
T=${1:-k}
mkdir -p gpurun_out
EMQX_TM_COMMIT_TRACE=1 timeout -k 10 300 python -u bench.py --churn 5 --warmup 1 > gpurun_out/churn_E_$T.json 2> gpurun_out/churn_E_$T.err
rc=$?; grep "tm commit" gpurun_out/churn_E_$T.err | tail -4; head -c 700 gpurun_out/churn_E_$T.json; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -v --timeout 420 --timeout-method thread tests -m gpu -x > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$T.log | head -20
exit $rc
