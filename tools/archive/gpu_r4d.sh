# Round-4 GPU pass d: concurrency tests + probe, then the whole GPU suite.
set -o pipefail
T=${1:-d}
mkdir -p gpurun_out
PT="python -u -m pytest -v -s --timeout 300 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_concurrency.py -m gpu > gpurun_out/pytest_conc_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_conc_$T.log; grep -E "FAILED|Error|form:" gpurun_out/pytest_conc_$T.log | head -20
timeout -k 10 200 python -u tools/probe_host_concurrency.py --form runs > gpurun_out/probe_conc_$T.jsonl 2> gpurun_out/probe_conc_$T.err && \
timeout -k 10 200 python -u tools/probe_host_concurrency.py --form runs --pinned >> gpurun_out/probe_conc_$T.jsonl 2>> gpurun_out/probe_conc_$T.err && \
timeout -k 10 200 python -u tools/probe_host_concurrency.py --form keys >> gpurun_out/probe_conc_$T.jsonl 2>> gpurun_out/probe_conc_$T.err
rc2=$?; cat gpurun_out/probe_conc_$T.jsonl; [ $rc2 -eq 0 ] || exit $rc2
timeout -k 10 900 python -u -m pytest -v --timeout 420 --timeout-method thread tests -m gpu -x > gpurun_out/pytest_gpu_$T.log 2>&1
rc3=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$T.log | head -20
[ $rc3 -eq 0 ] || exit $rc3
exit $rc
