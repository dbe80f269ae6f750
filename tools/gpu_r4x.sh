# Round-4 GPU pass x: the GPU suite with the replica runs form, then a replica aggregator sweep.
set -o pipefail
T=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 420 --timeout-method thread tests -m gpu -x > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$T.log | head -20; exit $rc
