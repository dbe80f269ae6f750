set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_u.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_u.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_u.log | head -20; exit $rc
