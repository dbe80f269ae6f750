set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_filter.log 2>&1 && tail -3 gpurun_out/pytest_filter.log && \
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_t.log 2>&1 ; rc=$?; tail -3 gpurun_out/pytest_filter.log gpurun_out/pytest_gpu_t.log; exit $rc
