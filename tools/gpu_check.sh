set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_s.log 2>&1 && tail -3 gpurun_out/pytest_gpu_s.log && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench_s.json 2> gpurun_out/bench_s.err && cat gpurun_out/bench_s.json | head -c 600
