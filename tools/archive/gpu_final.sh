set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_y.log 2>&1 && tail -n 1 gpurun_out/pytest_gpu_y.log && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_y.log 2>&1 && tail -n 2 gpurun_out/smoke_y.log && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench_y.json 2> gpurun_out/bench_y.err && head -c 400 gpurun_out/bench_y.json
