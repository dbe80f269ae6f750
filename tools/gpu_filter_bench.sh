set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_filter.log 2>&1 && tail -n 2 gpurun_out/pytest_filter.log && \
timeout -k 10 400 python -u bench.py --filter-search 100000 > gpurun_out/bench_filter.json 2> gpurun_out/bench_filter.err && cat gpurun_out/bench_filter.json && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_filter -o prof -- python3 -u bench.py --filter-search 100000 --steps 5 --warmup 1 > gpurun_out/prof_filter.log 2>&1
rc=$?; tail -n 2 gpurun_out/pytest_filter.log; exit $rc
