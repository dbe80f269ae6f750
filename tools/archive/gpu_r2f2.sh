# round-2: matches_filter/3 at config C, 100K queries: GPU filter tests, bench line, kernel trace,
# FETCH/WRITE passes.  Usage: bash tools/gpu_r2f2.sh TAG
set -o pipefail
T=${1:-f}
O=gpurun_out/prof_filter_$T
mkdir -p $O/trace
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_filter.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_filter_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_filter_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --filter-search 100000 > gpurun_out/bench_filter_$T.json 2> gpurun_out/bench_filter_$T.err && head -c 1500 gpurun_out/bench_filter_$T.json && \
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 -u bench.py --filter-search 100000 --steps 3 --warmup 1 > $O/trace.log 2>&1 && \
bash tools/prof_filter_pmc.sh $O
