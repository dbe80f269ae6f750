# round 2: batcher pipeline + one-pass filter walk: their GPU tests, then the default bench
set -o pipefail
mkdir -p gpurun_out
T=${1:-r2d}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "batcher or filter or asan or nif" > gpurun_out/pytest_${T}.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_${T}.log; grep -E "FAILED|Error" gpurun_out/pytest_${T}.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err
rc=$?; head -c 300 gpurun_out/bench_${T}.json; echo; tail -n 3 gpurun_out/bench_${T}.err; exit $rc
