# Round-4 GPU gate pass: the GPU suite, the default bench line, smoke.
set -o pipefail
T=${1:-p}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 420 --timeout-method thread tests -m gpu -x > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$T.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; head -c 300 gpurun_out/bench_$T.json; echo; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$T.err; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; tail -3 gpurun_out/smoke_$T.log; exit $rc
