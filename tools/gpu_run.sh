# GPU gate: GPU tests, smoke, default bench line.  Usage: bash tools/gpu_run.sh TAG [pytest -k expr]
set -o pipefail
T=${1:-x}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "${KARG[@]}" > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$T.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 && tail -n 2 gpurun_out/smoke_$T.log && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err && head -c 600 gpurun_out/bench_$T.json
