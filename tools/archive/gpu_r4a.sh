# Round-4 GPU pass: new tests first, the GPU suite, smoke, a 2-rank bench rehearsal (gloo, one
# GPU), then the default N=1 bench line.  Usage: bash tools/gpu_r4a.sh TAG
set -o pipefail
T=${1:-a}
mkdir -p gpurun_out
PT="python -u -m pytest -v --timeout 200 --timeout-method thread"
timeout -k 10 400 $PT tests -m gpu -k "failed_runs_call or commit_from_delivery or real_engines or gpu_batcher" \
    > gpurun_out/pytest_new_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_new_$T.log; grep -E "FAILED|Error|error" gpurun_out/pytest_new_$T.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 $PT tests -m gpu -x > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$T.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 && tail -n 2 gpurun_out/smoke_$T.log || exit 1
EMQX_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 20 --warmup 5 \
    > gpurun_out/bench_gloo2_$T.json 2> gpurun_out/bench_gloo2_$T.err
rc=$?; tail -n 5 gpurun_out/bench_gloo2_$T.err; head -c 400 gpurun_out/bench_gloo2_$T.json; echo
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; tail -n 3 gpurun_out/bench_$T.err; head -c 600 gpurun_out/bench_$T.json; echo
exit $rc
