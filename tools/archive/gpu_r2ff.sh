# round-2: return_first kernel — alive masks in registers, frontier capacity; sweep in FIRST mode + parity
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/sweep.py run --mode first --variants head base ff256 ff192 noalive_first > gpurun_out/sweep_r2ff.jsonl 2> gpurun_out/sweep_r2ff.err
rc=$?; cat gpurun_out/sweep_r2ff.jsonl; tail -n 3 gpurun_out/sweep_r2ff.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_reducers.py > gpurun_out/pytest_r2ff.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_r2ff.log; exit $rc
