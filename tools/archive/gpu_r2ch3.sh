set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_replica.py tests/test_native_asan.py tests/test_shard.py > gpurun_out/pytest_r2ch3.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_r2ch3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --churn 15 > gpurun_out/churn_tree3.json 2> gpurun_out/churn_tree3.err || exit $?
cat gpurun_out/churn_tree3.json
