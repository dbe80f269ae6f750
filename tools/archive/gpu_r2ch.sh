# round-2: in-place list edits — churn/replica/ASan GPU tests, then config-E churn A/B (HEAD engine vs tree)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_replica.py tests/test_native_asan.py tests/test_gpu_reducers.py > gpurun_out/pytest_r2ch.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_r2ch.log; [ $rc -eq 0 ] || exit $rc
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_headeng.so timeout -k 10 400 python -u bench.py --churn 15 > gpurun_out/churn_head.json 2> gpurun_out/churn_head.err || exit $?
timeout -k 10 400 python -u bench.py --churn 15 > gpurun_out/churn_tree.json 2> gpurun_out/churn_tree.err || exit $?
head -c 1200 gpurun_out/churn_head.json; echo; head -c 1200 gpurun_out/churn_tree.json
