# round-2: result-ids kernel + batcher slots
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_reducers.py tests/test_batcher.py tests/test_shard.py tests/test_replica.py > gpurun_out/pytest_r2o.log 2>&1
rc=$?; tail -n 5 gpurun_out/pytest_r2o.log; [ $rc -eq 0 ] || exit $rc
HOSTPATH=1 bash tools/gpu_batcher.sh r2o 65536:13:200 65536:14:200 262144:13:200 4096:13:200 || exit $?
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_nslot4.so bash tools/gpu_batcher.sh r2o4 65536:13:200 65536:14:200 262144:13:200 4096:13:200
