set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_sweep.sh r2lz head base eagerfnv || exit $?
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_reducers.py > gpurun_out/pytest_r2lz.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_r2lz.log; exit $rc
