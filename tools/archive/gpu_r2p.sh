# round-2: pre-scan word lookups (TM_PRELOOK) — sweep, then parity tests on the pre10 build
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_sweep.sh r2p base base2 pre8 pre10 pre12 || exit $?
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_pre10.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py > gpurun_out/pytest_r2p.log 2>&1
rc=$?; tail -n 5 gpurun_out/pytest_r2p.log; exit $rc
