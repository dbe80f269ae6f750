# round-2 check: new GPU tests, the LDS sweep, batcher + host-path timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py::test_host_batch_pipelined_vs_oracle tests/test_gpu_filter.py::test_topic_index_word_list_topics \
    tests/test_batcher.py tests/test_nif_sequence.py > gpurun_out/pytest_r2n.log 2>&1
rc=$?; tail -n 5 gpurun_out/pytest_r2n.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_sweep.sh r2n base tb2560_f448 tb2048_f512 tb2304_f480 tb2048_f576 tb1792_f544 || exit $?
HOSTPATH=1 bash tools/gpu_batcher.sh r2n 65536:13:200 65536:14:200 65536:13:100 262144:13:200 4096:13:200 65536:8:200
