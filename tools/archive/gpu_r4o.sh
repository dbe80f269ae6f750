# Round-4 GPU pass o: the first-calls slowdown of a second engine (hardware queues shared by
# more streams than GPU_MAX_HW_QUEUES?), the churn trace with the known-kind apply path, and
# the churn / image tests.
set -o pipefail
T=${1:-o}
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u tools/probe_pinned_numa.py --order hipHostMalloc,torch_pin_memory --reps 8 \
    > gpurun_out/probe_hwq16_$T.jsonl 2> gpurun_out/probe_hwq16_$T.err
rc=$?; cut -c1-300 gpurun_out/probe_hwq16_$T.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/probe_hwq16_$T.err; exit $rc; }
timeout -k 10 300 python -u tools/probe_pinned_numa.py --order hipHostMalloc,torch_pin_memory --reps 8 --release-c-lane \
    > gpurun_out/probe_hwq8_rel_$T.jsonl 2> gpurun_out/probe_hwq8_rel_$T.err
rc=$?; cut -c1-300 gpurun_out/probe_hwq8_rel_$T.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/probe_hwq8_rel_$T.err; exit $rc; }
EMQX_TM_COMMIT_TRACE=1 timeout -k 10 300 python -u bench.py --churn 5 --warmup 1 > gpurun_out/churn_E_$T.json 2> gpurun_out/churn_E_$T.err
rc=$?; grep "tm commit" gpurun_out/churn_E_$T.err | tail -3; head -c 500 gpurun_out/churn_E_$T.json; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -v --timeout 420 --timeout-method thread tests/test_gpu_image.py tests/test_gpu_fullsize.py -k "image or config_e" -x > gpurun_out/pytest_churn_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_churn_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_churn_$T.log | head; exit $rc
