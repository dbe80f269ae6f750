# Round-4 GPU pass m: the delta-vs-full image tests, pinned-buffer NUMA probe (config B with config C alive), and an
# aggregator sweep over delivery threads.
set -o pipefail
T=${1:-m}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_image.py -x > gpurun_out/pytest_image_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_image_$T.log; grep -E "FAILED|Error|assert" gpurun_out/pytest_image_$T.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_pinned_numa.py > gpurun_out/probe_pinned_numa_$T.jsonl 2> gpurun_out/probe_pinned_numa_$T.err
rc=$?; cat gpurun_out/probe_pinned_numa_$T.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/probe_pinned_numa_$T.err; exit $rc; }
PIN=1 timeout -k 10 300 python -u tools/batcher_gpu.py 65536:14:200:0:0:6:65536:2:6:0:8 65536:15:200:0:0:6:65536:2:6:0:8 \
    65536:16:200:0:0:6:65536:2:6:0:8 65536:15:200:0:1:6:65536:2:6:0:8 65536:14:100:0:0:6:65536:2:6:0:8 \
    65536:14:200:0:0:8:65536:2:6:0:8 > gpurun_out/batcher_$T.jsonl 2> gpurun_out/batcher_$T.err
rc=$?; cut -c1-330 gpurun_out/batcher_$T.jsonl; exit $rc
