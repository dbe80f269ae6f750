# Round-4 GPU pass b: the GPU suite (host paths rewritten for concurrent readers), the runs
# pinned/pageable probe on config B, and a 2-rank sharded (config D) rehearsal over gloo.
set -o pipefail
T=${1:-b}
mkdir -p gpurun_out
PT="python -u -m pytest -v --timeout 240 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_concurrency.py -m gpu > gpurun_out/pytest_conc_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_conc_$T.log; grep -E "FAILED|Error|one thread" gpurun_out/pytest_conc_$T.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 $PT tests -m gpu -x > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$T.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/probe_runs_pinned.py --config B > gpurun_out/probe_runs_B_$T.jsonl 2> gpurun_out/probe_runs_B_$T.err
rc=$?; cat gpurun_out/probe_runs_B_$T.jsonl; [ $rc -eq 0 ] || exit $rc
PIN=1 timeout -k 10 300 python -u tools/batcher_gpu.py 65536:13:200:0:0 65536:13:200:0:1 65536:13:200:0:2 \
    65536:13:200:0:1:6:65536:2:6:16 65536:13:200:0:1:6:65536:2:12:32 65536:13:200:0:0:6:65536:2:6:16 \
    65536:13:200:0:0:6:65536:2:12:32 > gpurun_out/batcher_pf_$T.jsonl 2> gpurun_out/batcher_pf_$T.err
rc=$?; cat gpurun_out/batcher_pf_$T.jsonl; [ $rc -eq 0 ] || exit $rc
EMQX_BENCH_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --mode sharded --config D --scale 0.25 \
    --steps 20 --warmup 3 > gpurun_out/bench_D_gloo2_$T.json 2> gpurun_out/bench_D_gloo2_$T.err
rc=$?; tail -n 5 gpurun_out/bench_D_gloo2_$T.err; head -c 1500 gpurun_out/bench_D_gloo2_$T.json; echo
exit $rc
