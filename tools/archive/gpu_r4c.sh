# Round-4 GPU pass c: host-form concurrency probe (plain and under rocprofv3 runtime trace),
# the GPU suite minus the overlap test, runs pinned/pageable probe, batcher prefetch sweep,
# 2-rank sharded (config D) rehearsal over gloo.
set -o pipefail
T=${1:-c}
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/probe_host_concurrency.py --form runs > gpurun_out/probe_conc_$T.jsonl 2> gpurun_out/probe_conc_$T.err
rc=$?; cat gpurun_out/probe_conc_$T.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/probe_conc_$T.err; exit $rc; }
timeout -k 10 200 python -u tools/probe_host_concurrency.py --form keys >> gpurun_out/probe_conc_$T.jsonl 2>> gpurun_out/probe_conc_$T.err
rc=$?; tail -2 gpurun_out/probe_conc_$T.jsonl; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --runtime-trace --kernel-trace --stats -d gpurun_out/prof_conc_$T -o conc -- \
    python3 -u tools/probe_host_concurrency.py --form runs --threads 1,4 --reps 4 > gpurun_out/probe_conc_prof_$T.log 2>&1
rc=$?; tail -3 gpurun_out/probe_conc_prof_$T.log; [ $rc -eq 0 ] || exit $rc
PT="python -u -m pytest -v --timeout 240 --timeout-method thread"
timeout -k 10 800 $PT tests -m gpu -x -k "not host_form_readers_overlap" > gpurun_out/pytest_gpu_$T.log 2>&1
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
