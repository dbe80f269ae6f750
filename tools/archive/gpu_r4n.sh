# Round-4 GPU pass n: pinned-buffer order probe, the default bench line (15 delivery threads),
# and the 2-rank sharded (config D) rehearsal over gloo for its host RSS without the slot-table mirror.
set -o pipefail
T=${1:-n}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_pinned_numa.py --order hipHostMalloc,torch_pin_memory,pageable --rounds 2 --reps 8 \
    > gpurun_out/probe_pinned_numa_$T.jsonl 2> gpurun_out/probe_pinned_numa_$T.err
rc=$?; cut -c1-300 gpurun_out/probe_pinned_numa_$T.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/probe_pinned_numa_$T.err; exit $rc; }
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; head -c 300 gpurun_out/bench_$T.json; echo; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$T.err; exit $rc; }
EMQX_BENCH_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --mode sharded --config D --scale 0.25 \
    --steps 20 --warmup 3 > gpurun_out/bench_D_gloo2_$T.json 2> gpurun_out/bench_D_gloo2_$T.err
rc=$?; tail -n 3 gpurun_out/bench_D_gloo2_$T.err; head -c 800 gpurun_out/bench_D_gloo2_$T.json; echo
exit $rc
