# Round-4 GPU pass l: the default bench line, smoke, and an aggregator sweep.
set -o pipefail
T=${1:-l}
mkdir -p gpurun_out
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; head -c 400 gpurun_out/bench_$T.json; echo; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$T.err; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; tail -3 gpurun_out/smoke_$T.log; [ $rc -eq 0 ] || exit $rc
PIN=1 timeout -k 10 300 python -u tools/batcher_gpu.py 65536:14:200:0:0:6:65536:2:6:0:8 65536:14:200:0:1:6:65536:2:6:0:8 \
    65536:14:200:0:3:6:65536:2:6:0:4 65536:14:200:0:2:6:65536:2:6:0:8 65536:13:200:0:1:6:65536:2:6:0:8 \
    > gpurun_out/batcher_$T.jsonl 2> gpurun_out/batcher_$T.err
rc=$?; cut -c1-330 gpurun_out/batcher_$T.jsonl; exit $rc
