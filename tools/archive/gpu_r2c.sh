# round 2: targeted tests (FIRST wave kernel, replicas, shards, config D), full GPU suite, default bench,
# gloo rehearsal of the mode-1 bench, config-D shard bench
set -o pipefail
mkdir -p gpurun_out
T=${1:-r2c}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "first or replica or shard or config_d" > gpurun_out/pytest_${T}_a.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_${T}_a.log; grep -E "FAILED|Error" gpurun_out/pytest_${T}_a.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "not (first or replica or shard or config_d)" > gpurun_out/pytest_${T}_b.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_${T}_b.log; grep -E "FAILED|Error" gpurun_out/pytest_${T}_b.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err
rc=$?; head -c 700 gpurun_out/bench_${T}.json; echo; tail -n 3 gpurun_out/bench_${T}.err
[ $rc -eq 0 ] || exit $rc
EMQX_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --scale 0.1 --batcher-seconds 0 > gpurun_out/bench_${T}_gloo2.json 2> gpurun_out/bench_${T}_gloo2.err
rc=$?; tail -c 600 gpurun_out/bench_${T}_gloo2.json; tail -n 5 gpurun_out/bench_${T}_gloo2.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode sharded --config D --shard-of 8 --steps 20 --warmup 3 > gpurun_out/bench_${T}_D.json 2> gpurun_out/bench_${T}_D.err
rc=$?; cat gpurun_out/bench_${T}_D.json; tail -n 3 gpurun_out/bench_${T}_D.err; exit $rc
