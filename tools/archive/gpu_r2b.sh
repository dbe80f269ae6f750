# round 2: replica + sharded step + config D tests; gloo rehearsal of the mode-1 bench; D shard bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_replica.py tests/test_shard.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "replica or shard or config_d or filter_kats or router_kats" > gpurun_out/pytest_r2b.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_r2b.log; grep -E "FAILED|Error" gpurun_out/pytest_r2b.log | head -20
[ $rc -eq 0 ] || exit $rc
EMQX_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 --scale 0.1 --batcher-seconds 0 > gpurun_out/bench_r2b_gloo2.json 2> gpurun_out/bench_r2b_gloo2.err
rc=$?; tail -c 1500 gpurun_out/bench_r2b_gloo2.json; tail -n 5 gpurun_out/bench_r2b_gloo2.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --mode sharded --config D --shard-of 8 --steps 20 --warmup 3 > gpurun_out/bench_r2b_D.json 2> gpurun_out/bench_r2b_D.err
rc=$?; cat gpurun_out/bench_r2b_D.json; tail -n 3 gpurun_out/bench_r2b_D.err; exit $rc
