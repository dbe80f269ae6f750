# round-2: rehearse the N>1 bench path (replicated mode: master + read replica via image broadcast)
# with 2 ranks on the one GPU over gloo, full config C
set -o pipefail
mkdir -p gpurun_out
export EMQX_BENCH_BACKEND=gloo
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err
rc=$?; tail -n 5 gpurun_out/bench_gloo2.err; head -c 2500 gpurun_out/bench_gloo2.json; exit $rc
