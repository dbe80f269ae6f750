#!/bin/bash
# round 3: the N>1 path rehearsed on one GPU: 2 ranks over gloo (master + replica), two
# batches in flight per rank
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
EMQX_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 30 --warmup 3 > gpurun_out/r3g2_bench.json 2> gpurun_out/r3g2_bench.err
echo "gloo2 rc=$?"
