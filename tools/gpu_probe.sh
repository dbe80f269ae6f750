#!/bin/bash
# round 3: aggregator A/B, one vs two compute streams, same process and box, pinned
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
S=""
for rep in 1 2; do
  for st in 1 2; do
    S="$S 65536:13:200:0:0:6:65536:$st 65536:13:200:0:1:6:65536:$st 65536:13:200:1:0:6:65536:$st"
  done
done
PIN=1 GPU_MAX_HW_QUEUES=8 timeout -k 10 500 python -u tools/batcher_gpu.py $S > gpurun_out/r3ab.jsonl 2> gpurun_out/r3ab.err
echo "ab rc=$?"
