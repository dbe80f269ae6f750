#!/bin/bash
# round 3: config D, one full-size shard of 8, with this round's tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u bench.py --mode sharded --config D --shard-of 8 --steps 50 > gpurun_out/r3_D.json 2> gpurun_out/r3_D.err
echo "D rc=$?"
