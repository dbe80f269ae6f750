#!/bin/bash
# round 3: two direct buffer sets in flight with more hardware queues per process
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python -u bench.py --quick > gpurun_out/r3y_bench.json 2> gpurun_out/r3y_bench.err
echo "bench rc=$?"
