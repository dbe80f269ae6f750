#!/bin/bash
# round 3: mode 1 over gloo with real engines (two processes on the one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_replica.py > gpurun_out/r3t_replica.log 2>&1
echo "replica rc=$?"
