#!/bin/bash
# round 3: RCCL (nccl backend) at world size 1 on the real device
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu tests/test_gpu_rccl.py > gpurun_out/r3s_rccl.log 2>&1
echo "rccl rc=$?"
