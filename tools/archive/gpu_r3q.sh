#!/bin/bash
# round 3: host keys path (570 MB D2H per call) plain, with SDMA off (blit-kernel copies),
# and under rocprofv3 memory-copy tracing (where it measured 12.9 ms)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/prof_hostpath.py > gpurun_out/r3q_plain.log 2>&1
echo "plain rc=$?"
HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u tools/prof_hostpath.py > gpurun_out/r3q_nosdma.log 2>&1
echo "nosdma rc=$?"
