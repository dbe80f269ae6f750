#!/bin/bash
# round 3: kernel trace + stats of the default step loop (two batches in flight)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3pp -o two -- python3 -u bench.py --quick --steps 50 > gpurun_out/r3pp_bench.json 2> gpurun_out/r3pp_bench.err
echo "prof rc=$?"
