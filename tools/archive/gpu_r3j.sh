#!/bin/bash
# round 3: non-temporal deep probes A/B (same process) + where the keys host path spends its time
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 700 python -u tools/sweep.py run --variants base ntd2 ntd3 ntd4 base ntd3 --steps 20 > gpurun_out/r3j_sweep.jsonl 2> gpurun_out/r3j_sweep.err
echo "sweep rc=$?"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r3j_host -o host -- python3 -u tools/prof_hostpath.py > gpurun_out/r3j_host.log 2>&1
echo "host prof rc=$?"
