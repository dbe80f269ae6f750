#!/bin/bash
# round 3: same-process A/B of k_match_fast before / after the fused-id copy-out (config C)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u tools/sweep.py run --variants prev base prev base2 --steps 20 > gpurun_out/r3g_sweep.jsonl 2> gpurun_out/r3g_sweep.err
echo "sweep rc=$?"
