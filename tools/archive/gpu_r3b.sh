#!/bin/bash
# round 3: the default bench line (with the new runs / rebuild / churn-E / config-B legs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u bench.py > gpurun_out/r3b_bench.json 2> gpurun_out/r3b_bench.err
echo "bench rc=$?"
