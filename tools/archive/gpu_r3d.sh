#!/bin/bash
# round 3 gate on the current tree: GPU suite, smoke, default bench line (timed)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/r3d_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3d_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
s=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_bench.err
rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - s ))s"; exit $rc
