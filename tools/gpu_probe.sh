#!/bin/bash
# round 3: the default bench line with two batches in flight, then smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u bench.py > gpurun_out/r3z_bench.json 2> gpurun_out/r3z_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3z_smoke.log 2>&1
echo "smoke rc=$?"
