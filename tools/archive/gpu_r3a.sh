#!/bin/bash
# round 3: new concurrency / runs tests first, then the whole GPU suite and smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_concurrency.py tests/test_batcher.py -m gpu > gpurun_out/r3a_new.log 2>&1
rc=$?
echo "new tests rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/r3a_gpu.log 2>&1
rc=$?
echo "gpu suite rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3a_smoke.log 2>&1
echo "smoke rc=$?"
