#!/bin/bash
# round 3: '+' child cached beside each slot (32-B slots): GPU suite, then the bench step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/r3u_pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --quick > gpurun_out/r3u_bench_quick.json 2> gpurun_out/r3u_bench_quick.err
echo "bench rc=$?"
