#!/bin/bash
# round 3: large D2H copies by a kernel into pinned memory: host keys path alone, the GPU
# suite, then the default bench line (pinned, with this source's PMC profile in profiles/)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/prof_hostpath.py > gpurun_out/r3r_hostpath.log 2>&1
rc=$?; echo "hostpath rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/r3r_pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/r3r_bench.json 2> gpurun_out/r3r_bench.err
echo "bench rc=$?"
