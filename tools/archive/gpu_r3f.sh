#!/bin/bash
# round 3: fused ids (walk writes route ids) + shard exchange variants: GPU suite, smoke,
# config-D shard bench (all exchanges), rocprof of the sharded step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_shard.py tests/test_batcher.py > gpurun_out/r3f_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > gpurun_out/r3f_gpu.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3f_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --mode sharded --config D --shard-of 8 --steps 20 --warmup 3 > gpurun_out/r3f_D.json 2> gpurun_out/r3f_D.err
rc=$?; echo "D bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3f_prof -o D -- python3 -u bench.py --mode sharded --config D --shard-of 8 --steps 10 --warmup 2 > gpurun_out/r3f_prof.log 2>&1
echo "prof rc=$?"
timeout -k 10 120 tools/gather_roof > gpurun_out/r3f_gather_roof.jsonl 2>&1
echo "gather rc=$?"
timeout -k 10 300 python -u bench.py --quick --batcher-seconds 0 --steps 20 > gpurun_out/r3f_quick.json 2> gpurun_out/r3f_quick.err
echo "quick bench rc=$?"
