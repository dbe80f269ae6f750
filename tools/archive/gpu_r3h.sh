#!/bin/bash
# round 3: wave-block compaction + rank-chunk merge: shard/batcher tests, D-shard bench + profile,
# and the keys-kernel A/B against the previous source (same process)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_shard.py tests/test_batcher.py tests/test_replica.py tests/test_gpu_words.py tests/test_gpu_concurrency.py > gpurun_out/r3h_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --mode sharded --config D --shard-of 8 --steps 20 --warmup 3 > gpurun_out/r3h_D.json 2> gpurun_out/r3h_D.err
rc=$?; echo "D bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3h_prof -o D -- python3 -u bench.py --mode sharded --config D --shard-of 8 --steps 10 --warmup 2 > gpurun_out/r3h_prof.log 2>&1
echo "prof rc=$?"
timeout -k 10 600 python -u tools/sweep.py run --variants prev base prev base --steps 20 > gpurun_out/r3h_sweep.jsonl 2> gpurun_out/r3h_sweep.err
echo "sweep rc=$?"
