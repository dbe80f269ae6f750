#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 200 python -u tools/dbg_ids.py > gpurun_out/r3i_dbg.log 2>&1
echo "dbg rc=$?"
AMD_SERIALIZE_KERNEL=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu "tests/test_batcher.py::test_gpu_batcher_over_engine_vs_oracle" > gpurun_out/r3i_test.log 2>&1
echo "test rc=$?"
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_words.py tests/test_gpu_filter.py > gpurun_out/r3i_words.log 2>&1
echo "words rc=$?"
