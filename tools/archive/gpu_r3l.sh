#!/bin/bash
# round 3: filter walk with prefix-group ends (bounded seeks): filter tests, then kernel
# traces of the 100 K-query batch, mixed and per query kind
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_filter.py tests/test_oracle_filter.py > gpurun_out/r3l_tests.log 2>&1
rc=$?; echo "filter tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in mix 0 1 2; do
  kind=""; [ "$k" != "mix" ] && kind="--filter-kinds $k"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3l_prof_$k -o f -- python3 -u bench.py --filter-search 100000 $kind > gpurun_out/r3l_bench_$k.json 2> gpurun_out/r3l_bench_$k.err
  rc=$?; echo "kind $k rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
