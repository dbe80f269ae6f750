#!/bin/bash
# round 3: filter walk with window reuse (records kept across in-window seeks): filter tests,
# kernel traces of the 100 K-query batch (mixed, one-'+' kind) and of 9 K one-'+' queries
# (tail test); then host paths and the aggregator unpinned vs pinned to the GPU's socket
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_filter.py tests/test_oracle_filter.py > gpurun_out/r3n_tests.log 2>&1
rc=$?; echo "filter tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in mix 1 1s; do
  args="--filter-search 100000"
  [ "$k" = "1" ] && args="$args --filter-kinds 1"
  [ "$k" = "1s" ] && args="--filter-search 9000 --filter-kinds 1"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3n_prof_$k -o f -- python3 -u bench.py $args > gpurun_out/r3n_bench_$k.json 2> gpurun_out/r3n_bench_$k.err
  rc=$?; echo "kind $k rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
cat /sys/bus/pci/devices/*/numa_node 2>/dev/null | sort | uniq -c > gpurun_out/r3n_numa.txt
timeout -k 10 900 python -u tools/numa_check.py > gpurun_out/r3n_numa.jsonl 2> gpurun_out/r3n_numa.err
echo "numa rc=$?"
