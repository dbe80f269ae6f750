#!/bin/bash
# round 3: is the one-'+' filter batch tail-bound? kernel time at 3 K / 10 K / 33 K queries;
# then host paths and the aggregator unpinned vs pinned to the GPU's socket
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for q in 9000 30000; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r3m_prof_$q -o f -- python3 -u bench.py --filter-search $q --filter-kinds 1 > gpurun_out/r3m_bench_$q.json 2> gpurun_out/r3m_bench_$q.err
  rc=$?; echo "q $q rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
cat /sys/bus/pci/devices/*/numa_node 2>/dev/null | sort | uniq -c > gpurun_out/r3m_numa.txt
timeout -k 10 900 python -u tools/numa_check.py > gpurun_out/r3m_numa.jsonl 2> gpurun_out/r3m_numa.err
echo "numa rc=$?"
