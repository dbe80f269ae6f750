#!/bin/bash
# round 3: host paths and the aggregator unpinned vs pinned to the GPU's socket
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
cat /sys/bus/pci/devices/*/numa_node 2>/dev/null | sort | uniq -c > gpurun_out/r3k_numa.txt
lscpu | grep -i numa >> gpurun_out/r3k_numa.txt
timeout -k 10 900 python -u tools/numa_check.py > gpurun_out/r3k_numa.jsonl 2> gpurun_out/r3k_numa.err
echo "numa rc=$?"
