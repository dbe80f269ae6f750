#!/bin/bash
# round 3: host op costs on the box + batcher knob sweep at config C (65,536 publishers)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
g++ -O2 -std=c++17 tools/cpu_costs.cpp -o /tmp/cpu_costs && /tmp/cpu_costs > gpurun_out/r3e_costs.json
cat /sys/devices/system/clocksource/clocksource0/current_clocksource >> gpurun_out/r3e_costs.json
timeout -k 10 500 python -u tools/batcher_gpu.py 65536:13:200:0:1:4 65536:13:200:0:1:6 65536:13:200:0:1:8 \
  65536:14:200:0:1:4 65536:13:200:0:0:4 65536:13:200:0:0:8 65536:13:200:1:0:4 65536:13:200:1:0:8 \
  65536:13:200:0:1:8:32768 65536:13:200:0:1:4:32768 65536:13:50:0:1:4 262144:13:200:0:1:4 \
  > gpurun_out/r3e_sweep.jsonl 2> gpurun_out/r3e_sweep.err
echo "sweep rc=$?"
