#!/bin/bash
# Kernel trace + PMC passes of the bench workload (config C, 1M publishes/step) on one GPU.
# Each counter group is its own rocprofv3 run (rocprofv3 does not split passes).
# Usage (on the GPU box, from the repo root): bash tools/prof_pmc.sh <outdir> [extra bench args]
set -o pipefail
OUT=${1:-gpurun_out/prof}
shift || true
ARGS="--profile --sequential --steps 4 --warmup 1 $*"  # one launch at a time: per-kernel durations and counters
export TMPDIR=/tmp
mkdir -p "$OUT"
# which kernel source these counters belong to (bench.py only reports a matching profile)
sha256sum emqx_amd/csrc/match_kernels.hip emqx_amd/csrc/layout.h emqx_amd/csrc/device_api.h emqx_amd/csrc/wave.h > "$OUT/src.sha"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- \
      python -u bench.py $ARGS > "$OUT/$name.bench.json" 2> "$OUT/$name.bench.err"
}
run trace --kernel-trace --stats &&
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE &&
run tcc --pmc TCC_HIT_sum TCC_MISS_sum &&
run sq --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
echo "prof rc=$?"
