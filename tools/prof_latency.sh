#!/bin/bash
# Memory-latency and address-translation PMC passes of the bench workload (config C, 1 M
# publishes, one launch at a time), one rocprofv3 run per counter group (per-block limits:
# <= 4 TCP, <= 4 TCC, <= 2 TA, <= 2 GRBM).  Summarise with tools/summarize_latency.py.
# Usage (on the GPU box, from the repo root): bash tools/prof_latency.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/lat}
ARGS="--profile --sequential --steps 4 --warmup 1"
export TMPDIR=/tmp
mkdir -p "$OUT"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- \
      python -u bench.py $ARGS > "$OUT/$name.bench.json" 2> "$OUT/$name.bench.err"
}
run lat --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCP_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum \
    TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum &&
run tlb --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum \
    TCC_EA0_RDREQ_DRAM_sum TCC_TAG_STALL_sum TCC_LATENCY_FIFO_FULL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum &&
run utc --pmc TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_CLIENT_UTCL1_INFLIGHT_sum \
    TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE
echo "lat rc=$?"
