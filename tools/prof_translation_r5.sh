#!/bin/bash
# Round 5, the walk's address-translation bound:
#  1. the region-grouped random-gather ceiling twice (is G = 2 lanes per 2 MiB region's dip real?)
#  2. UTCL1 / TA counters of those same gather launches (which unit the G = 2 dip sits in)
#  3. k_match_fast's translation counters at edge load 1/16 (default) and 1/4 (a 4x smaller table)
# Usage (GPU box, repo root): bash tools/prof_translation_r5.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/xlat}
export TMPDIR=/tmp
mkdir -p "$OUT"
timeout -k 10 120 tools/gather_roof regions 16 > "$OUT/regions_a.jsonl" &&
timeout -k 10 120 tools/gather_roof regions 16 > "$OUT/regions_b.jsonl" &&
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum \
    TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum --output-format csv -d "$OUT/gr_utc" -o gr_utc -- \
    tools/gather_roof regions 16 > "$OUT/gr_utc.jsonl" 2> "$OUT/gr_utc.err" &&
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum \
    TCP_TCC_READ_REQ_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE --output-format csv -d "$OUT/gr_ta" -o gr_ta -- \
    tools/gather_roof regions 16 > "$OUT/gr_ta.jsonl" 2> "$OUT/gr_ta.err" || exit $?
ARGS="--profile --sequential --steps 4 --warmup 1"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- \
      python -u bench.py $ARGS > "$OUT/$name.bench.json" 2> "$OUT/$name.bench.err"
}
UTC="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
run utc16 --pmc $UTC &&
EMQX_TM_EDGE_LOAD_INV=4 run utc4 --pmc $UTC &&
EMQX_TM_EDGE_LOAD_INV=4 run trace4 --kernel-trace --stats
echo "xlat rc=$?"
