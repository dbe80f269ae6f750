#!/bin/bash
# k_filter_walk on this round's source: kernel traces of the mixed 100 K-query batch and of the
# one-'+' queries alone (split into parts, EMQX_TM_FILTER_SPLIT=16384:4096, and unsplit), then
# FETCH_SIZE / WRITE_SIZE passes of the mixed batch.  Summary: tools/filter_prof_r5.py OUT.
set -o pipefail
OUT=${1:-gpurun_out/prof_filter_r5}
export TMPDIR=/tmp
mkdir -p "$OUT"
run() {
  local name=$1 q=$2 kinds=$3; shift 3
  timeout -s KILL 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- \
      python -u bench.py --filter-search "$q" $kinds --steps 3 --warmup 1 > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run mixed 100000 "" --kernel-trace --stats &&
EMQX_TM_FILTER_SPLIT=16384:4096 run plus 9000 "--filter-kinds 1" --kernel-trace --stats &&
EMQX_TM_FILTER_SPLIT=0 run plus_nosplit 9000 "--filter-kinds 1" --kernel-trace --stats &&
run fetch 100000 "" --pmc FETCH_SIZE &&
run write 100000 "" --pmc WRITE_SIZE
echo "prof rc=$?"
