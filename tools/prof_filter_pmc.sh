#!/bin/bash
# k_filter_walk: kernel trace + FETCH_SIZE / WRITE_SIZE passes of the --filter-search bench.
set -o pipefail
OUT=${1:-gpurun_out/prof_filter_pmc}
export TMPDIR=/tmp
mkdir -p "$OUT"
run() {
  local name=$1; shift
  timeout -s KILL 240 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o "$name" -- \
      python -u bench.py --filter-search 100000 --steps 2 --warmup 0 > "$OUT/$name.json" 2> "$OUT/$name.err"
}
run fetch --pmc FETCH_SIZE &&
run write --pmc WRITE_SIZE
echo "prof rc=$?"
