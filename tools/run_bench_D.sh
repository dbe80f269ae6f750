#!/bin/bash
# Config D (100 M route keys) on ONE MI355X: mode 1's per-GPU copy (the whole index on one
# device, publishes data-parallel over replicas).  The generator and the build run for minutes
# without output, so a heartbeat (time + host memory) goes to OUT.hb meanwhile.
# Usage: bash tools/run_bench_D.sh OUT_PREFIX [SCALE] [STEPS]
set -o pipefail
OUT=${1:-gpurun_out/bench_D}
SCALE=${2:-1.0}
STEPS=${3:-20}
mkdir -p "$(dirname "$OUT")"
( while sleep 40; do echo "$(date +%T) $(free -g | awk '/Mem:/ {print "used_gib", $3, "avail_gib", $7}')" >> "$OUT.hb"; done ) &
HB=$!
timeout -k 10 1080 python -u bench.py --config D --scale "$SCALE" --quick --batcher-seconds 0 --steps "$STEPS" --warmup 3 \
    > "$OUT.json" 2> "$OUT.err"
rc=$?
kill $HB 2>/dev/null
echo "bench D rc=$rc"
exit $rc
