#!/bin/bash
# Instruction-mix PMC pass of the bench workload (k_match_fast): where the issue slots go.
# Usage (GPU box, repo root): bash tools/prof_insts.sh <outdir>
set -o pipefail
OUT=${1:-gpurun_out/insts}
export TMPDIR=/tmp
mkdir -p "$OUT"
rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES \
    --output-format csv -d "$OUT/mix" -o mix -- python -u bench.py --profile --steps 2 --warmup 1 > "$OUT/mix.bench.json" 2> "$OUT/mix.bench.err"
echo "insts rc=$?"
