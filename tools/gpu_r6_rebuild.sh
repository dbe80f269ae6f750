#!/bin/bash
# Round-6 rebuild-stall probe (on the GPU box): repeated forced full rebuilds of config C with
# matches beside them, pinned as bench.py pins; then the ABI/parity smoke of the new build.
set -o pipefail
T=${1:-rb}
mkdir -p gpurun_out
export TMPDIR=/tmp
PIN=1 timeout -k 10 400 python -u tools/rebuild_probe_r6.py ${REPS:-6} > gpurun_out/r06_rebuild_probe_$T.jsonl \
    2> gpurun_out/r06_rebuild_probe_$T.err || { tail -n 20 gpurun_out/r06_rebuild_probe_$T.err; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_$T.log 2>&1 \
    || { tail -n 20 gpurun_out/r06_smoke_$T.log; exit 2; }
echo "rebuild probe done"
