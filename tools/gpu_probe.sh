#!/bin/bash
# round 3: FETCH/WRITE of the filter walk with window reuse
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/prof_filter_pmc.sh gpurun_out/r3w_filter_pmc > gpurun_out/r3w.log 2>&1
rc=$?; cat gpurun_out/r3w.log; exit $rc
