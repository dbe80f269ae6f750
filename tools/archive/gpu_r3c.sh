#!/bin/bash
# runs host path: sub-batch / tpw sweep at full config C
set -o pipefail
cd "$GRAFT_REPO_ROOT"
cat > /tmp/sweep_runs.py <<'PY'
import os, subprocess, sys
PY
for cfg in "131072 0" "262144 0" "262144 64" "524288 0" "1048576 0"; do
  set -- $cfg
  EMQX_TM_RUNS_SUB=$1 EMQX_TM_RUNS_TPW=$2 timeout -k 10 300 python -u tools/prof_runs.py --scale 1.0 --reps 8 > gpurun_out/r3c_$1_$2.log 2>&1 || exit 1
  echo "sub $1 tpw $2: $(grep runs: gpurun_out/r3c_$1_$2.log)"
done
