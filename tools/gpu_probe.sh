#!/bin/bash
# round 3: whole-batch parity at full size for configs C and E with this round's tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u tools/parity_full.py --config C --out gpurun_out/r3_parity_full_C.json > gpurun_out/r3_parity_C.log 2>&1
rc=$?; echo "C rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/parity_full.py --config E --out gpurun_out/r3_parity_full_E.json > gpurun_out/r3_parity_E.log 2>&1
echo "E rc=$?"
