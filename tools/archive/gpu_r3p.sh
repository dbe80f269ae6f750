#!/bin/bash
# round 3: PMC passes of the headline config-C step with this round's kernel source (the
# bench line's roofline.traffic), then the default bench line pinned to the GPU's socket
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/prof_pmc.sh gpurun_out/r3p_prof > gpurun_out/r3p_prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
grep -q "prof rc=0" gpurun_out/r3p_prof.log || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/r3p_bench.json 2> gpurun_out/r3p_bench.err
echo "bench rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r3p_hostpath -o h -- python3 -u tools/prof_hostpath.py > gpurun_out/r3p_hostpath.log 2>&1
echo "hostpath rc=$?"
