# kernel + memory-copy trace of the batcher at 65,536 publishers (no PMC counters)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_bat -o bat --output-format csv \
    -- python3 tools/batcher_gpu.py 65536:13:200 > gpurun_out/prof_bat.log 2>&1
rc=$?; tail -n 3 gpurun_out/prof_bat.log; find gpurun_out/prof_bat -name "*.csv" | head; exit $rc
