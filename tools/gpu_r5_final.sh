#!/bin/bash
# Round-5 final pass, part 1 (on the GPU box, repo root): the GPU suite, smoke(), (with
# INFLIGHT_AB=1) the in-flight A/B, and the default bench line.  Every GPU step has its own time limit; the first
# failure ends the script.
set -o pipefail
T=${1:-final}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/r05_pytest_gpu_$T.log 2>&1 || { tail -n 20 gpurun_out/r05_pytest_gpu_$T.log; exit 1; }
tail -n 2 gpurun_out/r05_pytest_gpu_$T.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_$T.log 2>&1 || exit 2
if [ -n "$INFLIGHT_AB" ]; then  # two vs three batches in flight (measured once: no gain from three)
  for k in 2 3; do
    timeout -k 10 300 python -u bench.py --quick --batcher-seconds 0 --in-flight $k --steps 40 --warmup 5 \
        > gpurun_out/r05_bench_if${k}_$T.json 2> gpurun_out/r05_bench_if${k}_$T.err || exit 3
  done
fi
timeout -k 10 700 python -u bench.py > gpurun_out/r05_bench_$T.json 2> gpurun_out/r05_bench_$T.err || exit 4
echo "final part 1 done"
