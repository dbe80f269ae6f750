#!/bin/bash
# Round-6 GPU pass (on the GPU box, repo root): the GPU suite, smoke(), the default bench line.
# STEPS picks the steps (default "test smoke bench").  Every GPU step has its own time limit;
# the first failure ends the script.
set -o pipefail
T=${1:-r6}
STEPS=${STEPS:-"test smoke bench"}
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    test)
      EMQX_TM_TEST_MEMLOG=gpurun_out/r06_memlog_$T.txt timeout -k 10 480 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
          > gpurun_out/r06_pytest_gpu_$T.log 2>&1 || { tail -n 30 gpurun_out/r06_pytest_gpu_$T.log; exit 1; }
      tail -n 2 gpurun_out/r06_pytest_gpu_$T.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke_$T.log 2>&1 \
          || { tail -n 20 gpurun_out/r06_smoke_$T.log; exit 2; } ;;
    bench)
      timeout -k 10 700 python -u bench.py > gpurun_out/r06_bench_$T.json 2> gpurun_out/r06_bench_$T.err \
          || { tail -n 20 gpurun_out/r06_bench_$T.err; exit 4; }
      cp gpurun_out/bench_detail.json gpurun_out/r06_bench_detail_$T.json
      wc -c gpurun_out/r06_bench_$T.json ;;
    rebuild)
      PIN=1 timeout -k 10 400 python -u tools/rebuild_probe_r6.py ${REPS:-4} > gpurun_out/r06_rebuild_probe_$T.jsonl \
          2> gpurun_out/r06_rebuild_probe_$T.err || { tail -n 20 gpurun_out/r06_rebuild_probe_$T.err; exit 6; } ;;
    quick)
      timeout -k 10 300 python -u bench.py --quick --batcher-seconds 0 --steps 40 > gpurun_out/r06_quick_$T.json \
          2> gpurun_out/r06_quick_$T.err || { tail -n 20 gpurun_out/r06_quick_$T.err; exit 5; } ;;
  esac
done
echo "r6 pass done: $STEPS"
