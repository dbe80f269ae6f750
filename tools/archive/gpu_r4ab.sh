# Round-4 GPU pass ab (gate of the final kernel source): the PMC passes first (summarised into
# the box's profiles/ so the bench line's roofline carries their traffic), the GPU suite, the
# bench line, smoke.
set -o pipefail
T=${1:-ab}
mkdir -p gpurun_out
bash tools/prof_pmc.sh gpurun_out/prof_$T > gpurun_out/prof_$T.log 2>&1
rc=$?; tail -3 gpurun_out/prof_$T.log; [ $rc -eq 0 ] || exit $rc
python tools/summarize_prof.py gpurun_out/prof_$T profiles/r04_prof_final > gpurun_out/prof_${T}_summary.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -v --timeout 420 --timeout-method thread tests -m gpu -x > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$T.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 480 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; head -c 300 gpurun_out/bench_$T.json; echo; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$T.err; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_$T.log; exit $rc
