# Round-4 GPU pass aa: same-process A/B of the '+'-edge placement (tools/sweep.py variants,
# alternating), then the bench line, the PMC passes of this kernel source, and smoke.
set -o pipefail
T=${1:-aa}
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/sweep.py run --variants plusnear plushash plusnear2 plushash2 --steps 30 > gpurun_out/sweep_plus_$T.jsonl 2> gpurun_out/sweep_plus_$T.err
rc=$?; cat gpurun_out/sweep_plus_$T.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/sweep_plus_$T.err; exit $rc; }
timeout -k 10 480 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; head -c 300 gpurun_out/bench_$T.json; echo; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$T.err; exit $rc; }
bash tools/prof_pmc.sh gpurun_out/prof_$T > gpurun_out/prof_$T.log 2>&1
rc=$?; tail -3 gpurun_out/prof_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; tail -2 gpurun_out/smoke_$T.log; exit $rc
