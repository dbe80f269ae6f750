# Round-4 GPU pass i: the B-order probe, the PMC passes of the final kernel source, the default
# bench line and smoke.
set -o pipefail
T=${1:-i}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_runs_order.py > gpurun_out/probe_runs_order_$T.jsonl 2> gpurun_out/probe_runs_order_$T.err
rc=$?; cat gpurun_out/probe_runs_order_$T.jsonl; [ $rc -eq 0 ] || { tail -3 gpurun_out/probe_runs_order_$T.err; exit $rc; }
bash tools/prof_pmc.sh gpurun_out/prof_$T > gpurun_out/prof_$T.log 2>&1
rc=$?; tail -3 gpurun_out/prof_$T.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; head -c 600 gpurun_out/bench_$T.json; echo; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$T.err; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1
rc=$?; tail -3 gpurun_out/smoke_$T.log
exit $rc
