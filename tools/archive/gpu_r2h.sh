# round 2: quick bench (batcher stages), matches_filter at 100K queries (bench + kernel trace + FETCH/WRITE)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --quick > gpurun_out/bench_r2h.json 2> gpurun_out/bench_r2h.err || exit $?
head -c 200 gpurun_out/bench_r2h.json; echo
timeout -k 10 400 python -u bench.py --filter-search 100000 > gpurun_out/bench_filter_r2h.json 2> gpurun_out/bench_filter_r2h.err || exit $?
cat gpurun_out/bench_filter_r2h.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_filter_r2h -o prof -- python3 -u bench.py --filter-search 100000 --steps 5 --warmup 1 > gpurun_out/prof_filter_r2h.log 2>&1 || exit $?
bash tools/prof_filter_pmc.sh gpurun_out/prof_filter_pmc_r2h
