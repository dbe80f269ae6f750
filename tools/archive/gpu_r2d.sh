# round-2: config D, one full-size shard of an 8-way filter-hash split (the per-GPU share), and
# the matches_filter profile of the final tree
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py --mode sharded --config D --shard-of 8 --steps 20 --warmup 3 > gpurun_out/bench_D_r2.json 2> gpurun_out/bench_D_r2.err || exit $?
head -c 900 gpurun_out/bench_D_r2.json; echo
bash tools/gpu_r2f3.sh fin
