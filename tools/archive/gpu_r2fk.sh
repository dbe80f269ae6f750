# round-2: k_filter_walk time per query kind (0 stored, 1 one '+', 2 prefix + '#'), config C
set -o pipefail
export TMPDIR=/tmp
for k in 0 1 2; do
  O=gpurun_out/prof_fk$k; mkdir -p $O
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o trace -- \
      python3 -u bench.py --filter-search 100000 --filter-kinds $k --steps 2 --warmup 1 > $O/bench.json 2> $O/bench.err || exit $?
  head -c 400 $O/bench.json; echo
done
