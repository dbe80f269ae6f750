# Round-4 GPU pass r: the config-C build's commit trace and the bench line with the ids /
# u32-span aggregator row.
set -o pipefail
T=${1:-r}
mkdir -p gpurun_out
EMQX_TM_COMMIT_TRACE=1 timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; grep "tm commit" gpurun_out/bench_$T.err | head -4 | cut -c1-400; head -c 300 gpurun_out/bench_$T.json; echo; exit $rc
