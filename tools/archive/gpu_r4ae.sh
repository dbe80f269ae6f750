# Round-4 GPU pass ae: physically contiguous VRAM for the big device buffers
# (EMQX_TM_DEV_CONTIG=1) against hipMalloc: the random-gather ceiling, the bench line, and the
# latency / translation PMC passes.
set -o pipefail
T=${1:-ae}
mkdir -p gpurun_out
timeout -k 10 180 ./tools/gather_roof default 16 > gpurun_out/gather_default_$T.jsonl 2>&1 || exit $?
timeout -k 10 180 ./tools/gather_roof contig 16 > gpurun_out/gather_contig_$T.jsonl 2>&1 || exit $?
grep -h '"table_MiB": 16384' gpurun_out/gather_default_$T.jsonl gpurun_out/gather_contig_$T.jsonl
timeout -k 10 480 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_default_$T.json 2> gpurun_out/bench_default_$T.err
rc=$?; head -c 200 gpurun_out/bench_default_$T.json; echo; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_default_$T.err; exit $rc; }
EMQX_TM_DEV_CONTIG=1 timeout -k 10 480 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_contig_$T.json 2> gpurun_out/bench_contig_$T.err
rc=$?; head -c 200 gpurun_out/bench_contig_$T.json; echo; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_contig_$T.err; exit $rc; }
EMQX_TM_DEV_CONTIG=1 bash tools/prof_latency.sh gpurun_out/lat_contig_$T > gpurun_out/lat_contig_$T.log 2>&1
rc=$?; tail -2 gpurun_out/lat_contig_$T.log; exit $rc
