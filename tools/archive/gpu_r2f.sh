# round 2: quick bench (batcher stage split, modes) after NT keys + edge load 1/16
set -o pipefail
mkdir -p gpurun_out
T=${1:-r2f}
timeout -k 10 400 python -u bench.py --quick > gpurun_out/bench_${T}.json 2> gpurun_out/bench_${T}.err
rc=$?; head -c 300 gpurun_out/bench_${T}.json; echo; tail -n 3 gpurun_out/bench_${T}.err; exit $rc
