set -o pipefail
mkdir -p gpurun_out
T=${1:-s}
shift
timeout -k 10 600 python -u tools/sweep.py run --variants "$@" > gpurun_out/sweep_$T.jsonl 2> gpurun_out/sweep_$T.err
rc=$?; cat gpurun_out/sweep_$T.jsonl; tail -n 3 gpurun_out/sweep_$T.err; exit $rc
