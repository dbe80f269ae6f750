# batcher sweep on the GPU box: bash tools/gpu_batcher.sh TAG P:T:W ...
set -o pipefail
mkdir -p gpurun_out
T=${1:-b}
shift
timeout -k 10 400 python -u tools/batcher_gpu.py "$@" > gpurun_out/batcher_$T.jsonl 2> gpurun_out/batcher_$T.err
rc=$?; cat gpurun_out/batcher_$T.jsonl; tail -n 3 gpurun_out/batcher_$T.err; exit $rc
