#!/bin/bash
# Round-5 final pass, part 2: the dominant kernel's kernel trace + PMC passes (tools/prof_pmc.sh)
# summarised for profiles/, then the 2-rank replicated rehearsal over gloo on the one GPU.
set -o pipefail
T=${1:-final}
mkdir -p gpurun_out
bash tools/prof_pmc.sh gpurun_out/prof_$T || exit 1
python tools/summarize_prof.py gpurun_out/prof_$T gpurun_out/r05_prof_$T || exit 1
EMQX_BENCH_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 20 --warmup 5 --batcher-seconds 0 \
    > gpurun_out/r05_bench_gloo2_$T.json 2> gpurun_out/r05_bench_gloo2_$T.err || exit 2
echo "final part 2 done"
