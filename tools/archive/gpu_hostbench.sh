# the batcher's host machinery alone on the GPU box's CPUs (custom backend, fixed 142 ids)
set -o pipefail
mkdir -p gpurun_out
for th in 1 4 8 13; do timeout -k 5 60 tools/batcher_host_bench 65536 142 2 $th; done > gpurun_out/hostbench.jsonl 2>&1
cat gpurun_out/hostbench.jsonl; nproc; cat /sys/fs/cgroup/cpu.max
