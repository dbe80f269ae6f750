set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_sweep.sh r2kn base rpl1 cpu4 cpu16 qcopy16 qcopy4 el32
