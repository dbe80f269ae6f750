set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_sweep.sh r2cv base cpv cpv8 base2
