set -o pipefail
bash tools/gpu_r2f2.sh ${1:-f} && bash tools/gpu_r2fk.sh
