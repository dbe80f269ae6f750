set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_sweep.sh r2oc base rpl1 r1p4_f256s96 r1p6_f256s96 r1p4_f192s64
