# round-2 final tree: instruction mix of k_match_fast (same counters as round 1's r01_inst_mix)
set -o pipefail
bash tools/prof_insts.sh gpurun_out/insts_r2 && ls gpurun_out/insts_r2/mix
