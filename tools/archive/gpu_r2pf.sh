# round-2 final tree: every topic of the full config C and E batches vs the oracle (ALL, COUNT, FIRST)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/parity_full.py --config C --out gpurun_out/parity_full_C_r2.json > gpurun_out/parity_full_C_r2.log 2>&1 || exit $?
tail -n 3 gpurun_out/parity_full_C_r2.log
timeout -k 10 300 python -u tools/parity_full.py --config E --out gpurun_out/parity_full_E_r2.json > gpurun_out/parity_full_E_r2.log 2>&1 || exit $?
tail -n 3 gpurun_out/parity_full_E_r2.log
