set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --churn 15 > gpurun_out/churn_tree2.json 2> gpurun_out/churn_tree2.err || exit $?
cat gpurun_out/churn_tree2.json
