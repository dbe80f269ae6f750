# Round-4 GPU pass t: first-batch totals of fresh engines, and a long churn run (30 epochs)
# with the overflow re-run logged.
set -o pipefail
T=${1:-t}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/probe_first_total.py > gpurun_out/first_total_$T.jsonl 2> gpurun_out/first_total_$T.err
rc=$?; cat gpurun_out/first_total_$T.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/first_total_$T.err; exit $rc; }
timeout -k 10 400 python -u bench.py --churn 30 --warmup 1 > gpurun_out/churn30_$T.json 2> gpurun_out/churn30_$T.err
rc=$?; python -c "import json; d=json.loads(open('gpurun_out/churn30_$T.json').read().strip().splitlines()[-1]); print({k: d[k] for k in ('commit_ms_p50','commit_ms_p99','match_reruns','parity','full_rebuild_epochs')})"; grep -i "re-run\|overflow" gpurun_out/churn30_$T.err | head; exit $rc
