# Round-4 GPU pass u: the bench line with the commit trace twice (pass r's churn-leg overflow:
# now logged and re-run, with the last epoch's parity in the line).
set -o pipefail
T=${1:-u}
mkdir -p gpurun_out
for k in 1 2; do
  EMQX_TM_COMMIT_TRACE=1 timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_${T}$k.json 2> gpurun_out/bench_${T}$k.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/bench_${T}$k.json').read().strip().splitlines()[-1]); c=d['churn_E']; print({'value': d['value'], 'reruns': c.get('match_reruns'), 'parity': c['parity'], 'commit_ms_p50': c['commit_ms_p50']})" || exit $?
  grep -i "re-run\|overflow\|PARITY" gpurun_out/bench_${T}$k.err | head -5
done
