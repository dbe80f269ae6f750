# Round-4 GPU pass w: headline with 2 vs 3 batches in flight, alternating on one box.
set -o pipefail
T=${1:-w}
mkdir -p gpurun_out
: > gpurun_out/inflight_ab_$T.jsonl
for k in 2 3 2 3; do
  timeout -k 10 300 python -u bench.py --quick --steps 50 --warmup 5 --no-cpu-baseline --in-flight $k > gpurun_out/inflight_$k.json 2> gpurun_out/inflight_$k.err || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/inflight_$k.json').read().strip().splitlines()[-1]); print(json.dumps({'in_flight': $k, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'p99_batch_ms': d.get('p99_batch_ms'), 'kernel_ms': d['roofline']['kernel_ms']}))" >> gpurun_out/inflight_ab_$T.jsonl || exit $?
done
cat gpurun_out/inflight_ab_$T.jsonl
