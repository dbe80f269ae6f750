# Round-4 GPU pass q: the headline with 8 vs 16 hardware queues, alternating on one box.
set -o pipefail
T=${1:-q}
mkdir -p gpurun_out
: > gpurun_out/hwq_ab_$T.jsonl
for q in 8 16 8 16; do
  EMQX_BENCH_HWQ=$q timeout -k 10 240 python -u bench.py --quick --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/hwq_$q.json 2> gpurun_out/hwq_$q.err || exit $?
  python -c "import json,sys; d=json.loads(open('gpurun_out/hwq_$q.json').read().strip().splitlines()[-1]); print(json.dumps({'hwq': $q, 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'kernel_ms': d['roofline']['kernel_ms'], 'one': (d.get('one_batch_in_flight') or {}).get('ms_per_step')}))" >> gpurun_out/hwq_ab_$T.jsonl || exit $?
done
cat gpurun_out/hwq_ab_$T.jsonl
