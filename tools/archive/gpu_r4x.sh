# Round-4 GPU pass x: the GPU suite with the replica runs form, then the bench line (with the
# aggregator on a read replica).
set -o pipefail
T=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 420 --timeout-method thread tests -m gpu -x > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$T.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 480 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
rc=$?; head -c 300 gpurun_out/bench_$T.json; echo; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_$T.err; exit $rc; }
python -c "import json; d=json.loads(open('gpurun_out/bench_$T.json').read().strip().splitlines()[-1]); b=d['batcher']; print([(x['transport'][:4], x['callback'][:9], round(x['publishes_per_s']/1e6,1)) for x in b['runs']]); r=b['on_replica']; print('replica', r['replica_load_s'], [(x['transport'][:4], x['callback'][:9], round(x['publishes_per_s']/1e6,1), x['littles_law']['ok']) for x in r['runs']])"
