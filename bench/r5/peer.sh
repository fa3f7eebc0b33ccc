# push-only ws peer exchange: the exchange tests (2/4/8 processes on one GPU), then
# bench.py --gpus 4 / 8 --dp shard at the headline with every rank on device 0
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ws_gpu.py -k "peer_exchange" > gpurun_out/r5p_pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r5p_pytest.log | tail -25; [ $rc -eq 0 ] || exit $rc
for N in 4 8; do
  DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus $N --dp shard --steps 3 --warmup 1 --json-out gpurun_out/r5p_bench$N.json > gpurun_out/r5p_bench$N.log 2>&1 || { tail -30 gpurun_out/r5p_bench$N.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r5p_bench$N.json')); print($N, d['value'], d['config']['parallelism'], d['ws_exchange'], repr(d['engine_note']), d['rounds'], d['converged'], d['b'], d['ws_blocks'])"
done
