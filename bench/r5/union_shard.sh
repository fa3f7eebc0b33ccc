# 6,144-row unions at world > 1: two-process exchange tests, then the sharded headline rehearsed with 2
# ranks sharing one GPU (peer exchange), union 6,144 (default) vs 3,072 (DPSVM_WS_UNION)
set -o pipefail
mkdir -p gpurun_out/r5us
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_ws_gpu.py \
  -k "wide_union or multi_block_peer_exchange_processes or eight_processes" > gpurun_out/r5us/pytest.log 2>&1 \
  || { tail -40 gpurun_out/r5us/pytest.log; exit 1; }
tail -2 gpurun_out/r5us/pytest.log
for u in 6144 3072; do
  DPSVM_WS_UNION=$u DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus 2 --dp shard --steps 3 --warmup 1 \
    --json-out gpurun_out/r5us/g2_$u.json > gpurun_out/r5us/g2_$u.log 2>&1 || { tail -8 gpurun_out/r5us/g2_$u.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r5us/g2_$u.json')); print('P=2 union $u', d['value'], d['config']['parallelism'], d['ws_exchange'], d['ws_blocks'], d['converged'], d['rounds'], d['b'], d['engine_note'])"
done
