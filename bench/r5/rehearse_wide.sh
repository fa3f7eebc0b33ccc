# sharded headline with 2 and 4 ranks sharing one GPU: 2 ranks take the 6,144-row union over the peer exchange,
# 4 ranks fall back to 3,072 rows (64 blocks) because 128 spinning solve workgroups a rank would not be resident;
# plus the multi-process exchange tests
set -o pipefail
mkdir -p gpurun_out/r5rw
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_ws_gpu.py -k "processes" \
  > gpurun_out/r5rw/pytest.log 2>&1 || { tail -30 gpurun_out/r5rw/pytest.log; exit 1; }
tail -1 gpurun_out/r5rw/pytest.log
for P in 2 4; do
  DPSVM_FORCE_DEVICE=0 timeout -k 10 500 python3 -u bench.py --gpus $P --dp shard --steps 3 --warmup 1 --reference-check off \
    --json-out gpurun_out/r5rw/g$P.json > gpurun_out/r5rw/g$P.log 2>&1 || { tail -12 gpurun_out/r5rw/g$P.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r5rw/g$P.json')); print('P=$P', d['value'], d['config']['parallelism'], d['ws_exchange'], d['ws_blocks'], d['converged'], d['rounds'], d['b'], d['engine_note'])"
done
