# sharded headline with 4 ranks sharing one GPU after the wide-union change: the exchange is refused at 128 blocks
# (spinning solve workgroups of 4 ranks would crowd out the producers) — check it still converges on the fallback
set -o pipefail
mkdir -p gpurun_out/r5r4
DPSVM_FORCE_DEVICE=0 timeout -k 10 500 python3 -u bench.py --gpus 4 --dp shard --steps 2 --warmup 1 --reference-check off \
  --json-out gpurun_out/r5r4/g4.json > gpurun_out/r5r4/g4.log 2>&1 || { tail -12 gpurun_out/r5r4/g4.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r5r4/g4.json')); print('P=4', d['value'], d['config']['parallelism'], d['ws_exchange'], d['ws_blocks'], d['converged'], d['rounds'], d['b'], d['engine_note'])"
