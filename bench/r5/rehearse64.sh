# sharded headline with the coupling-chosen 64 blocks: 2 and 4 ranks sharing one GPU (peer exchange), then smoke
set -o pipefail
mkdir -p gpurun_out
for P in 2 4; do
  DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus $P --dp shard --steps 3 --warmup 1 --json-out gpurun_out/r5h_g$P.json > gpurun_out/r5h_g$P.log 2>&1 || { tail -8 gpurun_out/r5h_g$P.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r5h_g$P.json')); print($P, d['value'], d['config']['parallelism'], d['ws_exchange'], d['ws_blocks'], d['converged'], d['rounds'], d['b'], d['engine_note'])"
done
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
