# multi-rank rehearsals on one GPU with the final defaults (8-round graph blocks): bench.py --gpus 2 / 4
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for g in 2 4; do
  DPSVM_FORCE_DEVICE=0 timeout -k 10 400 python3 -u bench.py --gpus $g --steps 2 --warmup 1 --json-out gpurun_out/r4s_spawn$g.json > gpurun_out/r4s_spawn$g.out 2> gpurun_out/r4s_spawn$g.err || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/r4s_spawn$g.json').read().strip().split('\n')[-1]); print('gpus=$g', d['value'], d['n_gpus'], d['config']['parallelism'], d.get('dp_policy'), d.get('exchange'), d.get('converged'), d.get('rounds'), d.get('b'))"
done
